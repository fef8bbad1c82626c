# Round 4: wheel rows -- periodic cold re-centring (every restart_iter iterations) with a larger
# max_iter; MAX_ITER counts, certificate, time per 2,048-env solve; then bitwise check of the
# non-wheel models against the previous commit's library (periodic restarts past max_iter 50
# change nothing there)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
L=operational-space-control_amd/lib
timeout -k 10 200 python tools/ab_bitwise.py $L/ab/base/libosc_batch.so $L/libosc_batch.so > $O/ab_restart_bitwise.txt 2>&1 || exit 22
for sd in 86 91 93; do
  for t in '{}' '{"max_iter": 100}' '{"max_iter": 200}' '{"max_iter": 100, "restart_iter": 14}' '{"max_iter": 200, "restart_iter": 14}' '{"max_iter": 200, "restart_iter": 20}' '{"max_iter": 120, "restart_iter": 20}'; do
    timeout -k 10 120 python tools/wheel_census.py 2048 $sd tumbling bernoulli 1 "$t" --brief >> $O/sweep_$sd.jsonl 2>> $O/sweep.err || exit 11
  done
done
echo done

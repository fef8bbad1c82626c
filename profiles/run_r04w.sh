# Round 4: wheel rows -- with the active-set fallback behind it, a shorter interior-point cap:
# statuses, certificate and time per 2,048-env solve (duals on) for max_iter 20..50
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
for sd in 86 91; do
  for t in '{}' '{"max_iter": 40}' '{"max_iter": 30}' '{"max_iter": 25}' '{"max_iter": 20}'; do
    timeout -k 10 120 python tools/wheel_census.py 2048 $sd tumbling bernoulli 1 "$t" --brief >> $O/sweep_$sd.jsonl 2>> $O/sweep.err || exit 11
  done
done
timeout -k 10 120 python tools/wheel_census.py 2048 81 standing ones 1 '{"max_iter": 30}' --brief >> $O/sweep_81.jsonl 2>> $O/sweep.err || exit 12
timeout -k 10 120 python tools/wheel_census.py 2048 81 standing ones 1 '{}' --brief >> $O/sweep_81.jsonl 2>> $O/sweep.err || exit 12
echo done

# Round 5: wheel refinement steps stop at convergence (y step and the rows' multipliers) instead
# of a fixed twelve -- wheel census + timing against the previous library, bitwise check of the
# models without wheel rows, wheel GPU tests.  (Experiment build, not adopted: DESIGN.md §3.3.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05w
mkdir -p $O
for lib in ab_old/libosc_batch.so libosc_batch.so; do
  for sc in "tumbling bernoulli" "standing ones"; do
    OSC_LIB_PATH=operational-space-control_amd/lib/$lib timeout -k 10 300 python tools/wheel_census.py 2048 91 $sc 1 '{}' --brief >> $O/wheel_ab.jsonl 2>> $O/wheel_ab.err || exit 31
  done
done
for seed in 86 87; do
  for sc in "tumbling bernoulli" "standing ones"; do
    timeout -k 10 300 python tools/wheel_census.py 2048 $seed $sc 4 --brief >> $O/census.jsonl 2>> $O/census.err || exit 32
  done
done
AB_CHECK=1 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_time.py operational-space-control_amd/lib/ab_old/libosc_batch.so operational-space-control_amd/lib/libosc_batch.so > $O/ab_nowheel.jsonl 2>&1 || exit 33
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 34
echo done

# Round 5: the wheel fallback's back substitution stops at the equality rows (their multipliers are
# never read) -- census + time + tau/x hash against the previous library, then the wheel GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/${GI_OUT:-r05gi}
mkdir -p $O
for seed in 91 92; do
for lib in ${AB_BASE:-ab_old}/libosc_batch.so libosc_batch.so; do
  for sc in "tumbling bernoulli" "standing ones"; do
    OSC_LIB_PATH=operational-space-control_amd/lib/$lib timeout -k 10 300 python tools/wheel_census.py 2048 $seed $sc 1 '{}' --brief >> $O/wheel_ab.jsonl 2>> $O/wheel_ab.err || exit 31
  done
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 34
echo done

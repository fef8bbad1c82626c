# Round 5: the dual kernel's contact NNLS in registers (was: runtime-indexed arrays in scratch) --
# per-phase clocks, wheel census time + tau/x hash against the previous library, the GPU tests
# that read duals.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/${DU_OUT:-r05du2}
mkdir -p $O
OSC_LIB_PATH=operational-space-control_amd/lib/duprof/libosc_batch.so timeout -k 10 300 python tools/wheel_census.py 2048 91 tumbling bernoulli 1 '{}' --brief > $O/dual_profile.txt 2> $O/err.txt || exit 30
for seed in 91 92; do
for lib in ${AB_BASE:-ab_old}/libosc_batch.so libosc_batch.so; do
  for sc in "tumbling bernoulli" "standing ones"; do
    OSC_LIB_PATH=operational-space-control_amd/lib/$lib timeout -k 10 300 python tools/wheel_census.py 2048 $seed $sc 1 '{}' --brief >> $O/wheel_ab.jsonl 2>> $O/wheel_ab.err || exit 31
  done
done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_wheels.py tests/test_gpu_joint_states.py tests/test_gpu_full_parity.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 34
echo done

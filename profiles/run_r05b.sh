# Round 5: re-run of the changed GPU tests, then an interleaved A/B of the split build
# (lib/libosc_batch.so) against the pre-split single-unit build (lib/ablate/presplit) and the
# three-waves-per-SIMD large-batch interior point (lib/ablate/w3, -DOSC_LARGE_WAVES=3).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_warm.py tests/test_gpu_wheels.py tests/test_gpu_joint_states.py tests/test_gpu_stages.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -le 1 ] || exit $rc
L=operational-space-control_amd/lib
AB_ROUNDS=5 AB_CHECK=1 AB_CONFIGS=unitree_go2:4096,unitree_go2:8192,unitree_go2:65536,walter_sr:4096 timeout -k 10 400 python tools/ab_time.py $L/libosc_batch.so $L/ablate/presplit/libosc_batch.so $L/ablate/w3/libosc_batch.so > $O/ab.jsonl 2>&1 || exit 31
grep summary $O/ab.jsonl

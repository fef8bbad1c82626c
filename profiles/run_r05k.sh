# Round 5: the warm fix-up pass folded into the warm launch (one-wave path) -- A/B of warm ticks
# against the separate fix-up launch, warm / wheel GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05k
mkdir -p $O
AB_WARM=1 AB_CHECK=1 AB_ROUNDS=5 AB_CONFIGS="unitree_go2:4096,walter_sr:4096,unitree_go2:2048,unitree_go2:65536" timeout -k 10 300 python tools/ab_time.py operational-space-control_amd/lib/ab_old/libosc_batch.so operational-space-control_amd/lib/libosc_batch.so > $O/ab_warm_fixup_fold.jsonl 2>&1 || exit 31
timeout -k 10 600 python -u -m pytest tests/test_gpu_warm.py tests/test_gpu_wheels.py tests/test_gpu_joint_states.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 32
echo done

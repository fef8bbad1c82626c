# Round 5: M-not-SPD flagged NUMERICAL in the assembly + warm fix-up folded into the warm launch:
# cold and warm A/B against the previous commit's library (bitwise flags), then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05m
mkdir -p $O
L0=operational-space-control_amd/lib/ab_old/libosc_batch.so
L1=operational-space-control_amd/lib/libosc_batch.so
AB_CHECK=1 AB_ROUNDS=3 AB_CONFIGS="unitree_go2:4096,walter_sr:4096,unitree_go2:65536" timeout -k 10 300 python tools/ab_time.py $L0 $L1 > $O/ab_cold.jsonl 2>&1 || exit 31
AB_WARM=1 AB_CHECK=1 AB_ROUNDS=5 AB_CONFIGS="unitree_go2:4096,walter_sr:4096,unitree_go2:65536" timeout -k 10 300 python tools/ab_time.py $L0 $L1 > $O/ab_warm.jsonl 2>&1 || exit 32
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 33
echo done

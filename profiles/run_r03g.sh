# Round-3: wheel-row status census on the duals test's batch (seed 86) and the sweep batch (91).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/wheel_sweep.py 2048 16 86 > $O/sweep86.jsonl 2> $O/sweep86.err &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_wheels.py -m gpu -q -k "kkt" --timeout 300 --timeout-method thread > $O/kkt.log 2>&1
echo "rc=$?" >> $O/kkt.log

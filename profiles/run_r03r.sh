# Round-3: wheel rows (rotated Newton systems, stall exit, converged refinement) -- wheel tests,
# census on seeds 86 and 91, whole GPU suite.  Outputs under gpurun_out/r03r.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v --durations=0 --timeout 300 --timeout-method thread > $O/wheels.log 2>&1
echo "wheels rc=$?" >> $O/wheels.log
SWEEP_EPS=1e-10 timeout -k 10 300 python -u tools/wheel_sweep.py 2048 32 91 > $O/sweep91.jsonl 2> $O/sweep91.err
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_wheels.py > $O/gpu_tests.log 2>&1
echo "suite rc=$?" >> $O/gpu_tests.log
echo done

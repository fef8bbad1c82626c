# Round-3: wheel rows with the slack-based refinement active set -- wheel / duals GPU tests,
# refinement diagnostics, sweep, whole GPU suite.  Outputs under gpurun_out/r03f.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v --durations=0 --timeout 300 --timeout-method thread > $O/wheels.log 2>&1
echo "wheels rc=$?" >> $O/wheels.log
timeout -k 10 300 python -u tools/wheel_sweep.py 2048 16 > $O/wheel_sweep.jsonl 2> $O/wheel_sweep.err
echo "sweep rc=$?" >> $O/wheel_sweep.err
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_wheels.py > $O/gpu_tests.log 2>&1
echo "suite rc=$?" >> $O/gpu_tests.log
echo done

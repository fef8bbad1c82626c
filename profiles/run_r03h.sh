# Round-3: wheel rows in rotated coordinates -- wheel / duals GPU tests, status census on the
# duals test's batch, whole GPU suite.  Outputs under gpurun_out/r03h.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v --durations=0 --timeout 300 --timeout-method thread > $O/wheels.log 2>&1
echo "wheels rc=$?" >> $O/wheels.log
timeout -k 10 300 python -u tools/wheel_sweep.py 2048 16 86 > $O/sweep86.jsonl 2> $O/sweep86.err
echo "sweep rc=$?" >> $O/sweep86.err
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_wheels.py > $O/gpu_tests.log 2>&1
echo "suite rc=$?" >> $O/gpu_tests.log
echo done

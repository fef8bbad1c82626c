# Round-3 wheel rows + duals check: the new GPU tests first (verbose, per-test timing), then the
# whole GPU suite.  Outputs under gpurun_out/r03b.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v --durations=0 --timeout 300 --timeout-method thread > $O/wheels.log 2>&1
echo "wheels rc=$?" >> $O/wheels.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_wheels.py > $O/gpu_tests.log 2>&1 || exit 11
echo done

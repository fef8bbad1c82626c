# Round-3: wheel rows, rotated Newton systems, IPM stop 1e-9 + converged refinement -- census on the
# duals test's batch, the wheel GPU tests.  Outputs under gpurun_out/r03o.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
SWEEP_EPS=1e-8,1e-10 timeout -k 10 400 python -u tools/wheel_sweep.py 2048 16 86 > $O/sweep86.jsonl 2> $O/sweep86.err
echo "sweep rc=$?" >> $O/sweep86.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v --durations=0 --timeout 300 --timeout-method thread > $O/wheels.log 2>&1
echo "wheels rc=$?" >> $O/wheels.log

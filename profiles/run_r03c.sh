# Round-3: wheel-row interior point settings sweep, then the wheel / duals GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/wheel_sweep.py 512 16 > $O/wheel_sweep.jsonl 2> $O/wheel_sweep.err
echo "sweep rc=$?" >> $O/wheel_sweep.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v --durations=0 --timeout 300 --timeout-method thread > $O/wheels.log 2>&1
echo "wheels rc=$?" >> $O/wheels.log
echo done

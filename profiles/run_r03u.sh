# Round-3: GPU kinematics tests after slide / ball joints and multi-joint bodies (MJCF chains),
# then the Go2 traces + HBM PMC passes (profiles/run_r03t_prof.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kinematics.py -x -v --timeout 120 --timeout-method thread > $O/kin_tests.log 2>&1 || exit 11
bash profiles/run_r03t_prof.sh > $O/prof.out 2>&1 || exit 12
echo done

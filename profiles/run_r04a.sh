# Round 4: the KKT-accepted refinement -- joint-state tests, then the whole GPU suite (no -x: every
# failure listed), the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_joint_states.py -v --timeout 200 --timeout-method thread > $O/joint_tests.log 2>&1
echo "joint rc $?"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread --deselect tests/test_gpu_joint_states.py > $O/gpu_tests.log 2>&1
echo "suite rc $?"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 11
echo done

# Round-3: wheel-row refinement diagnostics (0/2/5/10 refinement steps, standing + tumbling).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/wheel_diag.py $O/standing81.npz standing 81 > $O/diag.log 2>&1 &&
timeout -k 10 300 python -u tools/wheel_diag.py $O/tumbling82.npz tumbling 82 >> $O/diag.log 2>&1
echo "rc=$?" >> $O/diag.log

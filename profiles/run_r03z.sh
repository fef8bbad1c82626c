# Round-3 re-entry: per-env iteration counts at 65,536 (compaction study), GPU suite at the head.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 300 python -u tools/dump_iters.py $O/iters.npz > $O/iters.txt 2>&1 || exit 10
echo done

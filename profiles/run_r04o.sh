# Round 4: triangular solves with masked coefficients formed one step ahead (A/B time + bitwise
# against the previous commit's library), then the large-batch counters A/B and the wheel sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
L=operational-space-control_amd/lib
timeout -k 10 300 python tools/ab_time.py $L/ab/base/libosc_batch.so $L/libosc_batch.so $L/ab/base/libosc_batch.so $L/libosc_batch.so > $O/ab_solve_masked.jsonl 2>&1 || exit 21
timeout -k 10 200 python tools/ab_bitwise.py $L/ab/base/libosc_batch.so $L/libosc_batch.so > $O/ab_solve_masked_bitwise.txt 2>&1 || exit 22
echo ab
bash profiles/run_r04n.sh

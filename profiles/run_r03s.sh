# Round-3 checks at the wheel-row head (via gpurun): GPU suite, default bench line (north-star and
# mixed objects included), 2-rank gloo rehearsal.  Outputs under gpurun_out/r03s.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 11
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 12
bash tools/rehearse_ranks.sh > $O/rehearse.out 2>&1 || exit 13
echo done

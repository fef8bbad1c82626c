# Round-3: warm-start delta / centring 1.0 -- the GPU suite, smoke and the default bench line
# (warm, front-end warm tick, single-env tick objects).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zo
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 9
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 10
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 11
echo done

# Round-3 final head: smoke(), the whole GPU suite, the default bench line, rocprof kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zs
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 9
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 10
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 11
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 12
echo done

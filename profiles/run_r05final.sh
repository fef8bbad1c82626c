# Round 5 final check at the last commit: GPU suite, smoke, the driver-sized bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 31
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 32
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_20x5.json 2> $O/bench_20x5.err || exit 33
echo done

# Round 4: KKT-accepted refinement (stale multipliers of leaving rows fixed), early interior-point
# stops (Go2 1e-6, WaLTER 1e-8), warm fix-up redoing UNREFINED envs, wheel-row warm start -- the
# feature-off fingerprints regenerated, the whole GPU suite, the default bench line, kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 200 python tests/golden/make_feature_off_hashes.py > $O/feature_off_hashes.json 2> $O/hashes.err || exit 8
cp $O/feature_off_hashes.json tests/golden/feature_off_hashes.json
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "suite rc $?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 10
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 11
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 12
echo done

# Round 5: feature-off fingerprints regenerated for the refinement's one-change rounds (an
# intentional numerical change of the default kernels), then the GPU suite, smoke, and the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 200 python tests/golden/make_feature_off_hashes.py > $O/feature_off_hashes.json 2> $O/hashes.err || exit 31
cp $O/feature_off_hashes.json tests/golden/feature_off_hashes.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 32
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 33
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20x5.json 2> $O/bench_20x5.err || exit 34
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 35
echo done

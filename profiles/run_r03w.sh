# Round-3: pre-scaled LDL factor, multiply-free triangular solves (A/B: profiles/r03_ab_ldl_*.txt).
#   LDL harness (tools/mb_ldlcheck.hip), the GPU suite on the new in-tree build (the feature-off fingerprint test deselected:
#   an intentional numerical change, fingerprints regenerated), default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 60 ./tools/bin/mb_ldlcheck > $O/ldlcheck.txt 2>&1 || exit 11
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_wheels.py::test_feature_off_bitwise_unchanged > $O/gpu_tests.log 2>&1 || exit 13
timeout -k 10 120 python tests/golden/make_feature_off_hashes.py > $O/feature_off_hashes.json 2> $O/hashes.err || exit 14
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 15
echo done

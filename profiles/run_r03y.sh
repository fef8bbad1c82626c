# Round-3: wheel refinement acceptance against the env-wide |y| scale, on top of the pre-scaled
# LDL factor.  Diagnostic of the vanishing-row case (OSC_REFINE_DIAG build), wheel census on
# seeds 86 / 91, LDL harness, LDL layout microbenchmark (tools/mb_layout.hip), the whole GPU suite (feature-off fingerprints deselected: the
# prescale is an intentional numerical change; regenerated here), default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
OSC_LIB_PATH=operational-space-control_amd/lib/ablate/rdiag/libosc_batch.so DIAG_ONE=1 timeout -k 10 200 python tools/wheel_vanish_diag.py 512 > $O/vanish_diag.txt 2>&1 || exit 10
timeout -k 10 60 ./tools/bin/mb_ldlcheck > $O/ldlcheck.txt 2>&1 || exit 11
timeout -k 10 120 ./tools/bin/mb_layout > $O/mb_layout.txt 2>&1 || exit 17
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_wheels.py::test_feature_off_bitwise_unchanged > $O/gpu_tests.log 2>&1 || exit 12
timeout -k 10 120 python tests/golden/make_feature_off_hashes.py > $O/feature_off_hashes.json 2> $O/hashes.err || exit 13
timeout -k 10 300 python -u tools/wheel_sweep.py 2048 32 91 > $O/sweep91.jsonl 2> $O/sweep91.err || exit 14
timeout -k 10 300 python -u tools/wheel_sweep.py 2048 32 86 > $O/sweep86.jsonl 2> $O/sweep86.err || exit 15
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 16
echo done

# Round 5 first GPU pass: every GPU test (incl. the every-env oracle tests), the default bench
# line at the driver's window, and the HBM-input roofline passes.  A test FAILURE (exit 1) does
# not stop the later steps; anything else (timeout, abort, fault) does.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 30
echo "bench done"
bash profiles/run_r05_hbm.sh || exit $?

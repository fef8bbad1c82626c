# Round 5: after the wheel-row fallback moved behind every entry point (raw rows in the
# workspace) and wheel jobs joined osc_batch_solve_multi (ABI 4): the whole GPU suite, smoke(),
# and the seeded-certificate diagnostic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 32
timeout -k 10 120 python tools/seeded_diag.py unitree_go2 256 > $O/diag.log 2>&1 || exit 33
timeout -k 10 120 python tools/seeded_diag.py walter_sr 256 >> $O/diag.log 2>&1 || exit 34
echo done

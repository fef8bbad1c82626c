# Round 5: full GPU suite on the current build (two-kernel joint-state tick, lean assembly past
# one round of IPM waves), smoke, the non-OK env of the 65,536 joint-state batch (seed 11), and a
# status census of further 65,536-env joint-state batches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 32
for s in 11 12 13 14; do
  for jr in 0.5 1.0; do
    timeout -k 10 120 python tools/status_diag.py unitree_go2 65536 $s $jr >> $O/status.jsonl 2>> $O/status.err || exit 33
    timeout -k 10 120 python tools/status_diag.py walter_sr 65536 $s $jr >> $O/status.jsonl 2>> $O/status.err || exit 34
  done
done
echo done

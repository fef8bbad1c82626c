# Round 5: the refinement's one-change active-set rounds -- the UNREFINED fixture envs, a status
# census of 65,536-env joint-state batches, A/B timing against the all-at-once rounds, GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 100 python tools/unrefined_diag.py > $O/unref_new.jsonl 2>&1 || exit 31
for s in 11 12 13 14 15 16; do
  for jr in 0.5 1.0; do
    timeout -k 10 120 python tools/status_diag.py unitree_go2 65536 $s $jr >> $O/status.jsonl 2>> $O/status.err || exit 33
    timeout -k 10 120 python tools/status_diag.py walter_sr 65536 $s $jr >> $O/status.jsonl 2>> $O/status.err || exit 34
  done
done
AB_CHECK=1 timeout -k 10 300 python tools/ab_time.py operational-space-control_amd/lib/ab_old/libosc_batch.so operational-space-control_amd/lib/libosc_batch.so > $O/ab_refine_one_change.jsonl 2>&1 || exit 35
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
exit $rc

# Round 5: a wider status census at the closing build -- 65,536-env joint-state batches at joint
# ranges 0.5 / 1.0 / 1.5, seeds 21-28, Go2 and WaLTER (tools/status_diag.py: counts per status).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05census2
mkdir -p $O
for s in 21 22 23 24 25 26 27 28; do
  for jr in 0.5 1.0 1.5; do
    timeout -k 10 120 python tools/status_diag.py unitree_go2 65536 $s $jr >> $O/status.jsonl 2>> $O/status.err || exit 33
    timeout -k 10 120 python tools/status_diag.py walter_sr 65536 $s $jr >> $O/status.jsonl 2>> $O/status.err || exit 34
  done
done
echo done

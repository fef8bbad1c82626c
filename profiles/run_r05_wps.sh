# Round 5: assembly kernel at three waves per SIMD (launch bound; 168 VGPRs + spills) vs two.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05wps
mkdir -p $O
L=operational-space-control_amd/lib
AB_CHECK=1 AB_ROUNDS=3 AB_CONFIGS="unitree_go2:4096,walter_sr:4096" timeout -k 10 300 python tools/ab_time.py $L/libosc_batch.so $L/wps3/libosc_batch.so > $O/ab.jsonl 2> $O/ab.err || exit 31
echo done

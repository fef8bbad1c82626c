# Round 5: per-phase clocks of the assembly kernel (OSC_STAMPS build) for Go2 / WaLTER 4,096.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05ss
mkdir -p $O
OSC_STAMPS_LIB=operational-space-control_amd/lib/stamps/libosc_batch.so timeout -k 10 200 python tools/setup_stamps.py 4096 unitree_go2 walter_sr > $O/setup_stamps.jsonl 2> $O/setup_stamps.err || exit 30
echo done

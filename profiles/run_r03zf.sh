# Round-3 head: setup-kernel and IPM phase stamps (OSC_STAMPS build) at Go2 4,096 and 256 envs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zf
mkdir -p $O
S=operational-space-control_amd/lib/ablate/stamps/libosc_batch.so
OSC_STAMPS_LIB=$S timeout -k 10 200 python tools/setup_stamps.py 4096 > $O/setup_stamps_4096.jsonl 2>&1 || exit 10
OSC_STAMPS_LIB=$S timeout -k 10 200 python tools/setup_stamps.py 256 > $O/setup_stamps_256.jsonl 2>&1 || exit 11
OSC_STAMPS_LIB=$S timeout -k 10 200 python tools/stamps.py 4096 > $O/ipm_stamps_4096.json 2>&1 || exit 12
echo done

# Round 4: per-phase clocks of the wheel-row interior point (OSC_STAMPS build), 2,048 envs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04zb
mkdir -p $O
OSC_STAMPS_LIB=operational-space-control_amd/lib/ab/stamps/libosc_batch.so timeout -k 10 200 python tools/stamps.py 2048 noslip walter_sr > $O/stamps_wheels_2048.jsonl 2>&1 || exit 11
echo done

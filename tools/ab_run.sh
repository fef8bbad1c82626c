# A/B on the GPU box of libosc_batch.so variants built by tools/ab_build.sh:
#   bash tools/ab_run.sh tag v1 v2 [v3 ...]   -> gpurun_out/ab_<tag>.txt (times twice, then bitwise)
set -o pipefail
A=operational-space-control_amd/lib/ablate
T=$1; shift
L=""; for v in "$@"; do L="$L $A/$v/libosc_batch.so"; done
timeout -k 10 300 python tools/ab_time.py $L $L > gpurun_out/ab_$T.txt 2>&1 || exit 3
timeout -k 10 300 python tools/ab_bitwise.py $L >> gpurun_out/ab_$T.txt 2>&1 || exit 4
grep -v amdgpu.ids gpurun_out/ab_$T.txt

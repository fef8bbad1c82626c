# GPU box: tests with the in-tree build, then A/B of the MFMA vs VALU setup products + stamps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
A=operational-space-control_amd/lib/ablate
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 10
bash tools/ab_run.sh setup m1 m3 valu || exit 11
OSC_STAMPS_LIB=$A/st_m1/libosc_batch.so timeout -k 10 120 python tools/setup_stamps.py 4096 > gpurun_out/sst_m1.txt 2>&1 || exit 12

echo ok

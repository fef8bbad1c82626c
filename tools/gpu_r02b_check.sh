set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 10
OSC_STAMPS_LIB=operational-space-control_amd/lib/ablate/st0/libosc_batch.so timeout -k 10 200 python tools/stamps.py 4096 > gpurun_out/stamps0.json 2>&1 || exit 11
echo ok

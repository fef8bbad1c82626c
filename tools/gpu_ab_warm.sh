# GPU box: GPU tests, then the bench's warm numbers for two builds (A/B of the warm path)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
A=operational-space-control_amd/lib/ablate
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 10
for v in "$@"; do
  for n in 4096 65536; do
    OSC_LIB_PATH=$A/$v/libosc_batch.so timeout -k 10 200 python bench.py --nenv-per-gpu $n --steps 10 --no-cpu --no-single-env --no-front-end > gpurun_out/bw_${v}_${n}.json 2>> gpurun_out/bw.err || exit 11
  done
  OSC_LIB_PATH=$A/$v/libosc_batch.so timeout -k 10 200 python bench.py --robot walter_sr --no-cpu --no-single-env --no-front-end > gpurun_out/bw_${v}_walter.json 2>> gpurun_out/bw.err || exit 12
done
echo ok

# GPU box: GPU tests with the in-tree build (unless SKIP_TESTS=1), then A/B timing + bitwise of
# the ablate variants named on the command line:  bash tools/gpu_ab.sh tag v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 10
fi
bash tools/ab_run.sh "$@" || exit 11
echo ok

# Round-3: wheel rows -- envs left at max_iter are refined (kept refinement = KKT point -> OK):
# status changes against the previous head and the newly-OK envs against the exact oracle;
# phase stamps of the setup / IPM kernels; the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zg
mkdir -p $O
A=operational-space-control_amd/lib
for s in 91 86; do
  timeout -k 10 300 python tools/wheel_status_diff.py $A/ablate/r03head/libosc_batch.so $A/libosc_batch.so 2048 $s > $O/wheel_diff_$s.json 2> $O/wheel_diff_$s.err || exit 10
done
S=$A/ablate/stamps/libosc_batch.so
OSC_STAMPS_LIB=$S timeout -k 10 200 python tools/setup_stamps.py 4096 > $O/setup_stamps_4096.jsonl 2>&1 || exit 11
OSC_STAMPS_LIB=$S timeout -k 10 200 python tools/stamps.py 4096 > $O/ipm_stamps_4096.json 2>&1 || exit 12
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 13
echo done

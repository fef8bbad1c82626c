# Round-3: wheel rows -- refinement rounds continue per env until its steps converge; status changes
# against the previous head (newly-OK envs against the exact oracle), wheel census, GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zh
mkdir -p $O
A=operational-space-control_amd/lib
for s in 91 86 93; do
  timeout -k 10 300 python tools/wheel_status_diff.py $A/ablate/r03head/libosc_batch.so $A/libosc_batch.so 2048 $s > $O/wheel_diff_$s.json 2> $O/wheel_diff_$s.err || exit 10
done
timeout -k 10 300 python -u tools/wheel_sweep.py 2048 32 91 > $O/sweep91.jsonl 2> $O/sweep91.err || exit 14
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 13
echo done

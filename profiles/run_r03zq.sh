# Round-3: why ~0.3 % of joint-state Go2 QPs end OSC_SOLVE_UNREFINED (refinement-diag build) and
# the warm joint-state loop once the fix-up pass leaves those envs alone.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zq
mkdir -p $O
OSC_LIB_PATH=operational-space-control_amd/lib/ablate/rdiag/libosc_batch.so timeout -k 10 200 python tools/qpos_refine_diag.py 4096 > $O/diag.jsonl 2>&1 || exit 10
timeout -k 10 200 python tools/warm_qpos_status.py 4096 12 > $O/warm_qpos.jsonl 2>&1 || exit 11
timeout -k 10 300 python bench.py --no-cpu --no-single-env --no-north-star --no-mixed > $O/bench.json 2> $O/bench.err || exit 12
echo done

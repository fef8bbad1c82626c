# Round-3: refinement run to convergence accepted past the 1e-3 move bound (non-wheel models):
# the joint-state Go2 envs it used to reject against the oracle, the GPU suite, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zr
mkdir -p $O
E=0,42,124,158,286,610,669,893,902,1046,2064,2103
timeout -k 10 200 python tools/qpos_refine_diag.py 4096 $E > $O/diag.jsonl 2>&1 || exit 10
OSC_LIB_PATH=operational-space-control_amd/lib/ablate/rdiag/libosc_batch.so timeout -k 10 200 python tools/qpos_refine_diag.py 4096 > $O/diag_codes.jsonl 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --no-single-env --no-north-star --no-mixed > $O/bench.json 2> $O/bench.err || exit 12
echo done

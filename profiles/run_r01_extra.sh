# Round-1 auxiliary bench lines (via gpurun, after run_r01.sh): larger WaLTER batch, mixed robots,
# per-step contact-mask redraw.  Outputs under gpurun_out/prof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 300 python bench.py --robot walter_sr --nenv-per-gpu 32768 --steps 10 --no-cpu > $O/bench_walter_32768.json 2>> $O/bench.err || exit 21
timeout -k 10 300 python bench.py --robot mixed --no-cpu > $O/bench_mixed_4096x2.json 2>> $O/bench.err || exit 22
timeout -k 10 300 python bench.py --robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192 --no-cpu > $O/bench_walter_tumbling_8192_redraw.json 2>> $O/bench.err || exit 23
echo done

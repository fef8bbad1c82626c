# Round-2 (final head) bench lines for BASELINE configs[1]-[4] and Go2 65,536 on the GPU box (via
# gpurun); outputs under gpurun_out/r02b, copied into profiles/r02b_bench_*.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r02b
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu --no-single-env"
timeout -k 10 300 python bench.py > $O/bench_go2_4096.json 2> $O/bench.err || exit 11
timeout -k 10 200 python bench.py --robot walter_sr $B > $O/bench_walter_4096.json 2>> $O/bench.err || exit 12
timeout -k 10 200 python bench.py --nenv-per-gpu 65536 --steps 10 $B > $O/bench_go2_65536.json 2>> $O/bench.err || exit 13
timeout -k 10 300 python bench.py --robot mixed $B > $O/bench_mixed_4096x2.json 2>> $O/bench.err || exit 14
timeout -k 10 300 python bench.py --robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192 $B > $O/bench_walter_tumbling_8192.json 2>> $O/bench.err || exit 15
echo done

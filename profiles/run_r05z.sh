# Round 5 closing measurement, part 1: GPU suite, smoke, the driver-sized bench under a kernel
# trace, the default bench, and the other BASELINE configs as bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/${CLOSE_OUT:-r05z}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 31
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 32
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/trace20x5 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $O/bench_20x5.json 2> $O/bench_20x5.err || exit 33
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 34
B="--no-cpu --no-front-end --no-single-env --no-north-star --no-mixed --hbm-batches 0"
timeout -k 10 300 python bench.py --robot walter_sr $B > $O/bench_walter_4096.json 2>> $O/other.err || exit 35
timeout -k 10 300 python bench.py --robot walter_sr --nenv-per-gpu 8192 --scenario tumbling --mask bernoulli --mask-redraw 8 $B > $O/bench_walter_tumbling_8192.json 2>> $O/other.err || exit 36
timeout -k 10 300 python bench.py --nenv-per-gpu 8192 $B > $O/bench_go2_8192.json 2>> $O/other.err || exit 37
timeout -k 10 300 python bench.py --nenv-per-gpu 65536 --steps 50 --warmup 20 $B > $O/bench_go2_65536.json 2>> $O/other.err || exit 38
timeout -k 10 300 python bench.py --robot mixed $B > $O/bench_mixed.json 2>> $O/other.err || exit 39
echo done

# Round-2 measurement run on the GPU box (via gpurun): GPU tests, bench lines, rocprofv3 kernel
# trace.  Outputs under gpurun_out/r02; summaries are copied into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r02
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 10
fi
timeout -k 10 300 python bench.py > $O/bench_go2_4096.json 2> $O/bench.err || exit 11
timeout -k 10 200 python bench.py --robot walter_sr --no-cpu --no-single-env > $O/bench_walter_4096.json 2>> $O/bench.err || exit 12
timeout -k 10 200 python bench.py --nenv-per-gpu 65536 --steps 10 --no-cpu --no-single-env > $O/bench_go2_65536.json 2>> $O/bench.err || exit 13
timeout -k 10 300 python bench.py --robot mixed --no-cpu --no-single-env > $O/bench_mixed_4096x2.json 2>> $O/bench.err || exit 14
timeout -k 10 300 python bench.py --robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192 --no-cpu --no-single-env > $O/bench_walter_tumbling_8192.json 2>> $O/bench.err || exit 15
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 --no-cpu --no-warm --no-front-end --no-single-env > $O/trace_stdout.txt 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace65k -o run --output-format csv -- python3 bench.py --nenv-per-gpu 65536 --steps 10 --no-cpu --no-warm --no-front-end --no-single-env > $O/trace65k_stdout.txt 2>&1 || exit 17
echo done

# Round-2 end-of-session measurement on the GPU box (via gpurun): GPU tests, smoke, the default
# bench line (configs[1] with CPU baseline, warm, front end, single-env tick), configs[2]-[4] and
# Go2 65,536, rocprofv3 kernel traces.  Outputs under gpurun_out/r02f.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r02f
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu --no-single-env"
T="--no-cpu --no-warm --no-front-end --no-single-env"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 300 python bench.py > $O/bench_go2_4096.json 2> $O/bench.err || exit 12
timeout -k 10 200 python bench.py --robot walter_sr $B > $O/bench_walter_4096.json 2>> $O/bench.err || exit 13
timeout -k 10 200 python bench.py --nenv-per-gpu 65536 --steps 10 $B > $O/bench_go2_65536.json 2>> $O/bench.err || exit 14
timeout -k 10 300 python bench.py --robot mixed $B > $O/bench_mixed_4096x2.json 2>> $O/bench.err || exit 15
timeout -k 10 300 python bench.py --robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192 $B > $O/bench_walter_tumbling_8192.json 2>> $O/bench.err || exit 16
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 $T > $O/trace_stdout.txt 2>&1 || exit 17
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace65k -o run --output-format csv -- python3 bench.py --nenv-per-gpu 65536 --steps 10 $T > $O/trace65k_stdout.txt 2>&1 || exit 18
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_walter -o run --output-format csv -- python3 bench.py --robot walter_sr --steps 20 $T > $O/trace_walter_stdout.txt 2>&1 || exit 19
echo done

# Round 4 head: the whole GPU suite, smoke, the default bench line and its kernel stats, and the
# other BASELINE configs (WaLTER 4,096; WaLTER tumbling 8,192 with masks redrawn; Go2 8,192 and
# 65,536 with warm; mixed robots)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "suite rc $?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 10
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 11
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 12
echo head
timeout -k 10 200 python bench.py --robot walter_sr --nenv-per-gpu 4096 --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed > $O/bench_walter_4096.json 2>> $O/err.txt || exit 13
timeout -k 10 200 python bench.py --robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192 --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed > $O/bench_walter_tumbling_8192.json 2>> $O/err.txt || exit 14
timeout -k 10 200 python bench.py --nenv-per-gpu 8192 $B > $O/bench_go2_8192.json 2>> $O/err.txt || exit 15
timeout -k 10 200 python bench.py --nenv-per-gpu 65536 --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed > $O/bench_go2_65536.json 2>> $O/err.txt || exit 16
timeout -k 10 200 python bench.py --robot mixed --no-cpu --no-warm --no-front-end --no-single-env --no-north-star > $O/bench_mixed.json 2>> $O/err.txt || exit 17
timeout -k 10 200 python tools/wheel_census.py 2048 93 tumbling bernoulli 1 {} --dump=$O/dump_93.npz > $O/dump_93.jsonl 2>&1 || exit 18
timeout -k 10 300 python tools/wheel_census.py 2048 97 tumbling bernoulli 5 {} --dump=$O/dump_97.npz > $O/dump_97.jsonl 2>&1 || exit 19
OSC_LIB_PATH=operational-space-control_amd/lib/ab/giprof/libosc_batch.so timeout -k 10 200 python tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/giprof_86.txt 2>&1 || exit 20
echo done

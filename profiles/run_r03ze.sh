# Round-3 head: WaLTER configs[3] (tumbling, 8,192 envs, masks redrawn) and WaLTER 32,768 standing
# with the lockstep compaction on (default) and off (OSC_PARK_IT=0), bench lines + rocprof kernel
# traces + FETCH / WRITE passes of the compaction build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03ze
mkdir -p $O
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
W="--robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192"
timeout -k 10 300 python bench.py $W $B > $O/bench_walter_tumbling_8192.json 2> $O/bench.err || exit 10
OSC_PARK_IT=0 timeout -k 10 300 python bench.py $W $B > $O/bench_walter_tumbling_8192_off.json 2>> $O/bench.err || exit 11
timeout -k 10 300 python bench.py --robot walter_sr --nenv-per-gpu 32768 $B > $O/bench_walter_32768.json 2>> $O/bench.err || exit 12
OSC_PARK_IT=0 timeout -k 10 300 python bench.py --robot walter_sr --nenv-per-gpu 32768 $B > $O/bench_walter_32768_off.json 2>> $O/bench.err || exit 13
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py $W --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 21
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py $W --steps 3 --warmup 1 $B > $O/pmc1_stdout.txt 2>&1 || exit 22
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py $W --steps 3 --warmup 1 $B > $O/pmc2_stdout.txt 2>&1 || exit 23
echo done

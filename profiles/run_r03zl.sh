# Round-3 head: bench lines for every BASELINE config at one GPU (WaLTER 4,096 = configs[2];
# WaLTER tumbling 8,192 masks redrawn = configs[3]; Go2 8,192 = the 8-GPU north-star shard;
# Go2 65,536) and rocprof kernel traces of the Go2 8,192 / 65,536 solves.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zl
mkdir -p $O
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
timeout -k 10 200 python bench.py --robot walter_sr --nenv-per-gpu 4096 --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed > $O/bench_walter_4096.json 2>> $O/err.txt || exit 10
timeout -k 10 200 python bench.py --robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192 --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed > $O/bench_walter_tumbling_8192.json 2>> $O/err.txt || exit 11
timeout -k 10 200 python bench.py --nenv-per-gpu 8192 $B > $O/bench_go2_8192.json 2>> $O/err.txt || exit 12
timeout -k 10 200 python bench.py --nenv-per-gpu 65536 --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed > $O/bench_go2_65536.json 2>> $O/err.txt || exit 13
for N in 8192 65536; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace_$N -o run --output-format csv -- python3 bench.py --nenv-per-gpu $N --steps 20 $B > $O/trace_$N.txt 2>&1 || exit 14
done
echo done

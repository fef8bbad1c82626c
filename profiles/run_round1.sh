# Commands that produced the round-1 bench lines and rocprofv3 summaries (run on the GPU box via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python bench.py > gpurun_out/bench_go2.json 2> gpurun_out/bench_go2.err || exit 11
timeout -k 10 200 python bench.py --robot walter_sr --no-cpu > gpurun_out/bench_walter.json 2>> gpurun_out/bench_go2.err || exit 12
timeout -k 10 200 python bench.py --nenv-per-gpu 65536 --steps 10 --no-cpu > gpurun_out/bench_go2_65536.json 2>> gpurun_out/bench_go2.err || exit 13
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --no-cpu > gpurun_out/prof_stdout.txt 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/pmc1_stdout.txt 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/pmc2_stdout.txt 2>&1 || exit 16
echo done

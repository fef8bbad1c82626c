# Round-1 measurement run on the GPU box (via gpurun): bench lines, rocprofv3 kernel trace,
# PMC passes (HBM traffic; FP64 / issue counters).  Outputs under gpurun_out/prof; the
# summaries are copied into profiles/ (tools/pmc_summary.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/prof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench_go2_4096.json 2> $O/bench.err || exit 11
timeout -k 10 200 python bench.py --robot walter_sr --no-cpu > $O/bench_walter_4096.json 2>> $O/bench.err || exit 12
timeout -k 10 200 python bench.py --nenv-per-gpu 65536 --steps 10 --no-cpu > $O/bench_go2_65536.json 2>> $O/bench.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 --no-cpu --no-warm --no-front-end > $O/trace_stdout.txt 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-warm --no-front-end > $O/pmc1_stdout.txt 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-warm --no-front-end > $O/pmc2_stdout.txt 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/$O/pmc_inst -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-warm --no-front-end > $O/pmc3_stdout.txt 2>&1 || exit 17
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $R/$O/pmc_cyc -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-warm --no-front-end > $O/pmc4_stdout.txt 2>&1 || exit 18
echo done

# Round-2 (final head) measurement run on the GPU box (via gpurun): bench lines for BASELINE configs[1]-[4]
# and Go2 65,536, rocprofv3 kernel traces, PMC passes (HBM traffic; FP64 / issue counters) of the
# Go2 4,096 solve.  Outputs under gpurun_out/prof2; tools/pmc_summary.py gpurun_out/prof2
# r02_go2_4096 writes the profiles/ summaries.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/prof3
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu --no-warm --no-front-end --no-single-env"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace65k -o run --output-format csv -- python3 bench.py --nenv-per-gpu 65536 --steps 10 $B > $O/trace65k_stdout.txt 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc1_stdout.txt 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc2_stdout.txt 2>&1 || exit 17
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/$O/pmc_inst -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc3_stdout.txt 2>&1 || exit 18
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $R/$O/pmc_cyc -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc4_stdout.txt 2>&1 || exit 19
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_walter -o run --output-format csv -- python3 bench.py --robot walter_sr --steps 20 $B > $O/trace_walter_stdout.txt 2>&1 || exit 20
echo done

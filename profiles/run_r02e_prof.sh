# Round-2 PMC passes at the final head (via gpurun): HBM traffic (FETCH_SIZE / WRITE_SIZE, one
# counter pass each) and issue / FP64 counters of the Go2 4,096 solve, HBM traffic of the Go2
# 65,536 solve.  Outputs under gpurun_out/prof_e{4k,64k}; summarised by
#   python tools/pmc_summary.py gpurun_out/prof_e64k r02e_go2_65536 65536
#   python tools/pmc_summary.py gpurun_out/prof_e4k r02e_go2_4096
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
B="--no-cpu --no-warm --no-front-end --no-single-env"
O=gpurun_out/prof_e4k
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc1_stdout.txt 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc2_stdout.txt 2>&1 || exit 17
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/$O/pmc_inst -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc3_stdout.txt 2>&1 || exit 18
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $R/$O/pmc_cyc -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 $B > $O/pmc4_stdout.txt 2>&1 || exit 19
O=gpurun_out/prof_e64k
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --nenv-per-gpu 65536 --steps 10 $B > $O/trace_stdout.txt 2>&1 || exit 20
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --nenv-per-gpu 65536 --steps 3 --warmup 1 $B > $O/pmc1_stdout.txt 2>&1 || exit 21
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py --nenv-per-gpu 65536 --steps 3 --warmup 1 $B > $O/pmc2_stdout.txt 2>&1 || exit 22
echo done

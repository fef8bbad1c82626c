# Round 5 closing measurement, part 2: HBM traffic (FETCH_SIZE / WRITE_SIZE passes, cache-warm and
# HBM-sourced inputs) and SQ issue counters at 4,096 / 8,192 / 65,536.
# Summaries: python tools/pmc_summary.py gpurun_out/r05z2/<n> r05z_go2_<n> <n> [hbm]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed --hbm-batches 0"
mkdir -p gpurun_out/r05z2
for n in 4096 8192 65536; do
  O=gpurun_out/r05z2/$n
  mkdir -p $O
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --nenv-per-gpu $n --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 21
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --nenv-per-gpu $n --steps 3 --warmup 1 $B > $O/pmc1_stdout.txt 2>&1 || exit 22
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py --nenv-per-gpu $n --steps 3 --warmup 1 $B > $O/pmc2_stdout.txt 2>&1 || exit 23
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/$O/pmc_inst -o run --output-format csv -- python3 bench.py --nenv-per-gpu $n --steps 3 --warmup 1 $B > $O/pmc3_stdout.txt 2>&1 || exit 24
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $R/$O/pmc_cyc -o run --output-format csv -- python3 bench.py --nenv-per-gpu $n --steps 3 --warmup 1 $B > $O/pmc4_stdout.txt 2>&1 || exit 25
  echo "pmc $n"
done
O=gpurun_out/r05z2/hbm
mkdir -p $O
A="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed --hbm-only --hbm-batches 10"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py $A --steps 60 --warmup 20 > $O/trace_stdout.txt 2>&1 || exit 26
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py $A --steps 30 --warmup 10 > $O/pmc1_stdout.txt 2>&1 || exit 27
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py $A --steps 30 --warmup 10 > $O/pmc2_stdout.txt 2>&1 || exit 28
echo done

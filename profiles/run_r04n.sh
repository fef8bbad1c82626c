# Round 4: large-batch A/B with counters -- Go2 two-wave interior point (default past one
# resident wavefront per SIMD; Hr streamed from L2 every iteration) vs the one-wave kernel forced
# (osc_model_tuning.small_batch_max; Hr staged once in LDS), at 8,192 and 65,536 envs.  Kernel
# trace + four PMC passes over tools/tune_ab.py; summary: tools/pmc_ab_summary.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
for n in 8192 65536; do
  O=gpurun_out/r04n/$n
  mkdir -p $O
  A="tools/tune_ab.py unitree_go2 $n standing ones {} {\"small_batch_max\":1000000}"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 $A > $O/trace_stdout.txt 2>&1 || exit 21
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 $A > $O/pmc1_stdout.txt 2>&1 || exit 22
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 $A > $O/pmc2_stdout.txt 2>&1 || exit 23
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/$O/pmc_inst -o run --output-format csv -- python3 $A > $O/pmc3_stdout.txt 2>&1 || exit 24
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $R/$O/pmc_cyc -o run --output-format csv -- python3 $A > $O/pmc4_stdout.txt 2>&1 || exit 25
  echo "ab $n"
done
bash profiles/run_r04m.sh

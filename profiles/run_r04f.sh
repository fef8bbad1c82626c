# Round 4: wheel-row refinement rejections classified (OSC_REFINE_DIAG build: status 3 + 16 row
# still violated + 32 not kept (move / last step / not finite) + 64 rows not holding + 128 last
# step not converged + 256 moved > 0.1); IPM and setup per-phase stamps at Go2 4,096.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
OSC_LIB_PATH=$R/operational-space-control_amd/lib/diag/libosc_batch.so timeout -k 10 200 python tools/wheel_census.py 2048 86 tumbling bernoulli > $O/wheel_diag_86.jsonl 2>&1 || exit 11
OSC_LIB_PATH=$R/operational-space-control_amd/lib/diag/libosc_batch.so timeout -k 10 200 python tools/wheel_census.py 2048 93 tumbling bernoulli > $O/wheel_diag_93.jsonl 2>&1 || exit 12
export OSC_STAMPS_LIB=$R/operational-space-control_amd/lib/libosc_batch_stamps.so
timeout -k 10 120 python tools/stamps.py 4096 > $O/ipm_stamps_4096.jsonl 2>&1 || exit 16
timeout -k 10 120 python tools/setup_stamps.py 4096 > $O/setup_stamps_4096.jsonl 2>&1 || exit 17
echo done
X=operational-space-control_amd/bin/osc_tick_latency
C=operational-space-control_amd/config
for r in unitree_go2 walter_sr; do
  timeout -k 10 120 $X $r $C/$r.xml 2000 50 > $O/tick_${r}_floors_default.json 2>&1 || exit 18
  timeout -k 10 120 $X $r $C/$r.xml 2000 50 1.0 1.0 > $O/tick_${r}_floors_1_1.json 2>&1 || exit 19
  timeout -k 10 120 $X $r $C/$r.xml 2000 50 0.1 0.3 > $O/tick_${r}_floors_01_03.json 2>&1 || exit 20
done
echo ticks
L=operational-space-control_amd/lib
timeout -k 10 300 python tools/ab_time.py $L/libosc_batch.so $L/ab/la/libosc_batch.so $L/libosc_batch.so $L/ab/la/libosc_batch.so > $O/ab_ldl_lookahead.jsonl 2>&1 || exit 21
timeout -k 10 200 python tools/ab_bitwise.py $L/libosc_batch.so $L/ab/la/libosc_batch.so > $O/ab_ldl_lookahead_bitwise.txt 2>&1 || exit 22
echo ab

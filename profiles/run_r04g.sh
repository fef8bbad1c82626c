# Round 4: wheel-row refinement variants (OSC_WH_KKT: the generic KKT acceptance; OSC_WH_NOSTOL:
# active set lambda > s only) by census; single-env tick latency vs the warm-start floors.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
L=$R/operational-space-control_amd/lib
for v in default whkkt whnostol whkktnostol; do
  lib=$L/ab/$v/libosc_batch.so; [ $v = default ] && lib=$L/libosc_batch.so
  for sd in 86 93; do
    OSC_LIB_PATH=$lib timeout -k 10 200 python tools/wheel_census.py 2048 $sd tumbling bernoulli > $O/census_${v}_$sd.jsonl 2>&1 || exit 11
  done
done
echo census
X=operational-space-control_amd/bin/osc_tick_latency
C=operational-space-control_amd/config
for r in unitree_go2 walter_sr; do
  for f in "0.3 0.3" "1.0 0.3" "0.3 1.0" "0.1 1.0" "0.5 0.5" "0.2 0.5"; do
    set -- $f
    timeout -k 10 120 $X $r $C/$r.xml 2000 50 $1 $2 > $O/tick_${r}_$1_$2.json 2>&1 || exit 12
  done
done
echo ticks

# Diagnostic (GPU box): interior-point stop threshold (OSC_EPS_MU) with the full-space refinement
# on: bench time at configs[1]/[2] and per-env torque errors of 32,768-env batches against the
# exact-oracle torques in tools/refs (tools/ref_tau.py).
# Usage: bash tools/eps_refine_sweep.sh "1e-6 1e-7 1e-8 1e-9" [outdir]
set -o pipefail
EPS=${1:-"1e-7 1e-8 1e-9"}
O=${2:-gpurun_out/eps}
mkdir -p $O
for eps in $EPS; do
  for r in unitree_go2 walter_sr; do
    s=${r%%_*}; s=${s/unitree/go2}
    OSC_EPS_MU=$eps timeout -k 10 120 python bench.py --robot $r --no-cpu --no-single-env --no-warm --no-front-end > $O/b_${r}_${eps}.json 2>>$O/err || exit 3
    OSC_EPS_MU=$eps timeout -k 10 200 python tools/dump_tau.py $r tumbling bernoulli 32768 7 $O/${r}_tum_${eps}.npz tools/refs/${s}_tum.npz >> $O/dump.log 2>>$O/err || exit 4
    OSC_EPS_MU=$eps timeout -k 10 200 python tools/dump_tau.py $r standing ones 32768 2 $O/${r}_st_${eps}.npz tools/refs/${s}_st.npz >> $O/dump.log 2>>$O/err || exit 5
  done
done
echo done

set -o pipefail
mkdir -p gpurun_out/r03k
for v in "X=1" "OSC_RESTART_ITER=1000" "OSC_WHEEL_TOL=1e-2" "OSC_EPS_MU=1e-6" "OSC_REFINE_STEPS=0"; do
  env $v timeout -k 10 120 python -u tools/wheel_ws_dump.py gpurun_out/r03k/x.npz tumbling 86 2048 2,14,16,18,25,0,1,3 > gpurun_out/r03k/v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/r03k/v.log)"
done

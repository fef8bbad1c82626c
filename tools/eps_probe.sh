set -o pipefail
mkdir -p gpurun_out/r06eps
for e in default 3e-6 1e-5; do
  if [ "$e" = default ]; then unset OSC_EPS_MU; else export OSC_EPS_MU=$e; fi
  AB_ROUNDS=3 AB_CONFIGS=unitree_go2:4096,unitree_go2:8192,unitree_go2:65536 timeout -k 10 300 python tools/ab_time.py operational-space-control_amd/lib/libosc_batch.so > gpurun_out/r06eps/ab_$e.jsonl 2>&1 || exit 1
done
export OSC_EPS_MU=1e-5
timeout -k 10 400 python -u -m pytest tests/test_gpu_full_parity.py tests/test_gpu_joint_states.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06eps/parity_1e-5.log 2>&1
echo rc=$?

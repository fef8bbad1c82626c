# Diagnostic: step-fraction variants (libosc_batch_<v>.so built with -DOSC_ETA_*): parity + time.
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  export OSC_LIB_PATH=$PWD/operational-space-control_amd/lib/libosc_batch_$v.so
  timeout -k 5 120 python -m pytest tests/test_gpu_parity.py -q -k fresh > gpurun_out/eta_$v.log 2>&1
  tail -1 gpurun_out/eta_$v.log
  timeout -k 5 120 python tools/eps_sweep.py 1e-12 || exit 1
done

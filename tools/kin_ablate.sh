#!/bin/bash
# Stage ablation of the kinematics kernel: builds libosc_batch.so variants that stop before
# stage k (k = 0..5) under operational-space-control_amd/lib/ablate/kin_stop<k>/ (run here, cross-compiled), then on the GPU
#   for k in 0 1 2 3 4 5 full; do OSC_LIB_PATH=... python tools/kin_bench.py; done
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/operational-space-control_amd/csrc
if [ "$1" = "build" ]; then
  cd $R/operational-space-control_amd
  for k in 0 1 2 3 4 5; do
    python -m osc_amd.build -f --out $R/operational-space-control_amd/lib/ablate/kin_stop$k -DOSC_KIN_STOP=$k
  done
  wait
  exit 0
fi
for k in 0 1 2 3 4 5; do
  echo "stop before stage $k"
  OSC_LIB_PATH=$R/operational-space-control_amd/lib/ablate/kin_stop$k/libosc_batch.so timeout -k 10 60 python $R/tools/kin_bench.py --steps 20
done
echo "full"
timeout -k 10 60 python $R/tools/kin_bench.py --steps 20

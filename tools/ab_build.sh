#!/bin/bash
# Builds libosc_batch.so variants for A/B timing (tools/ab_time.py) under
# operational-space-control_amd/lib/ablate/<name>/ (cross-compiled here; travels to the GPU box).
#   bash tools/ab_build.sh name "-DFLAG=1 ..." [name2 "flags2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/operational-space-control_amd/csrc
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  mkdir -p $R/operational-space-control_amd/lib/ablate/$n
  /opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -fPIC -shared $f -I $R/include \
    $C/osc_batch.hip $C/osc_model.cpp $C/osc_mjcf.cpp $C/osc_producers.hip $C/osc_kinematics.hip \
    -o $R/operational-space-control_amd/lib/ablate/$n/libosc_batch.so 2>&1 | grep -E "error" || true &
done
wait

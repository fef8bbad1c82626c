#!/bin/bash
# Builds libosc_batch.so variants for A/B timing (tools/ab_time.py) under
# operational-space-control_amd/lib/ablate/<name>/ (cross-compiled here; travels to the GPU box).
#   bash tools/ab_build.sh name "-DFLAG=1 ..." [name2 "flags2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R/operational-space-control_amd
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  python -m osc_amd.build -f --out $R/operational-space-control_amd/lib/ablate/$n $f
done

# Round 4: A/B of the LLVM max-ILP machine scheduler (-mllvm -amdgpu-sched-strategy=max-ilp) against the default build, Go2 4,096 main leg, 100 + 300 steps, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04_ilp_ab
mkdir -p $O
L=operational-space-control_amd/lib
cp $L/libosc_batch.so /tmp/osc_default.so
B="--steps 300 --warmup 100 --no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
for r in 1 2 3; do
  for v in default ilp; do
    if [ $v = default ]; then cp /tmp/osc_default.so $L/libosc_batch.so; else cp operational-space-control_amd/lib_ab/libosc_batch_ilp.so $L/libosc_batch.so; fi
    timeout -k 10 120 python bench.py $B > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 11
  done
done
cp /tmp/osc_default.so $L/libosc_batch.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_wheels.py -q -k feature_off --timeout 200 --timeout-method thread > $O/feature_off_default.log 2>&1 || exit 12
cp operational-space-control_amd/lib_ab/libosc_batch_ilp.so $L/libosc_batch.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_wheels.py -q -k feature_off --timeout 200 --timeout-method thread > $O/feature_off_ilp.log 2>&1
echo "ilp feature-off rc $?"
cp /tmp/osc_default.so $L/libosc_batch.so
echo done

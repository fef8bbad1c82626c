# Round 5: fix-up pass in the two-model kernels -- mixed tests, then mixed bench A/B (old build in
# lib/ab_old vs the in-tree build), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05pf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 31
B="--robot mixed --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed --hbm-batches 0"
OLD=$R/operational-space-control_amd/lib/ab_old/libosc_batch.so
for i in 1 2 3; do
  timeout -k 10 200 env OSC_LIB_PATH=$OLD python bench.py $B > $O/old_$i.json 2>> $O/bench.err || exit 32
  timeout -k 10 200 python bench.py $B > $O/new_$i.json 2>> $O/bench.err || exit 33
done
echo done

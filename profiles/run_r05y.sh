# Round 5: the wheel basis completion's Gram-Schmidt with a compile-time shape (LDS reads issued
# ahead of the FMA chains; FMA order unchanged) -- setup stamps, wheel timing against the previous
# library, wheel GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05y
mkdir -p $O
OSC_STAMPS_LIB=operational-space-control_amd/lib/stamps/libosc_batch.so timeout -k 10 200 python tools/setup_stamps.py 2048 noslip > $O/setup_stamps.jsonl 2> $O/setup_stamps.err || exit 30
for lib in ab_old/libosc_batch.so libosc_batch.so; do
  for sc in "tumbling bernoulli" "standing ones"; do
    OSC_LIB_PATH=operational-space-control_amd/lib/$lib timeout -k 10 300 python tools/wheel_census.py 2048 91 $sc 1 '{}' --brief >> $O/wheel_ab.jsonl 2>> $O/wheel_ab.err || exit 31
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 34
echo done

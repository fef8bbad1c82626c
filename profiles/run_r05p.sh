# Round 5: wheel basis completion by Householder reflections -- wheel census (4 x 2,048, every env
# OK + certified), timing against the previous library, then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05p
mkdir -p $O
for lib in ab_old/libosc_batch.so libosc_batch.so; do
  for sc in "tumbling bernoulli" "standing ones"; do
    OSC_LIB_PATH=operational-space-control_amd/lib/$lib timeout -k 10 300 python tools/wheel_census.py 2048 91 $sc 1 '{}' --brief >> $O/wheel_ab.jsonl 2>> $O/wheel_ab.err || exit 31
  done
done
for seed in 86 87; do
  for sc in "tumbling bernoulli" "standing ones"; do
    timeout -k 10 300 python tools/wheel_census.py 2048 $seed $sc 4 >> $O/census.jsonl 2>> $O/census.err || exit 32
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 33
echo done

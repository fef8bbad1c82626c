# Round 5: the fused joint-state tick after the mask-slot fix -- its tests, an interleaved A/B
# against the two-kernel tick (lib/ablate/nofuse, -DOSC_NO_FUSED_TICK), and the default bench
# line in the driver's 20 + 5 window (headline after the north-star / mixed lines).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kinematics.py tests/test_gpu_joint_states.py tests/test_controller_shim.py tests/test_dropin.py tests/test_gpu_pipeline.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -le 1 ] || exit $rc
L=operational-space-control_amd/lib
TICK_ROUNDS=3 timeout -k 10 400 python tools/tick_ab.py $L/libosc_batch.so $L/ablate/nofuse/libosc_batch.so > $O/tick_ab.jsonl 2> $O/tick_ab.err || exit 31
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default_20x5.json 2> $O/bench_default_20x5.err || exit 32
echo done

# Round 5: the fused joint-state tick (kinematics in the assembly kernel's prologue): the tests
# that pin it (bitwise = kinematics + solve; every env vs the oracle) and the bench's front end.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kinematics.py tests/test_gpu_joint_states.py tests/test_controller_shim.py tests/test_dropin.py tests/test_gpu_pipeline.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -le 1 ] || exit $rc
for robot in unitree_go2 walter_sr; do
  timeout -k 10 300 python bench.py --robot $robot --no-cpu --no-single-env --no-north-star --no-mixed --hbm-batches 0 --no-warm > $O/bench_$robot.json 2> $O/bench_$robot.err || exit 30
done
timeout -k 10 300 python bench.py --nenv-per-gpu 65536 --steps 50 --warmup 20 --no-cpu --no-single-env --no-north-star --no-mixed --hbm-batches 0 --no-warm > $O/bench_go2_65536.json 2> $O/bench_go2_65536.err || exit 31
echo done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default_20x5.json 2> $O/bench_default_20x5.err || exit 32
echo bench-default
L=operational-space-control_amd/lib
AB_ROUNDS=5 AB_CHECK=1 AB_CONFIGS=unitree_go2:4096,unitree_go2:8192,unitree_go2:65536 timeout -k 10 300 python tools/ab_time.py $L/libosc_batch.so $L/ablate/su4/libosc_batch.so > $O/ab_setup_unroll4.jsonl 2>&1 || exit 33
grep summary $O/ab_setup_unroll4.jsonl

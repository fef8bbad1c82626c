# Round 4: refinement rounds 4 -> 8 (only envs still violating after round 4 run more) -- the
# 65,536-env Go2 joint-state census that left one env UNREFINED, the feature-off fingerprints,
# stage / joint-state / parity GPU tests, time at configs[1]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04_rounds
mkdir -p $O
timeout -k 10 200 python tools/tune_ab.py unitree_go2 65536 qpos1.0 bernoulli '{}' > $O/go2_qpos10_bern.jsonl 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests/test_gpu_wheels.py::test_feature_off_bitwise_unchanged tests/test_gpu_joint_states.py tests/test_gpu_stages.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc $?"
OSC_AB_ROUNDS=3 timeout -k 10 200 python tools/tune_ab.py unitree_go2 4096 standing ones '{}' > $O/go2_4096.jsonl 2>&1 || exit 12
echo done

# Round 4: early interior-point stops (Go2 1e-6, WaLTER 1e-8) + KKT-accepted refinement + warm
# start with wheel rows -- the feature-off fingerprints regenerated for this intentional numerical
# change, joint-state tests, the whole GPU suite, the default bench line and its kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 200 python tests/golden/make_feature_off_hashes.py > $O/feature_off_hashes.json 2> $O/hashes.err || exit 8
cp $O/feature_off_hashes.json tests/golden/feature_off_hashes.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_joint_states.py -v --timeout 200 --timeout-method thread > $O/joint_tests.log 2>&1
echo "joint rc $?"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread --deselect tests/test_gpu_joint_states.py > $O/gpu_tests.log 2>&1
echo "suite rc $?"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 11
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 12
echo done
T="timeout -k 10 120 python tools/tune_ab.py"
$T unitree_go2 4096 standing ones '{"eps_mu": 1e-9}' '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' '{"eps_mu": 1e-4}' > $O/tune_go2_4096.jsonl 2>&1 || exit 13
$T unitree_go2 4096 qpos0.5 ones '{"eps_mu": 1e-9}' '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' '{"eps_mu": 1e-4}' > $O/tune_go2_4096_qpos.jsonl 2>&1 || exit 14
$T unitree_go2 65536 standing ones '{"eps_mu": 1e-9}' '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' '{"eps_mu": 1e-4}' > $O/tune_go2_65536.jsonl 2>&1 || exit 15
$T walter_sr 4096 standing ones '{"eps_mu": 1e-12}' '{"eps_mu": 1e-8}' '{"eps_mu": 1e-6}' > $O/tune_walter_4096.jsonl 2>&1 || exit 16
$T walter_sr 8192 tumbling bernoulli '{"eps_mu": 1e-12}' '{"eps_mu": 1e-8}' '{"eps_mu": 1e-6}' > $O/tune_walter_8192_tum.jsonl 2>&1 || exit 17
echo tuned

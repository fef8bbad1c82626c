# Round 4: fallback back substitution by v_readlane + stored reciprocals (wheel tests, census time,
# per-phase cycles); WaLTER / Go2 refinement-step and early-stop sweep (tools/tune_ab.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wheels.py -q --timeout 200 --timeout-method thread > $O/wheel_tests.log 2>&1
echo "tests rc $?"
timeout -k 10 120 python tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/census_time_86.jsonl 2>&1 || exit 14
OSC_LIB_PATH=operational-space-control_amd/lib/ab/giprof/libosc_batch.so timeout -k 10 200 python tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/giprof_86.txt 2>&1 || exit 20
timeout -k 10 300 python tools/tune_ab.py walter_sr 4096 standing ones '{}' '{"refine_steps": 1}' '{"refine_steps": 3}' '{"eps_mu": 1e-9}' '{"eps_mu": 1e-7}' '{}' > $O/tune_walter_4096.jsonl 2>&1 || exit 30
timeout -k 10 300 python tools/tune_ab.py unitree_go2 4096 standing ones '{}' '{"refine_steps": 1}' '{"refine_steps": 3}' '{}' > $O/tune_go2_4096.jsonl 2>&1 || exit 31
echo done

# Round 4: wheel refine_steps 12 -> 4 now that stall-exit envs with a rejected refinement go to the fallback -- wheel + warm tests, censuses, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04zg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wheels.py tests/test_gpu_warm.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc $?"
for sd in 86 91 93; do
  timeout -k 10 200 python tools/wheel_census.py 2048 $sd tumbling bernoulli > $O/census_$sd.jsonl 2>&1 || exit 11
done
timeout -k 10 200 python tools/wheel_census.py 2048 81 standing ones > $O/census_standing_81.jsonl 2>&1 || exit 12
timeout -k 10 300 python tools/wheel_census.py 2048 97 tumbling bernoulli 5 > $O/census_warm_97.jsonl 2>&1 || exit 13
timeout -k 10 120 python tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/census_time_86.jsonl 2>&1 || exit 14
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/trace_stdout.txt 2>&1 || exit 15
echo done

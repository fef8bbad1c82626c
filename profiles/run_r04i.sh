# Round 4: wheel rows -- duals from stationarity (least squares for the rows' multipliers), the
# interior point's converged iterate kept where the refinement fails -- census x3 seeds + warm,
# the wheel GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
for sd in 86 91 93; do
  timeout -k 10 200 python tools/wheel_census.py 2048 $sd tumbling bernoulli > $O/census_$sd.jsonl 2>&1 || exit 11
done
timeout -k 10 200 python tools/wheel_census.py 2048 81 standing ones > $O/census_standing_81.jsonl 2>&1 || exit 12
timeout -k 10 300 python tools/wheel_census.py 2048 97 tumbling bernoulli 5 > $O/census_warm_97.jsonl 2>&1 || exit 13
timeout -k 10 400 python -u -m pytest tests/test_gpu_wheels.py -v --timeout 200 --timeout-method thread > $O/wheel_tests.log 2>&1
echo "tests rc $?"

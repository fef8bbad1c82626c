# Round 4: wheel-row census (cold tumbling x3 seeds, standing, warm ticks) after the KKT-refinement
# fixes; per-phase stamps of the IPM and setup kernels (OSC_STAMPS build) at Go2 4,096.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
W="timeout -k 10 200 python tools/wheel_census.py"
$W 2048 86 tumbling bernoulli > $O/wheel_census_86.jsonl 2>&1 || exit 11
$W 2048 91 tumbling bernoulli > $O/wheel_census_91.jsonl 2>&1 || exit 12
$W 2048 93 tumbling bernoulli > $O/wheel_census_93.jsonl 2>&1 || exit 13
$W 2048 81 standing ones > $O/wheel_census_standing_81.jsonl 2>&1 || exit 14
$W 2048 97 tumbling bernoulli 5 > $O/wheel_census_warm_97.jsonl 2>&1 || exit 15
export OSC_STAMPS_LIB=$R/operational-space-control_amd/lib/libosc_batch_stamps.so
timeout -k 10 120 python tools/stamps.py 4096 > $O/ipm_stamps_4096.jsonl 2>&1 || exit 16
timeout -k 10 120 python tools/setup_stamps.py 4096 > $O/setup_stamps_4096.jsonl 2>&1 || exit 17
echo done

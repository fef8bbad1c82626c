# Round 5: the dual kernel's per-phase clocks (-DOSC_DUAL_PROFILE build) on a tumbling wheel batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/${DU_OUT:-r05du}
mkdir -p $O
OSC_LIB_PATH=operational-space-control_amd/lib/duprof/libosc_batch.so timeout -k 10 300 python tools/wheel_census.py 2048 91 tumbling bernoulli 1 '{}' --brief > $O/dual_profile.txt 2> $O/err.txt || exit 31
echo done

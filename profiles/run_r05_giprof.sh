# Round 5: the wheel fallback's cycle profile (-DOSC_GI_PROFILE build) on one tumbling census batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/${GI_OUT:-r05giprof}
mkdir -p $O
OSC_LIB_PATH=operational-space-control_amd/lib/giprof/libosc_batch.so timeout -k 10 300 python tools/wheel_census.py 2048 91 tumbling bernoulli 1 '{}' --brief > $O/gi_profile.txt 2> $O/err.txt || exit 31
echo done

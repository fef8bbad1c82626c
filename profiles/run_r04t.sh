# Round 4: kernel trace of the wheel-row solve (2,048 tumbling envs, duals on): setup, interior
# point, active-set fallback, duals
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/trace_stdout.txt 2>&1 || exit 12
echo done

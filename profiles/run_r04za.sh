# Round 4: wheel setup -- CGS2 for every Gram-Schmidt pass vs CGS2 for the 48-row basis completion
# only (the 16-row sets by the register MGS): kernel traces of the 2,048-env wheel solve
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04za
mkdir -p $O
L=operational-space-control_amd/lib
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace_all -o run --output-format csv -- python3 tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/all.txt 2>&1 || exit 15
OSC_LIB_PATH=$L/ab/mixed/libosc_batch.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace_mixed -o run --output-format csv -- python3 tools/wheel_census.py 2048 86 tumbling bernoulli 1 {} --brief > $O/mixed.txt 2>&1 || exit 16
echo done

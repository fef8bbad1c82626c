# Round 4: steady-state kernel times at configs[1] -- rocprofv3 kernel trace over 300 timed steps
# (the default bench line times 20 after 5 warmup steps from an idle GPU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04_steady
mkdir -p $O
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 300 --warmup 50 $B > $O/trace_stdout.txt 2>&1 || exit 12
echo done

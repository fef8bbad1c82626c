# Round-1 kinematics front-end measurement (via gpurun): kernel trace of the default bench (which
# times osc_kinematics_kernel beside the headline) and FETCH_SIZE / WRITE_SIZE passes over
# tools/kin_bench.py (Go2 / WaLTER at 4,096 and 65,536 envs).  Outputs under gpurun_out/prof_kin.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/prof_kin
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --steps 20 --no-cpu > $O/trace_stdout.txt 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kin_trace -o run --output-format csv -- python3 tools/kin_bench.py --steps 20 > $O/kin_trace_stdout.txt 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 tools/kin_bench.py --steps 3 > $O/pmc1_stdout.txt 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 tools/kin_bench.py --steps 3 > $O/pmc2_stdout.txt 2>&1 || exit 17
echo done

# Round-3 final head: Go2 4,096 kernel trace + HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter
# pass each).  Summarised by  python tools/pmc_summary.py gpurun_out/r03zu r03zu_go2_4096 4096
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
O=gpurun_out/r03zu
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --nenv-per-gpu 4096 --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 21
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --nenv-per-gpu 4096 --steps 3 --warmup 1 $B > $O/pmc1_stdout.txt 2>&1 || exit 22
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py --nenv-per-gpu 4096 --steps 3 --warmup 1 $B > $O/pmc2_stdout.txt 2>&1 || exit 23
echo done

# Round-3 kernel traces + HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter pass each) of the Go2
# solve at 4,096, 8,192 and 65,536 envs per launch.  Summarised by
#   python tools/pmc_summary.py gpurun_out/r03t_<n> r03_go2_<n> <n>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
for N in 4096 8192 65536; do
  O=gpurun_out/r03t_$N
  mkdir -p $O
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py --nenv-per-gpu $N --steps 20 $B > $O/trace_stdout.txt 2>&1 || exit 21
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py --nenv-per-gpu $N --steps 3 --warmup 1 $B > $O/pmc1_stdout.txt 2>&1 || exit 22
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py --nenv-per-gpu $N --steps 3 --warmup 1 $B > $O/pmc2_stdout.txt 2>&1 || exit 23
done
echo done

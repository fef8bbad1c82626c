# Round 5: roofline.hbm_inputs -- Go2 4,096 with the inputs rotated through 10 copies (314 MB >
# the 256 MB Infinity Cache; bench.py --hbm-only): kernel trace + FETCH_SIZE / WRITE_SIZE passes,
# and the same passes of the cache-warm headline step for comparison.
# Summaries: python tools/pmc_summary.py gpurun_out/r05_hbm/hbm r05_hbm_go2_4096 4096 hbm
#            python tools/pmc_summary.py gpurun_out/r05_hbm/cache r05_cache_go2_4096 4096
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed --hbm-batches 0"
mkdir -p gpurun_out/r05_hbm
for mode in hbm cache; do
  O=gpurun_out/r05_hbm/$mode
  mkdir -p $O
  if [ $mode = hbm ]; then A="--hbm-only --hbm-batches 10"; else A="$B"; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 bench.py $A --steps 60 --warmup 20 > $O/trace_stdout.txt 2>&1 || exit 21
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 bench.py $A --steps 30 --warmup 10 > $O/pmc1_stdout.txt 2>&1 || exit 22
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 bench.py $A --steps 30 --warmup 10 > $O/pmc2_stdout.txt 2>&1 || exit 23
  echo "pmc $mode"
done
echo done

# per-kernel rocprofv3 stats of the cold solve for several library builds (AB_ONLY config)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for lib in "$@"; do
  n=$(basename $lib .so)
  AB_ONLY=${AB_ONLY:-unitree_go2:4096} timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$n -o $n --output-format csv -- python3 $R/tools/ab_time.py $R/$lib > $R/gpurun_out/prof_$n.log 2>&1 || exit $?
  f=$(find $R/gpurun_out/prof_$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; cut -d, -f1-5 "$f" | head -4
done

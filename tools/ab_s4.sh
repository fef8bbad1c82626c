# setup4 A/B: stamps of the four-envs-per-wave setup, A/B timing + bitwise vs the 64-lane setup
A=operational-space-control_amd/lib/ablate
OSC_SETUP4=1 OSC_STAMPS_LIB=$A/st_s41/libosc_batch.so timeout -k 10 120 python tools/setup_stamps.py 4096 2>&1 | grep unitree || exit 2
bash tools/ab_run.sh s4 s40 s41 || exit 3
cd /tmp && export TMPDIR=/tmp
for v in s40 s41; do AB_ONLY=unitree_go2:4096 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$v -o $v --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_time.py $GRAFT_REPO_ROOT/$A/$v/libosc_batch.so > $GRAFT_REPO_ROOT/gpurun_out/prof_$v.log 2>&1 || exit 4; done
for v in s40 s41; do python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])): print(sys.argv[2], r['Name'][:60].split('<')[0][-25:], r['Calls'], round(float(r['AverageNs'])/1000,2),'us')
" $GRAFT_REPO_ROOT/gpurun_out/prof_$v/${v}_kernel_stats.csv $v; done

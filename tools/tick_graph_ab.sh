set -o pipefail
O=gpurun_out/tg2; mkdir -p $O
B=operational-space-control_amd/bin/osc_tick_latency
C=operational-space-control_amd/config
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 10
for r in unitree_go2 walter_sr; do
  timeout -k 10 120 $B $r $C/$r.xml 2000 > $O/${r}_off.json 2>$O/${r}_off.err || exit 11
  OSC_TICK_GRAPH=1 timeout -k 10 120 $B $r $C/$r.xml 2000 > $O/${r}_on.json 2>$O/${r}_on.err || exit 12
  timeout -k 10 120 $B $r $C/$r.xml 2000 > $O/${r}_off2.json 2>>$O/${r}_off.err || exit 13
  OSC_TICK_GRAPH=1 timeout -k 10 120 $B $r $C/$r.xml 2000 > $O/${r}_on2.json 2>>$O/${r}_on.err || exit 14
done

timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $PWD/$O/prof -o run --output-format csv -- $B unitree_go2 $C/unitree_go2.xml 1000 > $O/prof_stdout.txt 2>&1 || exit 15
echo profiled
echo done

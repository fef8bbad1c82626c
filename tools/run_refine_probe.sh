A=operational-space-control_amd/lib/ablate
OSC_STAMPS_LIB=$A/st_xe/libosc_batch.so timeout -k 10 200 python tools/stamps.py 4096 2>&1 | grep unitree
bash tools/ab_run.sh xe s40 xe 2>&1 | grep -v walter
mkdir -p gpurun_out/rs1
for r in unitree_go2 walter_sr; do s=${r%%_*}; s=${s/unitree/go2}
 OSC_REFINE_STEPS=1 timeout -k 10 200 python tools/dump_tau.py $r tumbling bernoulli 32768 7 gpurun_out/rs1/${r}_tum.npz tools/refs/${s}_tum.npz 2>/dev/null
 OSC_REFINE_STEPS=1 timeout -k 10 200 python tools/dump_tau.py $r standing ones 32768 2 gpurun_out/rs1/${r}_st.npz tools/refs/${s}_st.npz 2>/dev/null
done

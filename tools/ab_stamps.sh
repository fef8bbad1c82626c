# IPM loop phase stamps of the unfused (refinement off: the refine kernel would overwrite them) and
# the fused build, then rocprof kernel stats of both product builds (Go2 4,096).
A=operational-space-control_amd/lib/ablate
OSC_REFINE_STEPS=0 OSC_STAMPS_LIB=$A/st_fuse0/libosc_batch.so timeout -k 10 200 python tools/stamps.py 4096 > gpurun_out/stamps_st_fuse0.json 2>&1 || exit 3
OSC_STAMPS_LIB=$A/st_fuse1/libosc_batch.so timeout -k 10 200 python tools/stamps.py 4096 > gpurun_out/stamps_st_fuse1.json 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
for v in fuse0 fuse1; do AB_ONLY=unitree_go2:4096 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$v -o $v --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_time.py $GRAFT_REPO_ROOT/$A/$v/libosc_batch.so > $GRAFT_REPO_ROOT/gpurun_out/prof_$v.log 2>&1 || exit 4; done

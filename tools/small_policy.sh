# One-wave fused kernel (interior point + refinement) vs two-wave kernel + refine kernel at large
# batches: OSC_SMALL_BATCH_MAX forces the one-wave variant for every batch size.
L=operational-space-control_amd/lib/libosc_batch.so
timeout -k 10 200 python tools/ab_time.py $L 2>&1 | grep nenv
OSC_SMALL_BATCH_MAX=100000000 timeout -k 10 200 python tools/ab_time.py $L 2>&1 | grep nenv
timeout -k 10 200 python tools/ab_time.py $L 2>&1 | grep nenv
OSC_SMALL_BATCH_MAX=100000000 timeout -k 10 200 python tools/ab_time.py $L 2>&1 | grep nenv

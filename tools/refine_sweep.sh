mkdir -p gpurun_out/r2j
for eps in 1e-12 1e-10 1e-9; do for st in 1 2; do
 OSC_EPS_MU=$eps OSC_REFINE_STEPS=$st timeout -k 10 120 python bench.py --no-cpu --no-single-env --no-warm --no-front-end > gpurun_out/r2j/b_${eps}_${st}.json 2>>gpurun_out/r2j/err || exit 3
done; done
OSC_EPS_MU=1e-9 OSC_REFINE_STEPS=1 timeout -k 10 200 python tools/dump_tau.py unitree_go2 tumbling bernoulli 32768 7 gpurun_out/r2j/go2_e9_s1.npz || exit 4
OSC_EPS_MU=1e-9 OSC_REFINE_STEPS=2 timeout -k 10 200 python tools/dump_tau.py unitree_go2 standing ones 32768 2 gpurun_out/r2j/go2st_e9_s2.npz || exit 5
OSC_EPS_MU=1e-12 OSC_REFINE_STEPS=1 timeout -k 10 200 python tools/dump_tau.py walter_sr tumbling bernoulli 32768 7 gpurun_out/r2j/wal_e12_s1.npz || exit 6

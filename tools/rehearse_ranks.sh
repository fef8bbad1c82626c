# One-GPU box: bench.py --gpus 2 end to end (spawned ranks, per-rank GPU solve, max-over-ranks
# reduction), both ranks on cuda:0 with barriers and the reduction over gloo.  Not a scaling number.
set -o pipefail
O=gpurun_out/rehearse; mkdir -p $O
OSC_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --no-cpu --no-warm --no-front-end --no-single-env > $O/go2_2ranks.json 2> $O/go2_2ranks.err || exit 3
timeout -k 10 200 python bench.py --gpus 1 --steps 10 --no-cpu --no-warm --no-front-end --no-single-env > $O/go2_1rank.json 2> $O/go2_1rank.err || exit 4
WORLD_SIZE=2 timeout -k 10 60 python bench.py --gpus 3 > $O/mismatch.out 2>&1; echo "mismatch rc=$?" >> $O/mismatch.out
echo done

set -o pipefail
O=gpurun_out/rehearse; mkdir -p $O
OSC_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --robot mixed --gpus 2 --steps 10 --no-cpu > $O/mixed_2ranks.json 2> $O/mixed_2ranks.err || exit 3
echo done

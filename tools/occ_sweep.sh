set -e
for n in 2048 4096 8192 16384; do
  echo "small n=$n"; OSC_SMALL_BATCH_MAX=100000000 timeout -k 5 120 python bench.py --no-cpu --nenv-per-gpu $n --steps 20 --warmup 3 | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print(d['ms_per_step'], d['roofline'].get('kernel_ms_split'))"
  echo "large n=$n"; OSC_SMALL_BATCH_MAX=0 timeout -k 5 120 python bench.py --no-cpu --nenv-per-gpu $n --steps 20 --warmup 3 | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print(d['ms_per_step'], d['roofline'].get('kernel_ms_split'))"
done

for v in 0 100000000; do
  echo "== OSC_SMALL_BATCH_MAX=$v"
  OSC_SMALL_BATCH_MAX=$v timeout -k 5 100 python tools/eps_sweep.py 1e-12 || exit 1
done

# Round-3: warm-start settings past one wavefront per SIMD (throughput-bound: the mean iterations
# set the time) and for the single-env controller tick -- bench.py warm / single_env objects.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zn
mkdir -p $O
B="--no-cpu --no-front-end --no-single-env --no-north-star --no-mixed"
for cfg in "0.3 0.1" "1.0 1.0" "0.3 1.0"; do
  set -- $cfg
  E="OSC_WARM_CENTER=$1 OSC_WARM_DELTA=$2"
  env $E timeout -k 10 200 python bench.py --nenv-per-gpu 65536 $B > $O/go2_65536_$1_$2.json 2>> $O/err.txt || exit 10
  env $E timeout -k 10 200 python bench.py --robot walter_sr --scenario tumbling --mask bernoulli --mask-redraw 8 --nenv-per-gpu 8192 $B > $O/walter_tumb_8192_$1_$2.json 2>> $O/err.txt || exit 11
  env $E timeout -k 10 200 python bench.py --robot walter_sr --nenv-per-gpu 32768 $B > $O/walter_32768_$1_$2.json 2>> $O/err.txt || exit 12
  env $E timeout -k 10 200 python bench.py --nenv-per-gpu 8192 $B > $O/go2_8192_$1_$2.json 2>> $O/err.txt || exit 13
  env $E timeout -k 10 200 python bench.py --no-cpu --no-front-end --no-warm --no-north-star --no-mixed > $O/single_$1_$2.json 2>> $O/err.txt || exit 14
done
echo done

# Round-3: warm-start settings at one wavefront per SIMD (4,096 envs, latency-bound: the slowest
# env's iterations set the time) -- bench.py warm object for WaLTER and Go2 per setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zm
mkdir -p $O
B="--no-cpu --no-front-end --no-single-env --no-north-star --no-mixed"
for cfg in "0.3 0.1 22" "1.0 0.1 22" "0.3 1.0 22" "1.0 1.0 22" "0.3 0.1 12" "1.0 1.0 12"; do
  set -- $cfg
  for robot in walter_sr unitree_go2; do
    OSC_WARM_CENTER=$1 OSC_WARM_DELTA=$2 OSC_WARM_RESTART=$3 timeout -k 10 200 python bench.py --robot $robot $B > $O/warm_${robot}_$1_$2_$3.json 2>> $O/err.txt || exit 10
  done
done
echo done

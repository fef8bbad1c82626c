# Round-3: one-wave vs two-wave IPM variant for Go2 past one resident wave per SIMD
# (OSC_SMALL_BATCH_MAX forces the one-wave kernel): 6,144 / 8,192 (north-star shard) / 16,384 / 65,536.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zi
mkdir -p $O
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
for N in 6144 8192 16384 65536; do
  timeout -k 10 200 python bench.py --nenv-per-gpu $N $B > $O/two_$N.json 2>> $O/err.txt || exit 10
  OSC_SMALL_BATCH_MAX=100000000 timeout -k 10 200 python bench.py --nenv-per-gpu $N $B > $O/one_$N.json 2>> $O/err.txt || exit 11
done
echo done

# Round-3 first GPU check after pruning the dead kernel variants: GPU tests, smoke, the default
# bench line (configs[1]) and the north-star per-GPU shard (Go2 8,192 envs: 65,536 over 8 GPUs)
# with its rocprofv3 kernel trace; bitwise fingerprints of the round-2 library and the head.  Outputs under gpurun_out/r03a.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
T="--no-cpu --no-warm --no-front-end --no-single-env"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --no-cpu --no-single-env > $O/bench_go2_4096.json 2> $O/bench.err || exit 12
timeout -k 10 300 python bench.py --nenv-per-gpu 8192 $T > $O/bench_go2_8192.json 2>> $O/bench.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace8192 -o run --output-format csv -- python3 bench.py --nenv-per-gpu 8192 --steps 20 $T > $O/trace8192_stdout.txt 2>&1 || exit 14
OSC_LIB_PATH=$R/baseline_lib/libosc_batch_r02.so timeout -k 10 300 python tests/golden/make_feature_off_hashes.py > $O/feature_off_hashes_r02lib.json 2>> $O/bench.err || exit 15
timeout -k 10 300 python tests/golden/make_feature_off_hashes.py > $O/feature_off_hashes_head.json 2>> $O/bench.err || exit 16
echo done

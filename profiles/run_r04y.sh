# Round 4: setup kernel's Ha tile loop unrolled 4 / 8 instead of fully (256 -> 100 VGPRs: the
# setup wavefronts then fill the CU to its LDS limit, 11 per CU instead of 8) -- A/B + bitwise
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
L=operational-space-control_amd/lib
timeout -k 10 400 python tools/ab_time.py $L/libosc_batch.so $L/ab/ha4/libosc_batch.so $L/ab/ha8/libosc_batch.so $L/libosc_batch.so $L/ab/ha4/libosc_batch.so $L/ab/ha8/libosc_batch.so > $O/ab_ha_unroll.jsonl 2>&1 || exit 21
timeout -k 10 200 python tools/ab_bitwise.py $L/libosc_batch.so $L/ab/ha4/libosc_batch.so > $O/ab_ha_bitwise.txt 2>&1 || exit 22
B="--no-cpu --no-warm --no-front-end --no-single-env --no-north-star --no-mixed"
OSC_LIB_PATH=$L/ab/ha4/libosc_batch.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace_ha4 -o run --output-format csv -- python3 bench.py --steps 50 $B > $O/trace_ha4.txt 2>&1 || exit 23
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/trace_base -o run --output-format csv -- python3 bench.py --steps 50 $B > $O/trace_base.txt 2>&1 || exit 24
echo done

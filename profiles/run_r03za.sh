# Round-3: lockstep compaction A/B (tools/park_sweep.py): bitwise vs compaction off, time per launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03za
mkdir -p $O
timeout -k 10 200 python -u tools/park_sweep.py unitree_go2 65536 standing ones 9,10,11,12,13 > $O/go2_65536.json 2> $O/go2_65536.err || exit 10
timeout -k 10 200 python -u tools/park_sweep.py unitree_go2 65536 tumbling bernoulli 10,11,12 > $O/go2_65536_tumb.json 2> $O/go2_65536_tumb.err || exit 11
timeout -k 10 200 python -u tools/park_sweep.py walter_sr 32768 standing ones 12,13,14,15 > $O/walter_32768.json 2> $O/walter_32768.err || exit 12
timeout -k 10 200 python -u tools/park_sweep.py walter_sr 8192 tumbling bernoulli 12,13,14,15 > $O/walter_8192_tumb.json 2> $O/walter_8192_tumb.err || exit 13
timeout -k 10 200 python -u tools/park_sweep.py unitree_go2 8192 standing ones 10,11,12 > $O/go2_8192.json 2> $O/go2_8192.err || exit 14
echo done

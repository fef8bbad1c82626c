# Round-3: setup / IPM kernel time against batch size (tools/setup_scaling.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zd
mkdir -p $O
timeout -k 10 200 python -u tools/setup_scaling.py unitree_go2 256,1024,2048,3072,4096,6144,8192 > $O/go2.jsonl 2> $O/go2.err || exit 10
timeout -k 10 200 python -u tools/setup_scaling.py walter_sr 1024,2048,4096,8192 > $O/walter.jsonl 2> $O/walter.err || exit 11
echo done

# Round-3: refinement rounds settle per env (batch independence) + lockstep compaction:
# bitwise A/B and WaLTER park-iteration sweep, then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03zb
mkdir -p $O
timeout -k 10 200 python -u tools/park_sweep.py walter_sr 8192 tumbling bernoulli 14,15,16,17,18 > $O/walter_8192_tumb.json 2> $O/walter_8192_tumb.err || exit 10
timeout -k 10 200 python -u tools/park_sweep.py walter_sr 32768 standing ones 14,15,16,17 > $O/walter_32768.json 2> $O/walter_32768.err || exit 11
timeout -k 10 200 python -u tools/park_sweep.py unitree_go2 65536 standing ones 12 > $O/go2_65536.json 2> $O/go2_65536.err || exit 12
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 13
echo done

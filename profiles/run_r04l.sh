# Round 4: full GPU suite + smoke after the wheel-dual QR / park-guard changes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc $?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 10
echo smoke ok

# Round 5: kernel trace of the 2,048-env tumbling wheel census batch (cold solves with duals).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/${WT_OUT:-r05wt}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 tools/wheel_census.py 2048 91 tumbling bernoulli 1 '{}' --brief > $O/census.jsonl 2> $O/err.txt || exit 31
echo done

# Round 5: the fix-up pass with a fixed fraction to the boundary (0.99) -- the census envs that
# stalled, A/B (bitwise flags) against the previous library, GPU suite (golden fixtures
# go2_stalled / walter_stalled included).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05af
mkdir -p $O
AB_CHECK=1 AB_ROUNDS=3 AB_CONFIGS="unitree_go2:4096,walter_sr:4096,walter_sr:65536" timeout -k 10 400 python tools/ab_time.py operational-space-control_amd/lib/ab_old/libosc_batch.so operational-space-control_amd/lib/libosc_batch.so > $O/ab.jsonl 2>&1 || exit 31
for c in "unitree_go2 21 1.0" "unitree_go2 22 0.5" "unitree_go2 24 1.0" "walter_sr 23 1.5" "walter_sr 24 1.5" "walter_sr 27 1.0"; do
  set -- $c
  timeout -k 10 120 python tools/status_diag.py $1 65536 $2 $3 >> $O/status.jsonl 2>> $O/status.err || exit 32
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 33
echo done

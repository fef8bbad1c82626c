# Round 5: the interior point's active-set stop (osc_model_tuning.as_stop_mu) -- kernel time,
# statuses, iterations and torque difference against the stop off, Go2 batches.  (An experiment
# build: the knob was measured slower everywhere and not kept -- DESIGN.md §6.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05t
mkdir -p $O
export OSC_AB_ROUNDS=3
V='{"as_stop_mu": 0.0} {"as_stop_mu": 1e-4} {"as_stop_mu": 1e-3} {"as_stop_mu": 1e-2}'
run() { timeout -k 10 240 python tools/tune_ab.py "$@" >> $O/asstop_ab.jsonl 2>> $O/asstop_ab.err; }
run unitree_go2 4096 standing ones '{"as_stop_mu": 0.0}' '{"as_stop_mu": 1e-4}' '{"as_stop_mu": 1e-3}' '{"as_stop_mu": 1e-2}' || exit 31
run unitree_go2 8192 tumbling bernoulli '{"as_stop_mu": 0.0}' '{"as_stop_mu": 1e-4}' '{"as_stop_mu": 1e-3}' '{"as_stop_mu": 1e-2}' || exit 32
run unitree_go2 65536 standing ones '{"as_stop_mu": 0.0}' '{"as_stop_mu": 1e-4}' '{"as_stop_mu": 1e-3}' '{"as_stop_mu": 1e-2}' || exit 33
run unitree_go2 4096 qpos0.5 ones '{"as_stop_mu": 0.0}' '{"as_stop_mu": 1e-4}' '{"as_stop_mu": 1e-3}' '{"as_stop_mu": 1e-2}' || exit 34
run unitree_go2 65536 qpos1.0 ones '{"as_stop_mu": 0.0}' '{"as_stop_mu": 1e-4}' '{"as_stop_mu": 1e-3}' '{"as_stop_mu": 1e-2}' || exit 35
echo done

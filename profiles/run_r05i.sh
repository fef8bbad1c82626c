# Round 5: interior-point stop (eps_mu) A/B now that the refinement's rounds change one row at a
# time -- kernel time, statuses, iterations and torque difference per setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/r05i
mkdir -p $O
export OSC_AB_ROUNDS=3
G='{"eps_mu": 1e-6} {"eps_mu": 1e-5} {"eps_mu": 1e-4} {"eps_mu": 3e-4}'
W='{"eps_mu": 1e-8} {"eps_mu": 1e-7} {"eps_mu": 1e-6} {"eps_mu": 1e-5}'
run() { timeout -k 10 200 python tools/tune_ab.py "$@" >> $O/eps_ab.jsonl 2>> $O/eps_ab.err; }
run unitree_go2 4096 standing ones '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' '{"eps_mu": 1e-4}' '{"eps_mu": 3e-4}' || exit 31
run unitree_go2 65536 standing ones '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' '{"eps_mu": 1e-4}' '{"eps_mu": 3e-4}' || exit 32
run unitree_go2 8192 tumbling bernoulli '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' '{"eps_mu": 1e-4}' '{"eps_mu": 3e-4}' || exit 33
run unitree_go2 65536 qpos1.0 ones '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' '{"eps_mu": 1e-4}' '{"eps_mu": 3e-4}' || exit 34
run walter_sr 4096 standing ones '{"eps_mu": 1e-8}' '{"eps_mu": 1e-7}' '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' || exit 35
run walter_sr 8192 tumbling bernoulli '{"eps_mu": 1e-8}' '{"eps_mu": 1e-7}' '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' || exit 36
run walter_sr 65536 qpos1.0 ones '{"eps_mu": 1e-8}' '{"eps_mu": 1e-7}' '{"eps_mu": 1e-6}' '{"eps_mu": 1e-5}' || exit 37
echo done

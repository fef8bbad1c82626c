# Round 4: interleaved (5 rounds, median) sweep of the early stop and refinement steps -- WaLTER
# standing / joint-state / tumbling, Go2 standing / joint-state
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
export OSC_AB_ROUNDS=5
O=gpurun_out/r04v
mkdir -p $O
W="{} {\"eps_mu\":1e-7} {\"eps_mu\":1e-6} {\"refine_steps\":1} {\"refine_steps\":3} {\"eps_mu\":1e-7,\"refine_steps\":1}"
timeout -k 10 300 python tools/tune_ab.py walter_sr 4096 standing ones $W > $O/walter_4096.jsonl 2>&1 || exit 30
timeout -k 10 300 python tools/tune_ab.py walter_sr 4096 qpos0.5 ones $W > $O/walter_4096_qpos.jsonl 2>&1 || exit 31
timeout -k 10 300 python tools/tune_ab.py walter_sr 8192 tumbling bernoulli $W > $O/walter_8192_tumbling.jsonl 2>&1 || exit 32
G="{} {\"eps_mu\":1e-5} {\"refine_steps\":1} {\"refine_steps\":3} {\"eps_mu\":1e-5,\"refine_steps\":1}"
timeout -k 10 300 python tools/tune_ab.py unitree_go2 4096 standing ones $G > $O/go2_4096.jsonl 2>&1 || exit 33
timeout -k 10 300 python tools/tune_ab.py unitree_go2 4096 qpos0.5 ones $G > $O/go2_4096_qpos.jsonl 2>&1 || exit 34
echo done

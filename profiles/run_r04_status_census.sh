# Round 4: status census of the default solver at 65,536 envs -- Go2 and WaLTER, synthetic
# standing / tumbling and joint states (GPU kinematics, joint ranges 0.5 and 1.0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04_status2
mkdir -p $O
for rb in unitree_go2 walter_sr; do
  for sc in "standing ones" "tumbling bernoulli" "qpos0.5 ones" "qpos1.0 bernoulli"; do
    timeout -k 10 200 python tools/tune_ab.py $rb 65536 $sc '{}' >> $O/status_65536.jsonl 2>> $O/err.txt || exit 11
  done
done
echo done

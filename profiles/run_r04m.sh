# Round 4: wheel-row interior point -- MAX_ITER census under tuning variants (re-centre iteration,
# stop tolerances), seeds 86 / 91, 2,048 tumbling envs each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
for sd in 86 91; do
  for t in '{}' '{"restart_iter": 12}' '{"restart_iter": 18}' '{"restart_iter": 40}' '{"restart_iter": 1000}' '{"wheel_tol": 1e-5}' '{"eps_mu": 1e-10}' '{"refine_steps": 20}' '{"max_iter": 100}' '{"max_iter": 200}'; do
    timeout -k 10 120 python tools/wheel_census.py 2048 $sd tumbling bernoulli 1 "$t" --brief >> $O/sweep_$sd.jsonl 2>> $O/sweep.err || exit 11
  done
done
echo wheel sweep done

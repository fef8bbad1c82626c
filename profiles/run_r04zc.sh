# Round 4: wheel-row refinement steps per round (tuning refine_steps; default 12 from when the
# rows' multipliers came from the refinement -- they now come from stationarity): statuses,
# certificate and time per 2,048-env solve
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r04zc
mkdir -p $O
for sd in 86 91 93; do
  for t in '{}' '{"refine_steps": 8}' '{"refine_steps": 6}' '{"refine_steps": 4}' '{"refine_steps": 3}'; do
    timeout -k 10 120 python tools/wheel_census.py 2048 $sd tumbling bernoulli 1 "$t" --brief >> $O/sweep_$sd.jsonl 2>> $O/sweep.err || exit 11
  done
done
for t in '{}' '{"refine_steps": 6}' '{"refine_steps": 4}'; do
  timeout -k 10 120 python tools/wheel_census.py 2048 81 standing ones 1 "$t" --brief >> $O/sweep_81.jsonl 2>> $O/sweep.err || exit 12
  timeout -k 10 200 python tools/wheel_census.py 2048 97 tumbling bernoulli 3 "$t" --brief >> $O/sweep_97w.jsonl 2>> $O/sweep.err || exit 13
done
echo done

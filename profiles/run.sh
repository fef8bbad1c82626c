# One GPU session on the box: the named steps in order, each under its own time limit, stopping
# at the first failure (its exit code names the step).  Replaces the per-experiment run_r0*.sh
# scripts of rounds 1-5.
#
#   gpurun -- 'bash profiles/run.sh <out> <step> [<step> ...]'
#
# Steps (output under gpurun_out/<out>/):
#   tests[=<pytest -k expr>]   GPU suite (or a selection) -> gpu_tests.log
#   file=<tests/file.py>       one GPU test file          -> gpu_<file>.log
#   smoke                      __graft_entry__.smoke()    -> smoke.log
#   trace                      bench --steps 20 --warmup 5 under rocprofv3 --kernel-trace --stats
#                              -> trace20x5/, bench_20x5.json
#   bench                      default bench (200 + 100)  -> bench_default.json
#   bench20                    the driver's bench command -> bench_20x5_plain.json
#   configs                    configs[2], [3], Go2 8,192 / 65,536, mixed as bench lines
#   pmc=<robot>:<nenv>         FETCH_SIZE and WRITE_SIZE passes (separate runs) of one batch
#   sq=<robot>:<nenv>          SQ issue counters of one batch
#   pmchbm                     FETCH / WRITE passes of bench --hbm-only (roofline.hbm_inputs)
#   ab=<old.so>                tools/ab_time.py <old.so> vs the in-tree library (AB_* env)
#   rocab=<lib.so>:<robot>:<nenv>  one library's cold solves under rocprofv3 --kernel-trace --stats
#                              -> rocab_<n>/ (per-kernel durations of an A/B side)
#   hostfed                    bench's host_fed object alone (4,096 and 8,192 envs)
#   rehearse                   bench.py --gpus 2 on this one GPU (ranks over gloo), host_fed on
#   py=<script args>           python <script args>       -> py_<n>.log
#   exe=<program args>         a built tool (tools/bin/...) -> exe_<n>.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
B="--no-cpu --no-front-end --no-single-env --no-north-star --no-mixed --no-warm --hbm-batches 0 --host-fed-envs="
n=0
for step in "$@"; do
  n=$((n + 1))
  key=${step%%=*}
  val=${step#*=}
  echo "[run.sh] step $n: $step"
  case "$key" in
    tests)
      sel=()
      [ "$val" != "tests" ] && sel=(-k "$val")
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread "${sel[@]}" > "$O/gpu_tests.log" 2>&1 || exit $((30 + n)) ;;
    file)
      timeout -k 10 600 python -u -m pytest "$val" -m gpu -v -s --timeout 300 --timeout-method thread > "$O/gpu_$(basename "$val" .py).log" 2>&1 || exit $((30 + n)) ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $((30 + n)) ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/trace20x5" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > "$O/bench_20x5.json" 2> "$O/bench_20x5.err" || exit $((30 + n)) ;;
    bench)
      timeout -k 10 400 python bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit $((30 + n)) ;;
    bench20)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_20x5_plain.json" 2> "$O/bench_20x5_plain.err" || exit $((30 + n)) ;;
    configs)
      timeout -k 10 300 python bench.py --robot walter_sr $B > "$O/bench_walter_4096.json" 2>> "$O/other.err" &&
      timeout -k 10 300 python bench.py --robot walter_sr --nenv-per-gpu 8192 --scenario tumbling --mask bernoulli --mask-redraw 8 $B > "$O/bench_walter_tumbling_8192.json" 2>> "$O/other.err" &&
      timeout -k 10 300 python bench.py --nenv-per-gpu 8192 $B > "$O/bench_go2_8192.json" 2>> "$O/other.err" &&
      timeout -k 10 300 python bench.py --nenv-per-gpu 65536 --steps 50 --warmup 20 $B > "$O/bench_go2_65536.json" 2>> "$O/other.err" &&
      timeout -k 10 300 python bench.py --robot mixed $B > "$O/bench_mixed.json" 2>> "$O/other.err" || exit $((30 + n)) ;;
    pmc)
      # -> $O/prof_<robot>_<nenv>/{trace,pmc_fetch,pmc_write}: tools/pmc_summary.py's input layout
      robot=${val%%:*}; nenv=${val#*:}; P="$R/$O/prof_${robot}_${nenv}"
      A="--robot $robot --nenv-per-gpu $nenv --steps 10 --warmup 3 $B"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- python3 bench.py $A > /dev/null 2>> "$O/pmc.err" &&
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$P/pmc_fetch" -o run --output-format csv -- python3 bench.py $A > /dev/null 2>> "$O/pmc.err" &&
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$P/pmc_write" -o run --output-format csv -- python3 bench.py $A > /dev/null 2>> "$O/pmc.err" || exit $((30 + n)) ;;
    pmchbm)
      P="$R/$O/prof_hbm"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- python3 bench.py --hbm-only --steps 20 --warmup 5 > /dev/null 2>> "$O/pmc.err" &&
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$P/pmc_fetch" -o run --output-format csv -- python3 bench.py --hbm-only --steps 20 --warmup 5 > /dev/null 2>> "$O/pmc.err" &&
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$P/pmc_write" -o run --output-format csv -- python3 bench.py --hbm-only --steps 20 --warmup 5 > /dev/null 2>> "$O/pmc.err" || exit $((30 + n)) ;;
    sq)
      robot=${val%%:*}; nenv=${val#*:}; P="$R/$O/prof_${robot}_${nenv}"
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_ANY -d "$P/pmc_cyc" -o run --output-format csv -- python3 bench.py --robot "$robot" --nenv-per-gpu "$nenv" --steps 10 --warmup 3 $B > /dev/null 2>> "$O/sq.err" || exit $((30 + n)) ;;
    ab)
      timeout -k 10 500 python tools/ab_time.py "$val" operational-space-control_amd/lib/libosc_batch.so > "$O/ab_$n.jsonl" 2>&1 || exit $((30 + n)) ;;
    rocab)
      lib=${val%%:*}; rest=${val#*:}
      AB_CONFIGS="$rest" AB_ONLY="$rest" AB_ROUNDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/rocab_$n" -o run --output-format csv -- python3 tools/ab_time.py "$lib" > "$O/rocab_$n.jsonl" 2>&1 || exit $((30 + n)) ;;
    hostfed)
      timeout -k 10 300 python bench.py --no-cpu --no-front-end --no-single-env --no-north-star --no-mixed --hbm-batches 0 --no-warm > "$O/bench_hostfed.json" 2> "$O/bench_hostfed.err" || exit $((30 + n)) ;;
    rehearse)
      OSC_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu --no-warm --no-front-end --no-single-env > "$O/rehearse_2ranks.json" 2> "$O/rehearse_2ranks.err" || exit $((30 + n)) ;;
    py)
      # shellcheck disable=SC2086
      timeout -k 10 600 python -u $val > "$O/py_$n.log" 2>&1 || exit $((30 + n)) ;;
    exe)
      # shellcheck disable=SC2086
      timeout -k 10 120 $val > "$O/exe_$n.log" 2>&1 || exit $((30 + n)) ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo done

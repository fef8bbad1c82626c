# Round-3: GPU kinematics tests (slide / ball / multi-joint bodies), A/B of the pre-scaled LDL
# factor (multiply-free triangular solves) against the committed kernel, then the Go2 traces +
# HBM PMC passes (profiles/run_r03t_prof.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kinematics.py -x -v --timeout 120 --timeout-method thread > $O/kin_tests.log 2>&1 || exit 11
A=operational-space-control_amd/lib/ablate
timeout -k 10 300 python tools/ab_time.py $A/base/libosc_batch.so $A/pre/libosc_batch.so $A/base/libosc_batch.so $A/pre/libosc_batch.so > $O/ab_pre.txt 2>&1 || exit 12
bash profiles/run_r03t_prof.sh > $O/prof.out 2>&1 || exit 13
echo done

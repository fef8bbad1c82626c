# A/B of library builds: GPU tests on the in-tree build, kernel timing vs the given builds,
# per-kernel rocprof times and setup-phase stamps of the in-tree build (Go2 4,096)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ty_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/ty_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_time.py "$@" > gpurun_out/ty_ab.txt 2>&1 || exit $?
cat gpurun_out/ty_ab.txt
AB_ONLY=unitree_go2:4096 bash tools/prof_libs.sh operational-space-control_amd/lib/libosc_batch.so > gpurun_out/ty_prof.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/setup_stamps.py 4096 > gpurun_out/ty_stamps.txt 2>&1 || exit $?
cat gpurun_out/ty_stamps.txt

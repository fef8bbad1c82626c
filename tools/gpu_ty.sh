mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ty_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_time.py operational-space-control_amd/lib/ab/head.so operational-space-control_amd/lib/ab/ty.so > gpurun_out/ty_ab.txt 2>&1
echo "ab rc=$?"
tail -5 gpurun_out/ty_tests.log; cat gpurun_out/ty_ab.txt

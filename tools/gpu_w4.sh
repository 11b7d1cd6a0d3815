set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_w4.py tests/test_gpu_wgrad_c5.py tests/test_gpu_glds.py -x -v --timeout 200 --timeout-method thread > gpurun_out/w4_t.log 2>&1; rc=$?
tail -40 gpurun_out/w4_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_w4.py > gpurun_out/w4_b.log 2>&1; rc=$?
cat gpurun_out/w4_b.log
exit $rc

mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_glds.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_glds.log 2>&1; rc=$?
tail -25 gpurun_out/t_glds.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_check.sh

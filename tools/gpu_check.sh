# quick GPU check of the touched kernels: their tests, the global_feat micro-benchmark, one bench line
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${CHECK_TESTS:-tests/test_gpu_glds.py tests/test_gpu_parity.py} > gpurun_out/t2.log 2>&1
timeout -k 10 300 python -u tools/bench_glds.py > gpurun_out/micro2.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err

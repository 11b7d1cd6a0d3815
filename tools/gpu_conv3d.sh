set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_conv3d.py > gpurun_out/t_conv3d.log 2>&1
timeout -k 10 300 python -u tools/bench_conv3d.py 4 64 64 > gpurun_out/bench_conv3d.txt 2>&1

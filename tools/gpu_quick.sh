timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_c5.py -q --timeout 120 --timeout-method thread > gpurun_out/wc5.log 2>&1; tail -3 gpurun_out/wc5.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q --timeout 150 --timeout-method thread > gpurun_out/par.log 2>&1; tail -2 gpurun_out/par.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err; tail -1 gpurun_out/b.json | cut -c 250-330; grep -A14 per-kernel gpurun_out/b.err

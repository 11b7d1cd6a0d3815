#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_glds.py tests/test_gpu_parity.py tests/test_gpu_gram.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_glds.log 2>&1 || { tail -30 gpurun_out/t_glds.log; exit 1; }
tail -2 gpurun_out/t_glds.log
timeout -k 10 200 python tools/bench_glds.py 2>/dev/null | grep dgrad
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2>gpurun_out/bench.err && cat gpurun_out/bench.json | cut -c1-200

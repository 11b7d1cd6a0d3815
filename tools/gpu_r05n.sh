#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_prefetch_draw.py tests/test_gpu_seg12.py > gpurun_out/pf.log 2>&1 || { tail -30 gpurun_out/pf.log; exit 1; }
tail -1 gpurun_out/pf.log
ARGS_B="--no-prefetch-draw" bash tools/ab_bench.sh

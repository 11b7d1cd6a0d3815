#!/bin/bash
# fwd_s12 one-barrier loop: parity, kernel micro-bench (in-tree vs variants vs two passes), step A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg12.py > gpurun_out/s12.log 2>&1
timeout -k 10 120 python -u tools/bench_s12.py --two-pass
for v in s12_nosb; do PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python -u tools/bench_s12.py; done
timeout -k 10 120 python -u tools/bench_s12.py
echo "== A/B: fused seg12 (a) vs two passes (b)"
ARGS_B="--no-fused-seg12" bash tools/ab_bench.sh

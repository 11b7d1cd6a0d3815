#!/bin/bash
set -e
for i in 1 2; do
timeout -k 10 120 python -u tools/bench_s12.py
PCS_LIB=abtest/s12_pair/libpcs.so timeout -k 10 120 python -u tools/bench_s12.py
done
PCS_LIB=abtest/s12_pair/libpcs.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg12.py 2>&1 | tail -2

#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_glds.py > gpurun_out/glds.log 2>&1 || { tail -30 gpurun_out/glds.log; exit 1; }
tail -1 gpurun_out/glds.log
VARS="gf_prev" bash tools/ab_gf.sh 2>&1 | grep -v amdgpu | grep -A2 "round" | grep "fwd\|==" 
VAR=gf_prev bash tools/ab_lib_step.sh 2>&1 | grep -v "dgrad:"

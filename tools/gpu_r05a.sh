#!/bin/bash
# round-5 GPU batch: fused seg12 parity, step A/Bs (fused seg12, draw placement), kernel profile
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg12.py > gpurun_out/s12.log 2>&1
echo "== A/B: fused seg12 (a) vs two passes (b)"
ARGS_B="--no-fused-seg12" bash tools/ab_bench.sh
echo "== A/B: draw beside the Gram (a) vs at the start (b)"
ARGS_B="--draw-at-start" bash tools/ab_bench.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s12 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_s12.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_draw -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --draw-at-start > gpurun_out/prof_draw.log 2>&1

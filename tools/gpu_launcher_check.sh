#!/bin/bash
# bench.py --gpus on a one-GPU box (run from the repo root): the default line, a 2-rank gloo
# rehearsal started by bench.py itself (no external launcher), and --gpus 8 refused (rc 2).
set -e
TAG=${1:-r03a}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
PCS_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --grid 64 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-kernel-timing > gpurun_out/dp2_gloo_$TAG.json 2> gpurun_out/dp2_gloo_$TAG.err
cat gpurun_out/dp2_gloo_$TAG.json
set +e
timeout -k 10 120 python -u bench.py --gpus 8 > gpurun_out/gpus8_$TAG.out 2>&1
rc=$?
set -e
echo "bench.py --gpus 8 on a 1-GPU box: rc=$rc"; tail -2 gpurun_out/gpus8_$TAG.out
[ $rc -eq 2 ]

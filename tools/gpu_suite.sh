#!/bin/bash
# Full GPU suite, smoke() and the default bench line at HEAD (run from the repo root on the box)
set -e
TAG=${1:-r02c}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rP --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json

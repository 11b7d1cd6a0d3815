#!/bin/bash
# Round-4 evidence at one build (repo root, GPU box): the GPU suite, smoke(), the default bench
# line with its per-kernel table, then tools/profile_round.sh (trace + PMC passes) for it.
# Usage: tools/evidence_r04.sh <tag> [bench.py args]
set -e
TAG=${1:-r04}
shift || true
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -v -rP --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_${TAG}_kernels.txt
cat gpurun_out/bench_$TAG.json
bash tools/profile_round.sh $TAG "$@" > gpurun_out/profile_$TAG.log 2>&1
head -14 profiles/rocprof_$TAG.md

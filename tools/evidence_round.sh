#!/bin/bash
# Round evidence on the GPU box (run from the repo root): the full GPU suite, smoke(), then
# tools/profile_round.sh for the bf16 and fp8 bench lines.  Usage: tools/evidence_round.sh <tag>
set -e
TAG=${1:-r02b}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -1 gpurun_out/smoke_$TAG.log
tools/profile_round.sh $TAG
tools/profile_round.sh ${TAG}_fp8 --dtype fp8

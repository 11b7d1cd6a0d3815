#!/bin/bash
# Round evidence at one build (repo root, GPU box): GPU suite, smoke, the bf16 bench line with
# its per-kernel table and rocprof/PMC passes, then the fp8 (with profile), fp32 and cfg3 lines.
# Usage: tools/evidence_full.sh <tag>
set -e
TAG=${1:-r05b}
mkdir -p gpurun_out
bash tools/evidence_r04.sh $TAG
timeout -k 10 400 python -u bench.py --dtype fp8 > gpurun_out/bench_fp8_$TAG.json 2> gpurun_out/bench_fp8_${TAG}_kernels.txt
cat gpurun_out/bench_fp8_$TAG.json
bash tools/profile_round.sh ${TAG}_fp8 --dtype fp8 > gpurun_out/profile_${TAG}_fp8.log 2>&1
timeout -k 10 400 python -u bench.py --dtype fp32 --no-cpu-baseline > gpurun_out/bench_fp32_$TAG.json 2> gpurun_out/bench_fp32_${TAG}_kernels.txt
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3_$TAG.json 2> gpurun_out/bench_cfg3_${TAG}_kernels.txt
tail -c 300 gpurun_out/bench_fp32_$TAG.json; tail -c 300 gpurun_out/bench_cfg3_$TAG.json

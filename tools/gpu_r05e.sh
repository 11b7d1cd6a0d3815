#!/bin/bash
# round-5 evidence: fp8 (cfg5) line with its profile, the fp32 line, cfg3 (ragged) line
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --dtype fp8 > gpurun_out/bench_fp8_r05a.json 2> gpurun_out/bench_fp8_r05a_kernels.txt
cat gpurun_out/bench_fp8_r05a.json
bash tools/profile_round.sh r05a_fp8 --dtype fp8 > gpurun_out/profile_r05a_fp8.log 2>&1
timeout -k 10 400 python -u bench.py --dtype fp32 --no-cpu-baseline > gpurun_out/bench_fp32_r05a.json 2> gpurun_out/bench_fp32_r05a_kernels.txt
cat gpurun_out/bench_fp32_r05a.json
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3_r05a.json 2> gpurun_out/bench_cfg3_r05a_kernels.txt
cat gpurun_out/bench_cfg3_r05a.json

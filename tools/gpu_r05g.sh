#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg12.py 2>&1 | tail -2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_g.log 2>&1
python3 tools/db_kernels.py gpurun_out/prof_g/run_results.db bn_stats_gram wgrad_kernel dgrad_wgrad_s1 fwd_s12

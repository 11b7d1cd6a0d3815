#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/suite_l.log 2>&1 || { tail -40 gpurun_out/suite_l.log; exit 1; }
tail -1 gpurun_out/suite_l.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_l.log 2>&1
python3 tools/db_kernels.py gpurun_out/prof_l/run_results.db fold_h gram_quad

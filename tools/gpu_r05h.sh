#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -rP --timeout 120 --timeout-method thread tests/test_gpu_seg12.py > gpurun_out/s12.log 2>&1 || { tail -30 gpurun_out/s12.log; exit 1; }
grep -E "Gram rel err|passed|failed" gpurun_out/s12.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_h.log 2>&1
python3 tools/db_kernels.py gpurun_out/prof_h/run_results.db "fwd_stream_kernel<64, 64" bn_stats_gram wgrad_kernel reduce_partials
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('step',d['ms_per_step'],d['value'])"

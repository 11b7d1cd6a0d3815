#!/bin/bash
# Routine GPU-box check: the -m gpu suite, then (only if it passed) a bench line (no CPU
# baseline) with the per-kernel table on stderr.  Each step under its own time limit.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/bench.json; tail -40 gpurun_out/bench.err
exit $rc

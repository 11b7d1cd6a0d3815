#!/bin/bash
# Routine GPU-box check: the -m gpu suite, then a bench line (no CPU baseline) with the
# per-kernel table on stderr.  Each step under its own time limit.
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
exit $rc

#!/bin/bash
# fused seg_conv1 backward: unit test, bf16 parity tests, then a bench line (no CPU baseline)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_fused_bwd.py tests/test_gpu_parity.py tests/test_gpu_data.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/t_fused.log 2>&1 || { tail -40 gpurun_out/t_fused.log; exit 1; }
tail -3 gpurun_out/t_fused.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/bench.json; grep -E "seg_conv1|step" gpurun_out/bench.err
exit $rc

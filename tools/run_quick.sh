mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -s -k "big_kernel or bf16_path" --timeout 120 --timeout-method thread > gpurun_out/quick.log 2>&1; rc=$?
grep -E "norm-rel|logits|cos|passed|failed|Error|bf16" gpurun_out/quick.log | head -60
exit $rc

# head variants (abtest/<name>/libpcs.so): tests/test_gpu_head_stream.py each, then alternating timing
set -e
VARS=${VARS:-$(ls abtest)}
for v in $VARS; do
  PCS_LIB=abtest/$v/libpcs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_head_stream.py -q --timeout 120 --timeout-method thread > gpurun_out/head_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/head_$v.log; exit 1; }
  echo "$v: $(tail -n 1 gpurun_out/head_$v.log)"
done
for i in 1 2 3; do for v in $VARS; do echo "== $v $(PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python tools/bench_head.py 20 2>&1 | grep -v amdgpu.ids)"; done; done

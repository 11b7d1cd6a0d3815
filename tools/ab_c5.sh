# same-box A/B of fused_c5.hip builds (abtest/<name>/libpcs.so, tools/build_variants.sh SRC=fused_c5):
# correctness of each build first, then alternating timing (tools/bench_c5.py)
set -e
mkdir -p gpurun_out
VARS=${VARS:-$(ls abtest)}
for v in $VARS; do
  PCS_LIB=abtest/$v/libpcs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_c5_dgrad.py -q -x --timeout 120 --timeout-method thread > gpurun_out/c5_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/c5_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c5_$v.log)"
done
for i in 1 2 3; do for v in $VARS; do echo "== $v"; PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python tools/bench_c5.py 10 2>&1 | grep -v amdgpu.ids; done; done

# same-box A/B of fused_seg4.hip (or fused_bwd.hip) builds (abtest/<name>/libpcs.so, tools/build_variants.sh SRC=fused_seg4):
# the fused-backward tests on each build, then alternating timing (tools/bench_seg.py)
set -e
mkdir -p gpurun_out
VARS=${VARS:-$(ls abtest)}
for v in $VARS; do
  PCS_LIB=abtest/$v/libpcs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_bwd.py -q -x --timeout 120 --timeout-method thread > gpurun_out/s4_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/s4_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/s4_$v.log)"
done
for i in 1 2 3; do for v in $VARS; do echo "== $v"; PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python tools/bench_seg.py 10 2>&1 | grep -v amdgpu.ids; done; done

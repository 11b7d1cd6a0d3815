# same-box A/B of fwd_stream.hip builds (abtest/<name>/libpcs.so, tools/build_variants.sh) on
# conv5's forward (bf16 and fp8 a5 stores): correctness of each build first, then alternating timing
set -e
mkdir -p gpurun_out
VARS=${VARS:-$(ls abtest)}
for v in $VARS; do
  PCS_LIB=abtest/$v/libpcs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fwd_stream.py tests/test_gpu_fp8.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/fs_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/fs_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/fs_$v.log)"
done
for i in 1 2 3; do for v in $VARS; do echo "== $v"; FS_SHAPES=${FS_SHAPES:-conv5} PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python tools/bench_fwd.py 10 2>&1 | grep -v amdgpu.ids; done; done

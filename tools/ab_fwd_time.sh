# timing-only A/B of fwd_stream.hip variants (no correctness: ablation builds compute wrong outputs)
set -e
VARS=${VARS:-$(ls abtest)}
for i in 1 2; do for v in $VARS; do echo "== $v"; PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python tools/bench_fwd.py 10 2>&1 | grep -v amdgpu.ids; done; done

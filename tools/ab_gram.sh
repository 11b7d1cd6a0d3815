# timing A/B of pcs_gram C = 128 builds (abtest/<name>/libpcs.so)
set -e
VARS=${VARS:-$(ls abtest)}
for i in 1 2; do for v in $VARS; do echo "== $v"; PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python tools/bench_gram128.py 20 2>&1 | grep -v amdgpu.ids; done; done

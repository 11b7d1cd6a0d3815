set -e
mkdir -p gpurun_out
for i in 1 2; do for v in ship abl1 abl2 abl3; do echo "== $v"; FS_SHAPES=conv5 PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python tools/bench_fwd.py 10 2>&1 | grep -v amdgpu.ids; done; done

# w4 kernel: parity tests (test_gpu_w4, the LDS-DMA suites beside it), then the cfg2 timing
# of w4 against the 8-wave kernel (tools/bench_w4.py) and the ablation builds listed in ABL_LIST
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_w4.py tests/test_gpu_wgrad_c5.py tests/test_gpu_glds.py -x -v --timeout 200 --timeout-method thread > gpurun_out/w4_t.log 2>&1; rc=$?
tail -5 gpurun_out/w4_t.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/w4_t.log; exit $rc; fi
timeout -k 10 300 python -u tools/bench_w4.py > gpurun_out/w4_b.log 2>&1; rc=$?
cat gpurun_out/w4_b.log
if [ $rc -ne 0 ]; then exit $rc; fi
D=point-cloud-cnn-segmentation_amd/csrc/abl
for n in $ABL_LIST; do
  echo "== W4_ABL=$n"
  PCS_LIB=$D/libpcs_w4abl$n.so W4_ONLY=1 timeout -k 10 120 python -u tools/bench_w4.py 2>&1 | grep -v amdgpu.ids || exit $?
done

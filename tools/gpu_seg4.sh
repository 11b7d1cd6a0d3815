# seg4 (fused_seg4.hip): the fused-backward parity tests, then seg4 vs the 8-wave kernel timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_bwd.py -v --timeout 120 --timeout-method thread > gpurun_out/seg4_t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/seg4_t.log | tail -30; tail -3 gpurun_out/seg4_t.log
if [ $rc -ne 0 ]; then grep -B5 -A30 "Error\b\|assert" gpurun_out/seg4_t.log | head -80; exit $rc; fi
for i in 1 2; do
  echo "== seg4"; timeout -k 10 120 python tools/bench_seg.py 10 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== seg8"; SEG_FLAGS=64 timeout -k 10 120 python tools/bench_seg.py 10 2>&1 | grep -v amdgpu.ids || exit 1
done

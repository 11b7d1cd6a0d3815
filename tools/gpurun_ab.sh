# same-box A/B: tests of the touched kernels, then micro + step benches of this tree and of
# abtest/old (a built copy of the previous commit)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${AB_TESTS:-tests/test_gpu_glds.py tests/test_gpu_parity.py tests/test_gpu_fp8.py tests/test_gpu_fullsize.py} > gpurun_out/t.log 2>&1
if [ -n "$AB_MICRO" ]; then
  timeout -k 10 200 python tools/bench_glds.py > gpurun_out/micro_new.txt 2>&1
  GLDS_FP8=1 timeout -k 10 200 python tools/bench_glds.py >> gpurun_out/micro_new.txt 2>&1
  (cd abtest/old && timeout -k 10 200 python tools/bench_glds.py > ../../gpurun_out/micro_old.txt 2>&1 && GLDS_FP8=1 timeout -k 10 200 python tools/bench_glds.py >> ../../gpurun_out/micro_old.txt 2>&1)
fi
for i in 1 2; do
for d in bf16 fp8; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dtype $d --no-cpu-baseline > gpurun_out/new_$d.$i.json 2>gpurun_out/new_$d.$i.err
(cd abtest/old && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dtype $d --no-cpu-baseline > ../../gpurun_out/old_$d.$i.json 2>../../gpurun_out/old_$d.$i.err)
done; done

set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_glds.py tests/test_gpu_parity.py tests/test_gpu_fp8.py tests/test_gpu_fullsize.py tests/test_gpu_gram.py > gpurun_out/t.log 2>&1
for i in 1 2; do
for d in bf16 fp8; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dtype $d --no-cpu-baseline > gpurun_out/new_$d.$i.json 2>gpurun_out/new_$d.err
(cd abtest/old && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dtype $d --no-cpu-baseline > ../../gpurun_out/old_$d.$i.json 2>../../gpurun_out/old_$d.err)
done; done

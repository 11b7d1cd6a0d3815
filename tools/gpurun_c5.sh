set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_parity.py > gpurun_out/t.log 2>&1
timeout -k 10 120 python tools/bench_conv5.py > gpurun_out/c5_new.txt 2>&1
(cd abtest/old && timeout -k 10 120 python tools/bench_conv5.py > ../../gpurun_out/c5_old.txt 2>&1)
timeout -k 10 120 python tools/bench_conv5.py >> gpurun_out/c5_new.txt 2>&1
for i in 1 2; do for d in fp8; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dtype $d --no-cpu-baseline > gpurun_out/new_$d.$i.json 2>gpurun_out/new_$d.$i.err
(cd abtest/old && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dtype $d --no-cpu-baseline > ../../gpurun_out/old_$d.$i.json 2>../../gpurun_out/old_$d.$i.err)
done; done

# extra bench lines at HEAD on the GPU box (run from the repo root): fp8 (cfg5), fp32 (parity
# dtype), cfg3 (occupied-only), the Conv3d kernels at 4 x 128^3 x 64 ch and at the 32 -> 64
# channel first U-Net level
set -e
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 300 python -u bench.py --dtype fp8 --no-cpu-baseline > gpurun_out/bench_fp8_$TAG.json 2> gpurun_out/bench_fp8_$TAG.err
tail -1 gpurun_out/bench_fp8_$TAG.json | cut -c1-400
timeout -k 10 400 python -u bench.py --dtype fp32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_fp32_$TAG.json 2> gpurun_out/bench_fp32_$TAG.err
tail -1 gpurun_out/bench_fp32_$TAG.json | cut -c1-400
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3_$TAG.json 2> gpurun_out/bench_cfg3_$TAG.err
tail -1 gpurun_out/bench_cfg3_$TAG.json | cut -c1-400
timeout -k 10 300 python -u tools/bench_conv3d.py 4 128 64 > gpurun_out/bench_conv3d_128_$TAG.txt 2>&1
timeout -k 10 300 python -u tools/bench_conv3d.py 4 128 32 > gpurun_out/bench_conv3d_128c32_$TAG.txt 2>&1
grep -v amdgpu.ids gpurun_out/bench_conv3d_128_$TAG.txt

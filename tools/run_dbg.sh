mkdir -p gpurun_out
for f in 2 1 0; do
PCS_FLAGS=$f timeout -k 10 120 python -u tools/gpu_debug.py train_c2 bf16 > gpurun_out/dbg_bf16_$f.log 2>&1 || exit 1
echo "== flags $f"; grep -E "bn_seg2|seg_conv2.weight|bn1.weight|global_feat.weight|bn5.weight|conv5.weight" gpurun_out/dbg_bf16_$f.log
done

#!/bin/bash
set -e
mkdir -p gpurun_out
PCS_LIB=abtest/seg4_vform/libpcs.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_bwd.py > gpurun_out/fb.log 2>&1 || { tail -30 gpurun_out/fb.log; exit 1; }
tail -1 gpurun_out/fb.log
VAR=seg4_vform bash tools/ab_lib_step.sh 2>&1 | grep -v "global_feat"
grep "seg_conv2\|seg_conv3" gpurun_out/abl_head.1.err gpurun_out/abl_seg4_vform.1.err

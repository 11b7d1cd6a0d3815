#!/bin/bash
# Counters of the seg_conv2 / seg_conv3 fused backward kernels (fused_seg4.hip and, with
# SEG_FLAGS=64, fused_seg.hip) on tools/bench_seg.py; one rocprofv3 --pmc pass per group.
set -e
OUT=gpurun_out/pmc_seg${SEG_FLAGS:-0}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$1 -o run -- python3 tools/bench_seg.py 3 > $OUT/$1.log 2>&1; }
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
run SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA
run GRBM_GUI_ACTIVE GRBM_COUNT
run FETCH_SIZE
run WRITE_SIZE
PMC_FILTER=seg python3 tools/pmc_w4.py $OUT

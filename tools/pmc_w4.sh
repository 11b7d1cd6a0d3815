#!/bin/bash
# Counters of the global_feat GEMM kernels (w4 and the 8-wave glds8) on tools/bench_w4.py:
# one rocprofv3 --pmc pass per counter group, each under its own limit; tools/pmc_w4.py
# prints per-kernel averages (clock, MFMA busy, instruction mix, wave states, LDS, HBM).
set -e
OUT=gpurun_out/pmc_w4
mkdir -p $OUT
export TMPDIR=/tmp W4_ROUNDS=1
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$1 -o run -- python3 tools/bench_w4.py > $OUT/$1.log 2>&1; }
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
run SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA
run GRBM_GUI_ACTIVE GRBM_COUNT
run FETCH_SIZE
run WRITE_SIZE
python3 tools/pmc_w4.py $OUT

#!/bin/bash
# Per-variant HBM traffic and clock of the global_feat GEMMs (tools/bench_glds.py, bf16):
# FETCH_SIZE and GRBM passes, each its own run; tools/pmc_glds_variants.py summarises.
set -e
OUT=gpurun_out/pmc_glds
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/bench_glds.py > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/grbm -o run -- python3 tools/bench_glds.py > $OUT/grbm.log 2>&1

#!/bin/bash
# Collects the rocprofv3 evidence for one round on the GPU box (run from the repo root):
#   1) --kernel-trace --stats                     (per-kernel durations)
#   2) --pmc FETCH_SIZE                           (own pass; 3 TCC slots)
#   3) --pmc WRITE_SIZE                           (own pass; 2 TCC slots)
#   4) --pmc 8 SQ counters (MFMA busy, VALU / MFMA instructions, wave states)
#   5) --pmc GRBM_GUI_ACTIVE GRBM_COUNT          (GPU-active cycles per launch)
# each under its own time limit, then summarises into profiles/ via tools/summarize_profile.py.
# Usage: tools/profile_round.sh r02 [bench.py args ...]   (default: the cfg2 bench line)
set -e
TAG=${1:-r02}
shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/grbm -o run -- python3 bench.py $ARGS > $OUT/grbm.log 2>&1
python3 tools/summarize_profile.py $OUT $TAG $ARGS

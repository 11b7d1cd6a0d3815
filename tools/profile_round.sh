#!/bin/bash
# Collects the rocprofv3 evidence for one round on the GPU box (run from the repo root):
#   1) --kernel-trace --stats      (per-kernel durations)
#   2) --pmc FETCH_SIZE            (own pass; TCC slots)
#   3) --pmc WRITE_SIZE            (own pass)
# then summarises into profiles/ via tools/summarize_profile.py.  Usage:
#   tools/profile_round.sh r01
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/summarize_profile.py $OUT $TAG

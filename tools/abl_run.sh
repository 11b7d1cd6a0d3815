#!/bin/bash
# GPU side of a timing ablation: tools/bench_glds.py against the shipped build and each
# abtest/abl<v>/libpcs.so variant built by tools/build_abl.sh (same box, alternating)
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 240 python -u tools/bench_glds.py > gpurun_out/abl_base.$rep.txt 2>&1
  for v in "$@"; do
    PCS_LIB=abtest/abl$v/libpcs.so timeout -k 10 240 python -u tools/bench_glds.py > gpurun_out/abl_$v.$rep.txt 2>&1
  done
done

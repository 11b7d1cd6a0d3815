#!/bin/bash
# A/B two library builds on one box: tools/ab.sh libA.so libB.so [rounds] [bench args...]
# Alternates A and B bench runs; prints value and ms/step for each.
A=$1; B=$2; R=${3:-2}; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for L in $A $B; do
    PCS_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --steps 12 "$@" > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$L', d['value'], d['ms_per_step'])"
  done
done

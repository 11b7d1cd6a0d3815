#!/bin/bash
# A/B: ab/libpcs_old.so (HEAD) vs the in-tree build, alternating, 3 rounds
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export PCS_LIB=$PWD/ab/libpcs_old.so; else unset PCS_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v',d['value'],d['ms_per_step'])"
  done
done

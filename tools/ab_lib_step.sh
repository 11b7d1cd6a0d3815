#!/bin/bash
# same-box step A/B of the in-tree build against abtest/<VAR>/libpcs.so (timing only; only builds
# whose outputs stay valid indices -- a variant that skips the pool epilogue faults the step),
# alternating processes, three rounds:  VAR="name [name ...]" [GREP=kernel-rows] bash tools/ab_lib_step.sh
set -e
for i in 1 2 3; do
  for v in head $VAR; do
    if [ $v = head ]; then unset PCS_LIB; else export PCS_LIB=abtest/$v/libpcs.so; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/abl_$v.$i.json 2> gpurun_out/abl_$v.$i.err
    echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/abl_$v.$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
    grep "${GREP:-fwd:global_feat\|dgrad:global_feat}" gpurun_out/abl_$v.$i.err | head -4 || true
  done
done

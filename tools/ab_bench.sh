#!/bin/bash
# same-box A/B of the default bench line against bench.py with extra arguments (ARGS_B),
# alternating processes, three rounds:  ARGS_B="--no-fused-seg12" bash tools/ab_bench.sh
set -e
for i in 1 2 3; do
  for v in a b; do
    if [ $v = a ]; then extra=""; else extra="$ARGS_B"; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS $extra > gpurun_out/abb_$v.$i.json 2> gpurun_out/abb_$v.$i.err
    echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/abb_$v.$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done

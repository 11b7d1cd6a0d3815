#!/bin/bash
# GPU side: tools/bench_glds.py and bench.py for the shipped build and each abtest/<name>/libpcs.so
# variant (tools/build_variants.sh), alternating, two rounds (MICRO=0 skips bench_glds)
set -e
mkdir -p gpurun_out
run() {   # run <name> <lib or empty>
  if [ -n "$2" ]; then export PCS_LIB=$2; else unset PCS_LIB; fi
  [ "${MICRO:-1}" = 0 ] || timeout -k 10 240 python -u tools/bench_glds.py > gpurun_out/var_$1.$rep.micro.txt 2>&1
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/var_$1.$rep.json 2> gpurun_out/var_$1.$rep.err
}
for rep in 1 2; do
  run base ""
  for v in "$@"; do run $v abtest/$v/libpcs.so; done
done

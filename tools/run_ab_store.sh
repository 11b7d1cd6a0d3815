#!/bin/bash
for v in default nostore; do
  if [ $v = default ]; then unset PCS_LIB; else export PCS_LIB=$PWD/gpurun_libs/$v/libpcs.so; fi
  echo "== $v"; timeout -k 10 200 python tools/bench_glds.py 2>/dev/null | grep "dgrad" || exit 1
done

#!/bin/bash
# same-box A/B of global_feat's GEMMs: the shipped build against abtest/<name>/libpcs.so builds,
# alternating processes, three rounds:  VARS="v1 v2" bash tools/ab_gf.sh
set -e
for i in 1 2 3; do
  for v in head $VARS; do
    if [ $v = head ]; then unset PCS_LIB; else export PCS_LIB=abtest/$v/libpcs.so; fi
    echo "== $v round $i"
    timeout -k 10 120 python -u tools/bench_gf.py
  done
done

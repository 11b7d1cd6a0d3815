#!/bin/bash
# fwd_s12 ablations (timing only)
set -e
timeout -k 10 120 python -u tools/bench_s12.py
for v in s12_nostats s12_nomask s12_nox s12_nos2 s12_nosb; do PCS_LIB=abtest/$v/libpcs.so timeout -k 10 120 python -u tools/bench_s12.py; done
timeout -k 10 120 python -u tools/bench_s12.py

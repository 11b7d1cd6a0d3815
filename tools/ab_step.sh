# same-box step-time A/B: the shipped build against abtest/<name>/libpcs.so builds, alternating
#   VARS="r03h" bash tools/ab_step.sh
set -e
for i in 1 2 3; do
  for v in head $VARS; do
    if [ $v = head ]; then unset PCS_LIB; else export PCS_LIB=abtest/$v/libpcs.so; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/step_$v.$i.json 2> gpurun_out/step_$v.$i.err
    echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/step_$v.$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done

#!/bin/bash
# round-5 evidence (bf16 line) + the draw's step cost
set -e
bash tools/evidence_r04.sh r05a
echo "== A/B: normal (a) vs keep bits drawn once (b, timing only)"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dc_a.$i.json 2>/dev/null
  timeout -k 10 200 python -u tools/draw_cost.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dc_b.$i.json 2>/dev/null
  python3 -c "import json;a=json.loads(open('gpurun_out/dc_a.$i.json').read().strip().splitlines()[-1]);b=json.loads(open('gpurun_out/dc_b.$i.json').read().strip().splitlines()[-1]);print('a',a['ms_per_step'],'b',b['ms_per_step'])"
done

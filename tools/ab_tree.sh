# same-box step A/B of the working tree against an older full tree (abtest/<name>_tree: its own
# engine and libpcs.so), alternating, three passes:  TREE=r03h bash tools/ab_tree.sh
set -e
T=abtest/${TREE:-r03h}_tree
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tree_head.$i.json 2> gpurun_out/tree_head.$i.err
  (cd $T && timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline) > gpurun_out/tree_old.$i.json 2> gpurun_out/tree_old.$i.err
  for v in head old; do echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/tree_$v.$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'], d.get('lib_sha16'))")"; done
done

"""Summarise tools/variants_run.sh output: per variant and round, the step time and the
global_feat kernel times of bench.py's per-kernel table, and the micro-benchmark lines."""
import glob
import json
import os
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
tags = sys.argv[2:] or ["dgrad:global_feat", "fwd:global_feat", "wgrad:global_feat"]
rows = {}
for js in sorted(glob.glob(os.path.join(d, "var_*.json"))):
    m = re.match(r"var_(.+)\.(\d+)\.json", os.path.basename(js))
    name, rep = m.group(1), m.group(2)
    try:
        rec = json.loads(open(js).read().strip().splitlines()[-1])
    except Exception:
        continue
    ks = {}
    for line in open(js[:-5] + ".err"):
        mm = re.match(r"#\s+(\S+)\s+([\d.]+) ms", line)
        if mm:
            ks[mm.group(1)] = float(mm.group(2))
    rows.setdefault(name, []).append((rep, rec["ms_per_step"], [ks.get(t) for t in tags]))
print("| variant | round | step ms | " + " | ".join(tags) + " |")
print("|---|---|---|" + "---|" * len(tags))
for name, rs in rows.items():
    for rep, ms, kk in rs:
        print(f"| {name} | {rep} | {ms:.2f} | " + " | ".join("-" if k is None else f"{k:.3f}" for k in kk) + " |")
for f in sorted(glob.glob(os.path.join(d, "var_*.micro.txt"))):
    print(f"\n{os.path.basename(f)}")
    print("".join(l for l in open(f) if "glds" in l))

"""Summarise a tools/gpurun_ab.sh run: step times and the per-kernel breakdown, new vs old."""
import json
import os
import re

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def kernels(path):
    res = {}
    if os.path.exists(path):
        for line in open(path):
            m = re.match(r"#\s+(\S+)\s+([\d.]+) ms", line)
            if m:
                res[m.group(1)] = float(m.group(2))
    return res


for d in ("bf16", "fp8"):
    for i in (1, 2):
        row = []
        for v in ("new", "old"):
            try:
                row.append(json.load(open(f"{OUT}/{v}_{d}.{i}.json"))["ms_per_step"])
            except (OSError, ValueError, KeyError):
                row.append(float("nan"))
        print(f"{d} run {i}: new {row[0]:.3f} ms  old {row[1]:.3f} ms  diff {row[0] - row[1]:+.3f}")
    kn, ko = kernels(f"{OUT}/new_{d}.1.err"), kernels(f"{OUT}/old_{d}.1.err")
    for k in sorted(set(kn) | set(ko), key=lambda k: -max(kn.get(k, 0), ko.get(k, 0))):
        dn, do = kn.get(k, 0.0), ko.get(k, 0.0)
        if abs(dn - do) > 0.05:
            print(f"   {k:26s} new {dn:7.3f}  old {do:7.3f}  {dn - do:+.3f}")

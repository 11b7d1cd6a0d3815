"""Condense a directory of raw A/B runs (profiles/<dir>/<variant>.<pass>.json plus the per-kernel
breakdown in .err / .kernels.txt) into one SUMMARY.md table: step ms per pass and the five
kernels that moved most, per variant.   python tools/condense_ab.py profiles/ab_r02_head"""
import glob
import json
import os
import re
import sys


def kernels(path):
    res = {}
    if os.path.exists(path):
        for line in open(path):
            m = re.match(r"#\s+(\S+)\s+([\d.]+) ms", line)
            if m:
                res[m.group(1)] = float(m.group(2))
    return res


def main(d):
    runs = {}
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        m = re.match(r"(.+)\.(\d+)\.json$", os.path.basename(f))
        if not m:
            continue
        try:
            line = open(f).read().strip().splitlines()[-1]
            ms = json.loads(line)["ms_per_step"]
        except (OSError, ValueError, KeyError, IndexError):
            continue
        base = f[:-5]
        k = kernels(base + ".kernels.txt") or kernels(base + ".err")
        runs.setdefault(m.group(1), []).append((int(m.group(2)), ms, k))
    if not runs:
        sys.exit(f"no runs in {d}")
    # new_<dtype> / old_<dtype> pairs compare within their dtype; otherwise against base / old
    group = lambda v: v.split("_", 1)[1] if v.startswith(("new_", "old_")) else ""   # noqa: E731
    refs = {}
    for v in runs:
        g = group(v)
        cand = ("old_" + g) if g else next((w for w in runs if w.startswith(("base", "var_base"))), sorted(runs)[0])
        refs[v] = cand if cand in runs else sorted(runs)[0]

    def mean_kernels(v):
        acc = {}
        for _, _, k in runs[v]:
            for n, t in k.items():
                acc.setdefault(n, []).append(t)
        return {n: sum(t) / len(t) for n, t in acc.items()}
    out = [f"# {os.path.basename(d)}: condensed A/B", "",
           "Condensed from the raw per-pass bench lines by tools/condense_ab.py (raw files pruned).", "",
           "| variant | reference | step ms per pass | kernels that moved most against the reference (ms) |",
           "|---|---|---|---|"]
    for v in sorted(runs, key=lambda v: (group(v), v != refs[v], v)):
        ref = refs[v]
        kref = mean_kernels(ref)
        rs = sorted(runs[v])
        steps = " / ".join(f"{ms:.2f}" for _, ms, _ in rs)
        kv = {}
        for _, _, k in rs:
            for n, t in k.items():
                kv.setdefault(n, []).append(t)
        kv = {n: sum(t) / len(t) for n, t in kv.items()}
        moved = sorted(((n, kref.get(n, 0.0), t) for n, t in kv.items()), key=lambda x: -abs(x[2] - x[1]))[:5]
        mv = ", ".join(f"{n} {a:.2f} → {b:.2f}" for n, a, b in moved if abs(b - a) >= 0.02) if v != ref else "—"
        out.append(f"| `{v}` | `{ref}` | {steps} | {mv or '(none ≥ 0.02 ms)'} |")
    extra = [f for f in os.listdir(d) if f.endswith((".patch", ".md", ".txt")) and not f.endswith(".kernels.txt")
             and f != "SUMMARY.md"]
    if extra:
        out += ["", "Kept beside this summary: " + ", ".join(f"`{f}`" for f in sorted(extra))]
    open(os.path.join(d, "SUMMARY.md"), "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1])

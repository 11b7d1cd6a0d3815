"""Summarise a tools/profile_round.sh run into profiles/rocprof_<tag>.md and
profiles/pmc_<tag>.json (per kernel: calls, average duration, HBM bytes per launch).

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming
read, so bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (our kernels stream 16 B per lane).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def find(pattern):
    hits = glob.glob(pattern, recursive=True)
    return hits[0] if hits else None


def short(name):
    """Kernel name without its parameter list and the anonymous-namespace prefix."""
    name = name.strip()
    if name.endswith(")"):
        depth = 0
        for i in range(len(name) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(name[i], 0)
            if depth == 0:
                name = name[:i]
                break
    return name.replace("void ", "").replace("(anonymous namespace)::", "")[:120]


def main():
    out, tag = sys.argv[1], sys.argv[2]
    stats = find(os.path.join(out, "trace", "**", "*kernel_stats.csv"))
    rows = []
    if stats:
        with open(stats) as f:
            for r in csv.DictReader(f):
                rows.append(r)
    counters = defaultdict(lambda: defaultdict(list))
    for which in ("fetch", "write"):
        path = find(os.path.join(out, which, "**", "*counter_collection.csv"))
        if not path:
            continue
        with open(path) as f:
            for r in csv.DictReader(f):
                counters[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    pmc = {}
    for k, d in counters.items():
        fetch = d.get("FETCH_SIZE", [])
        write = d.get("WRITE_SIZE", [])
        nf, nw = len(fetch), len(write)
        ent = {}
        if nf:
            ent["fetch_kib_per_launch"] = sum(fetch) / nf
        if nw:
            ent["write_kib_per_launch"] = sum(write) / nw
        if nf and nw:
            ent["hbm_bytes_per_launch"] = (2 * ent["fetch_kib_per_launch"] + ent["write_kib_per_launch"]) * 1024
        pmc[short(k)] = ent
    os.makedirs("profiles", exist_ok=True)
    with open(f"profiles/pmc_{tag}.json", "w") as f:
        json.dump(pmc, f, indent=1, sort_keys=True)
    lines = [f"# rocprofv3 summary ({tag})", "",
             "Command: `rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py "
             "--steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing` (cfg2: 4 x 128^3 points, bf16), "
             "plus separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes.", "",
             "| kernel | calls | total ms | avg ms | % | HBM GB/launch (2*FETCH+WRITE) |",
             "|---|---|---|---|---|---|"]
    for r in rows:
        name = short(r["Name"])
        ent = pmc.get(name, {})
        gb = ent.get("hbm_bytes_per_launch")
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} | "
                     f"{gb / 1e9:.3f} |" if gb is not None else
                     f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} | - |")
    with open(f"profiles/rocprof_{tag}.md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()

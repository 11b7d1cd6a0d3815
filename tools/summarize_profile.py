"""Summarise a tools/profile_round.sh run into profiles/rocprof_<tag>.md and
profiles/pmc_<tag>.json (per kernel: calls, average duration, HBM bytes per launch, SQ
counters, MFMA busy).

    python3 tools/summarize_profile.py <outdir> <tag> [bench.py args]

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming
read, so bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (our kernels stream 16 B per lane).
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of
SIMD-cycles the matrix pipe was busy during the launch.  Calibrated on r02's glds kernel:
SQ_VALU_MFMA_BUSY_CYCLES = 16 x SQ_INSTS_MFMA (16x16x32 bf16 = 16 cycles, summed over the
chip) and GRBM_GUI_ACTIVE is summed over the 8 XCDs (GRBM_GUI_ACTIVE / 8 / duration = the
shader clock, 2.2 GHz under this load), so busy agrees with achieved TF/s / clock-scaled peak.
The JSON records the workload the counters describe ("meta"), which bench.py matches before
it reports a "traffic" figure.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


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


def bench_meta(argv):
    """Workload of the profiled bench.py command line (mirrors bench.py's defaults)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--grid", type=int, default=128)
    ap.add_argument("--scenes", type=int, default=4)
    ap.add_argument("--workload", default="cfg2")
    a, _ = ap.parse_known_args(argv)
    meta = {"workload": a.workload, "dtype": a.dtype, "command": "bench.py " + " ".join(argv)}
    # the build the counters describe: bench.py quotes "traffic" only for this exact libpcs.so
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import lib_sha16
    meta["lib_sha16"] = lib_sha16()
    if a.workload == "cfg2":
        meta["points_per_step"] = a.scenes * a.grid ** 3
    return meta


def main():
    out, tag = sys.argv[1], sys.argv[2]
    meta = bench_meta(sys.argv[3:])
    stats = find(os.path.join(out, "trace", "**", "*kernel_stats.csv"))
    rows = []
    if stats:
        with open(stats) as f:
            rows = list(csv.DictReader(f))
    counters = defaultdict(lambda: defaultdict(list))
    for which in ("fetch", "write", "sq", "grbm"):
        path = find(os.path.join(out, which, "**", "*counter_collection.csv"))
        if not path:
            continue
        with open(path) as f:
            for r in csv.DictReader(f):
                counters[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    pmc = {}
    for k, d in counters.items():
        ent = {c: sum(v) / len(v) for c, v in d.items() if v}
        if "FETCH_SIZE" in ent and "WRITE_SIZE" in ent:
            ent["hbm_bytes_per_launch"] = (2 * ent["FETCH_SIZE"] + ent["WRITE_SIZE"]) * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in ent and ent.get("GRBM_GUI_ACTIVE"):
            ent["mfma_busy"] = ent["SQ_VALU_MFMA_BUSY_CYCLES"] / (ent["GRBM_GUI_ACTIVE"] / XCDS * SIMDS)
        if ent.get("SQ_INSTS_MFMA"):
            ent["valu_per_mfma"] = ent.get("SQ_INSTS_VALU", 0.0) / ent["SQ_INSTS_MFMA"]
        if ent.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in ent:
                    ent[c.lower()[3:] + "_frac"] = ent[c] / ent["SQ_WAVE_CYCLES"]
        pmc[k] = ent
    lines = [f"# rocprofv3 summary ({tag})", "",
             f"Command: `rocprofv3 --kernel-trace --stats --output-format csv -- python3 {meta['command']}` "
             f"(workload {meta['workload']}, {meta['dtype']}), plus separate `--pmc FETCH_SIZE`, "
             "`--pmc WRITE_SIZE`, an 8-counter SQ pass and a GRBM pass "
             "(`tools/profile_round.sh`).", "",
             "HBM = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH correction). MFMA busy = "
             "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); clock = GRBM_GUI_ACTIVE / 8 / avg duration. Wait / issue-stall / "
             "active = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES.", "",
             "| kernel | calls | total ms | avg ms | % | HBM GB/launch | MFMA busy | clock GHz | VALU/MFMA | wait / stall / active |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        name = short(r["Name"])
        ent = pmc.get(name, {})
        gb = ent.get("hbm_bytes_per_launch")
        mb = ent.get("mfma_busy")
        vm = ent.get("valu_per_mfma")
        ws = [ent.get(c) for c in ("wait_any_frac", "wait_inst_any_frac", "active_inst_any_frac")]
        ga = ent.get("GRBM_GUI_ACTIVE")
        clk = ga / XCDS / (float(r["AverageNs"]) * 1e-9) / 1e9 if ga else None
        if clk is not None:
            ent["clock_ghz"] = clk
        lines.append(
            f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
            f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} | "
            f"{'-' if gb is None else f'{gb / 1e9:.3f}'} | {'-' if mb is None else f'{mb:.3f}'} | "
            f"{'-' if clk is None else f'{clk:.2f}'} | "
            f"{'-' if vm is None else f'{vm:.2f}'} | "
            f"{'-' if None in ws else ' / '.join(f'{w:.2f}' for w in ws)} |")
    os.makedirs("profiles", exist_ok=True)
    with open(f"profiles/pmc_{tag}.json", "w") as f:
        json.dump({"meta": meta, "kernels": pmc}, f, indent=1, sort_keys=True)
    with open(f"profiles/rocprof_{tag}.md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()

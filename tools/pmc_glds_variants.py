"""Summarises tools/pmc_glds_variants.sh: per bench_glds.py variant (in launch order, 5
dispatches each) the kernel, average duration, FETCH_SIZE (x2, gfx950 correction) and clock."""
import csv
import sys
from collections import defaultdict

NAMES = ["[glds] fwd, no epilogue", "[glds] fwd + stats", "[glds] fwd + stats + pool", "[glds] fwd + pool",
         "[big ] fwd, no epilogue", "[big ] fwd + stats", "[big ] fwd + stats + pool", "[big ] fwd + pool",
         "[glds] fwd + pool, signed W", "[glds] dgrad: mask + store", "[glds] dgrad: + bias + S1",
         "[gen ] dgrad"]


def load(path):
    rows = defaultdict(dict)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            if "gemm" not in k:
                continue
            d = rows[int(r["Dispatch_Id"])]
            d["k"] = k.split("(")[0].replace("(anonymous namespace)::", "")
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [rows[i] for i in sorted(rows)]


def main(out):
    fe = load(f"{out}/fetch/run_counter_collection.csv")
    gr = load(f"{out}/grbm/run_counter_collection.csv")
    for v, name in enumerate(NAMES):
        f5, g5 = fe[5 * v:5 * v + 5], gr[5 * v:5 * v + 5]
        if len(f5) < 5:
            break
        gb = sum(2 * d["FETCH_SIZE"] * 1024 for d in f5) / 5 / 1e9
        ms = sum(d["ns"] for d in g5) / 5 / 1e6
        clk = sum(d["GRBM_GUI_ACTIVE"] / 8 / d["ns"] for d in g5) / 5
        print(f"{name:32s} {f5[0]['k'][:40]:40s} {ms:8.3f} ms  fetch {gb:7.2f} GB  clock {clk:5.2f} GHz")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_glds")

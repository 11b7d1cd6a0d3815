"""Per-kernel averages of the tools/pmc_w4.sh passes (all counter CSVs under the given dir)."""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import short  # noqa: E402

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if os.environ.get("PMC_FILTER", "gemm") not in k:
                continue
            acc[k][r["Counter_Name"]].append((float(r["Counter_Value"]),
                                              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
for k, d in acc.items():
    ent = {c: sum(v for v, _ in xs) / len(xs) for c, xs in d.items()}
    dur = [t for xs in d.values() for _, t in xs]
    dur = sum(dur) / len(dur)
    print(f"== {k}  (avg {dur * 1e3:.3f} ms over the counted launches)")
    for c in sorted(ent):
        print(f"   {c:28s} {ent[c]:.4g}")
    ga = ent.get("GRBM_GUI_ACTIVE")
    if ga:
        print(f"   clock GHz                    {ga / 8 / dur / 1e9:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in ent:
            print(f"   mfma busy                    {ent['SQ_VALU_MFMA_BUSY_CYCLES'] / (ga / 8 * 1024):.3f}")
    wc = ent.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA"):
            if c in ent:
                print(f"   {c + ' / wave cyc':40s} {ent[c] / wc:.3f}")
    if "FETCH_SIZE" in ent:
        print(f"   HBM GB (2 FETCH + WRITE)     {(2 * ent['FETCH_SIZE'] + ent.get('WRITE_SIZE', 0)) * 1024 / 1e9:.2f}")

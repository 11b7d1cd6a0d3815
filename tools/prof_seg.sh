#!/bin/bash
# Counters of the fused seg backward kernel (tools/bench_seg.py), one rocprofv3 pass each.
set -e
OUT=gpurun_out/prof_seg
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/bench_seg.py 5 > $OUT/time.txt 2>&1
cat $OUT/time.txt
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $OUT/sq -o run -- python3 tools/bench_seg.py 1 > $OUT/sq.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq2 -o run -- python3 tools/bench_seg.py 1 > $OUT/sq2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/bench_seg.py 1 > $OUT/fetch.log 2>&1
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/prof_seg/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "seg_bwd" not in n and "seg4" not in n: continue
        agg[n[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:24s} {sum(v)/len(v):.4g}")
PY

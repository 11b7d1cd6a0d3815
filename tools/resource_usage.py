"""Per-kernel register / spill / occupancy table of a csrc tree (hipcc's kernel-resource-usage
remarks), for comparing a change against HEAD before spending GPU time on it:

    python tools/resource_usage.py point-cloud-cnn-segmentation_amd/csrc > /tmp/new.txt
    git archive HEAD point-cloud-cnn-segmentation_amd/csrc include | tar -x -C /tmp/head
    python tools/resource_usage.py /tmp/head/point-cloud-cnn-segmentation_amd/csrc > /tmp/head.txt
    diff /tmp/head.txt /tmp/new.txt

The per-file flags mirror csrc/Makefile's EXTRA lines."""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

EXTRA = {"gemm_glds.hip": ["-mllvm", "-disable-machine-sink"], "gram_glds.hip": ["-mllvm", "-disable-machine-sink"],
         "fused_seg4.hip": ["-fno-slp-vectorize"], "fwd_s12.hip": ["-fno-slp-vectorize"]}
KEYS = ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill")


def usage(csrc, f):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
           "-Rpass-analysis=kernel-resource-usage", "-c", f, "-o", os.devnull] + EXTRA.get(f, [])
    err = subprocess.run(cmd, cwd=csrc, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None and k in KEYS:
            cur[k] = v
    return [f"{f}: {r['name']} " + " ".join(f"{k.split()[0]}{'-spill' if 'Spill' in k else ''}={r.get(k, '?')}"
                                           for k in KEYS) for r in rows]


def main():
    csrc = sys.argv[1]
    files = sorted(f for f in os.listdir(csrc) if f.endswith(".hip"))
    with ThreadPoolExecutor(8) as ex:
        for lines in ex.map(lambda f: usage(csrc, f), files):
            for ln in lines:
                print(ln)


if __name__ == "__main__":
    main()

"""Which bf16-stored tensor carries the bf16 path's pre-pool gradient error?  

numpy only (no GPU): oracle/bf16_emulation.py, which reproduces the HIP bf16 path's per-tensor
gradient error (ratio 0.88-1.11, profiles/bf16_emulation_r02.md), is run with one group of
rounding sites at a time left in fp32 ("exact"), and with the fp32 step's max-pool argmax rows
imposed on the bf16 step ("fp32 argmax"), at G^3 points per scene (4 scenes, one train step,
replayed dropout).  Printed: 1 - cos against the all-fp32 emulation, per pre-pool tensor.
    python tools/bf16_ablation.py [G]      (default 64 = 262,144 points per scene)
"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "oracle")]
import numpy as np

import bf16_emulation as emu
import pointnet_oracle as orc
from pcs_amd.data import class_weights, synthetic_batch

TENSORS = ["conv1.weight", "conv2.weight", "conv3.weight", "conv4.weight", "conv5.weight", "global_feat.weight",
           "bn5.weight", "bn_global.weight", "seg_conv1.weight", "seg_conv2.weight"]


def cos1(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return 1.0 - float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-300))


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    sd = orc.init_params(2, 77)
    pts, lab, _ = synthetic_batch(4321, [G ** 3] * 4, 2, grid=G, dense=True)
    w = class_weights([lab[b] for b in range(4)], num_classes=2)
    masks = orc.dropout_masks(99, pts.shape[0] * pts.shape[1])
    info = {}
    t0 = time.time()
    _, ref = emu.train_step(sd, pts, lab, w, masks, store="fp32", info=info)
    idx32 = info["pool_idx"]
    print(f"## bf16 ablation, N = {G ** 3} points per scene (4 scenes), fp32 reference in {time.time() - t0:.0f} s",
          flush=True)
    print("| bf16 run | pool rows differing from fp32 | " + " | ".join(TENSORS) + " |")
    print("|---" * (len(TENSORS) + 2) + "|")
    runs = [("all sites bf16 (the HIP bf16 path)", (), None),
            ("fp32 argmax imposed", (), idx32),
            ("W exact", ("W",), None), ("Y exact", ("Y",), None), ("A exact", ("A",), None),
            ("a5 exact", ("a5",), None), ("dz exact", ("dz",), None), ("dy exact", ("dy",), None),
            ("DZ5 exact", ("DZ5",), None), ("H exact", ("H",), None), ("fold5 + dA4 exact", ("fold5", "dA4"), None),
            ("dA2 exact", ("dA2",), None),
            ("forward exact (W, Y, A, a5)", ("W", "Y", "A", "a5"), None),
            ("backward exact (dz, dy, DZ5, H, fold5, dA2, dA4)", ("dz", "dy", "DZ5", "H", "fold5", "dA2", "dA4"), None),
            ("everything exact", ("W", "Y", "A", "a5", "dz", "dy", "DZ5", "H", "fold5", "dA2", "dA4"), None)]
    for name, exact, pidx in runs:
        t0 = time.time()
        inf = {}
        _, g = emu.train_step(sd, pts, lab, w, masks, store="bf16", exact=exact, pool_idx=pidx, info=inf)
        flips = int((inf["pool_idx"] != idx32).sum()) if pidx is None else 0
        cells = " | ".join(f"{cos1(g[t], ref[t]):.3g}" for t in TENSORS)
        print(f"| {name} | {flips} / {idx32.size} | {cells} |  <!-- {time.time() - t0:.0f} s -->", flush=True)


if __name__ == "__main__":
    main()

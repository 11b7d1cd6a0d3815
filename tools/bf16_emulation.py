"""Is the bf16 path's gradient error storage-intrinsic?  (VERDICT r01 "What's weak" #4.)

For dense G^3 scenes (B = 4, one train-mode step, identical weights and replayed dropout
masks) this compares, per gradient tensor, 1 - cos of
  * HIP bf16 vs HIP fp32                      (what tests/test_gpu_fullsize.py bounds)
  * numpy bf16-storage emulation vs numpy fp32 (oracle/bf16_emulation.py: the same
    computation with every tensor the HIP bf16 path stores rounded to bf16 where it rounds)
  * HIP fp32 vs numpy fp32                    (sanity: both fp32 restatements agree)
If the first two columns agree, the HIP bf16 error is what bf16 storage costs this network.
    python tools/bf16_emulation.py [G ...]     (default 16 32 64; needs a GPU and ~40 GB RAM)
"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "oracle")]
import numpy as np
import torch

import bf16_emulation as emu
import pointnet_oracle as orc
from pcs_amd.data import class_weights, synthetic_batch
from pcs_amd.model import PointNetSegmentation

DEV = torch.device("cuda")


def cos1(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return 1.0 - float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-300))


def hip_grads(sd, pts, lab, w, masks, dt):
    m = PointNetSegmentation(2, compute_dtype=dt).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
    m.train()
    m.set_dropout_masks(*(torch.from_numpy(np.packbits(k, axis=1, bitorder="little")).to(DEV) for k in masks))
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    loss = crit(m(torch.from_numpy(pts).to(DEV)).contiguous().view(-1, 2), torch.from_numpy(lab).to(DEV).view(-1))
    loss.backward()
    g = {n: p.grad.detach().double().cpu().numpy() for n, p in m.named_parameters()}
    del m
    torch.cuda.empty_cache()
    return float(loss), g


def main():
    grids = [int(a) for a in sys.argv[1:]] or [16, 32, 64]
    sd = orc.init_params(2, 77)
    for G in grids:
        pts, lab, _ = synthetic_batch(4321, [G ** 3] * 4, 2, grid=G, dense=True)
        w = class_weights([lab[b] for b in range(4)], num_classes=2)
        masks = orc.dropout_masks(99, pts.shape[0] * pts.shape[1])
        t0 = time.time()
        lh32, h32 = hip_grads(sd, pts, lab, w, masks, "fp32")
        lh16, h16 = hip_grads(sd, pts, lab, w, masks, "bf16")
        le32, e32 = emu.train_step(sd, pts, lab, w, masks, store="fp32")
        le16, e16 = emu.train_step(sd, pts, lab, w, masks, store="bf16")
        print(f"\n## N = {G ** 3} points per scene (4 scenes, {G}^3 grid): loss HIP fp32 {lh32:.6f} bf16 {lh16:.6f}, "
              f"emulation fp32 {le32:.6f} bf16 {le16:.6f}  ({time.time() - t0:.0f} s)", flush=True)
        print("| tensor | HIP bf16 vs HIP fp32 | emulated bf16 vs fp32 | ratio | HIP fp32 vs numpy fp32 |")
        print("|---|---|---|---|---|")
        for n in h32:
            if (n.endswith(".bias") and not n.startswith(("bn", "seg_conv4"))) or n == "bn_global.bias":
                continue   # analytically ~0 (BN-cancelled conv biases, bn_global.bias)
            a, b, c = cos1(h16[n], h32[n]), cos1(e16[n], e32[n]), cos1(h32[n], e32[n])
            print(f"| {n} | {a:.3e} | {b:.3e} | {a / max(b, 1e-300):.2f} | {c:.1e} |", flush=True)


if __name__ == "__main__":
    main()

"""Dump the weights test_gpu_miou's fixture trains (300 fused fp32 steps) and the device eval
logits of the ragged val batch in fp32 / bf16 / fp8, for the CPU-side attribution of the bf16
eval error (tools/miou_attr.py).

    python tools/miou_dump.py gpurun_out/miou_r05
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]

import pcs_amd.data as pdata  # noqa: E402
from pcs_amd.model import PointNetSegmentation  # noqa: E402
from pcs_amd.optim import FusedAdam  # noqa: E402
from pcs_amd.train import FusedTrainStep  # noqa: E402

DEV = torch.device("cuda")
C = 2


def main(out):
    os.makedirs(out, exist_ok=True)
    torch.manual_seed(7)
    m = PointNetSegmentation(C).to(DEV)
    pts, lab, _ = pdata.synthetic_batch(11, [4096] * 4, C, grid=32)
    w = pdata.class_weights([lab[b][lab[b] >= 0] for b in range(lab.shape[0])], num_classes=C)
    step = FusedTrainStep(m, FusedAdam(m, lr=3e-3), class_weight=w)
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV)
    for i in range(300):
        step(x, y, seed=1000 + i)
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    np.savez(os.path.join(out, "trained_sd.npz"), **sd)
    vpts, vlab, _ = pdata.synthetic_batch(4242, [8192, 6000, 8192, 5000], C, grid=32)
    res = {"pts": vpts, "lab": vlab}
    for dt, trunk, key in (("fp32", "fp32", "fp32"), ("bf16", "fp32", "bf16"), ("fp8", "fp32", "fp8"),
                           ("bf16", "bf16", "bf16_trunk16"), ("fp8", "bf16", "fp8_trunk16")):
        mm = PointNetSegmentation(C, compute_dtype=dt, eval_trunk=trunk).to(DEV)
        mm.load_state_dict({k: torch.as_tensor(np.array(v)) for k, v in sd.items()})
        mm.eval()
        with torch.no_grad():
            res[f"logits_{key}"] = mm(torch.from_numpy(vpts).to(DEV)).float().cpu().numpy()
    np.savez(os.path.join(out, "val_logits.npz"), **res)
    print("wrote", out, flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/miou_r05")

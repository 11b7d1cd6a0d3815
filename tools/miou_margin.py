"""Where the mIoU difference of the bf16 / fp8 eval path comes from, on the weights the
test_gpu_miou fixture trains (40 fused steps) and on longer-trained ones:

* training determinism: the fixture's 40 steps run twice, max |difference| of the weights;
* per trained checkpoint: the fp64 oracle's eval logits on the ragged val batch, the device
  fp32 / bf16 / fp8 predictions, the number of flipped points, the mIoU difference and the
  oracle's logit margin |l1 - l0| at the flipped points (how close to the decision boundary).

    python tools/miou_margin.py
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]

import pointnet_oracle as orc  # noqa: E402
import pcs_amd.data as pdata  # noqa: E402
from pcs_amd.metrics import ConfusionMeter  # noqa: E402
from pcs_amd.model import PointNetSegmentation  # noqa: E402
from pcs_amd.optim import FusedAdam  # noqa: E402
from pcs_amd.train import FusedTrainStep  # noqa: E402

DEV = torch.device("cuda")
C = 2


def train(steps, report_at):
    torch.manual_seed(7)
    m = PointNetSegmentation(C).to(DEV)
    pts, lab, _ = pdata.synthetic_batch(11, [4096] * 4, C, grid=32)
    w = pdata.class_weights([lab[b][lab[b] >= 0] for b in range(lab.shape[0])], num_classes=C)
    step = FusedTrainStep(m, FusedAdam(m, lr=3e-3), class_weight=w)
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV)
    out = {}
    for i in range(steps):
        step(x, y, seed=1000 + i)
        if i + 1 in report_at:
            torch.cuda.synchronize()
            out[i + 1] = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    return out


def device_eval(sd, pts, lab, dtype):
    m = PointNetSegmentation(C, compute_dtype=dtype).to(DEV)
    m.load_state_dict({k: torch.as_tensor(np.array(v)) for k, v in sd.items()})
    m.eval()
    meter = ConfusionMeter(C, DEV)
    with torch.no_grad():
        lg = m(torch.from_numpy(pts).to(DEV))
        meter.update(lg, torch.from_numpy(lab).to(DEV))
    return lg.float().cpu().numpy(), meter.compute()["miou"]


def main():
    marks = (40, 120, 300)
    a = train(40, {40})[40]
    b = train(max(marks), set(marks))
    diff = max(float(np.abs(np.asarray(a[k], np.float64) - np.asarray(b[40][k], np.float64)).max())
               for k in a if a[k].dtype.kind == "f")
    print(f"training determinism (40 steps, two runs): max |dw| = {diff:.3e}", flush=True)
    pts, lab, _ = pdata.synthetic_batch(4242, [8192, 6000, 8192, 5000], C, grid=32)
    v = lab.reshape(-1) >= 0
    for s in marks:
        sd = b[s]
        ref, _ = orc.forward({k: np.asarray(x, np.float64) if x.dtype.kind == "f" else x
                              for k, x in sd.items()}, pts, train=False)
        rp = ref.argmax(-1).reshape(-1)
        marg = np.abs(ref[..., 1] - ref[..., 0]).reshape(-1)
        cm = np.zeros((C, C), np.int64)
        np.add.at(cm, (lab.reshape(-1)[v], rp[v]), 1)
        inter = np.diag(cm)
        ref_miou = float(np.mean(inter / (cm.sum(0) + cm.sum(1) - inter)))
        print(f"steps {s}: oracle mIoU {ref_miou:.6f}, prediction histogram {np.bincount(rp[v], minlength=C)}, "
              f"points with margin < 1e-2: {int((marg[v] < 1e-2).sum())}, < 1e-1: {int((marg[v] < 1e-1).sum())}",
              flush=True)
        for dt in ("fp32", "bf16", "fp8"):
            lg, mi = device_eval(sd, pts, lab, dt)
            fl = (lg.argmax(-1).reshape(-1) != rp) & v
            mf = marg[fl]
            q = np.quantile(mf, [0.5, 1.0]) if fl.any() else (0.0, 0.0)
            print(f"  {dt}: mIoU {mi:.6f} (diff {mi - ref_miou:+.2e}), flipped {int(fl.sum())} of {int(v.sum())}, "
                  f"oracle margin at flips median {q[0]:.2e} max {q[1]:.2e}", flush=True)


if __name__ == "__main__":
    main()

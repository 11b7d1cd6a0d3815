"""How the fp8 wide layer (compute dtype "fp8") changes predictions, against fp32 and bf16:

1. golden cases (random-init weights, the reference's own step): argmax agreement with fp32
   and mIoU against the labels per dtype;
2. training: the same init trained K steps on cfg1-sized synthetic scenes in fp32 and in fp8
   (FusedTrainStep + FusedAdam), loss curves and held-out mIoU;
3. the fp32-trained weights evaluated (eval-mode BN) in each dtype on a held-out cfg1 batch
   and at cfg2 size (4 x 128^3): argmax agreement and mIoU difference.

    python tools/fp8_accuracy.py [steps]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]

from golden_util import CASES, inputs, load  # noqa: E402
from pcs_amd.data import class_weights, synthetic_batch  # noqa: E402
from pcs_amd.metrics import ConfusionMeter, miou  # noqa: E402
from pcs_amd.model import PointNetSegmentation  # noqa: E402
from pcs_amd.optim import FusedAdam  # noqa: E402
from pcs_amd.train import FusedTrainStep  # noqa: E402

DEV = torch.device("cuda")
DTYPES = ("fp32", "bf16", "fp8")


def model_from(sd, C, dtype, train):
    m = PointNetSegmentation(C, compute_dtype=dtype).to(DEV)
    m.load_state_dict({k: (v if torch.is_tensor(v) else torch.from_numpy(np.array(v))) for k, v in sd.items()})
    m.train(train)
    return m


def miou_of(logits, labels, C):
    return miou(ConfusionMeter(C, DEV).update(logits, labels).cm.cpu().numpy())


def compare(logits, labels, C, tag):
    ref = logits["fp32"]
    valid = labels.reshape(-1) >= 0
    m32 = miou_of(ref, labels, C)
    out = {}
    for dt in DTYPES[1:]:
        a = logits[dt]
        agree = float((a.argmax(-1).reshape(-1) == ref.argmax(-1).reshape(-1))[valid].float().mean())
        mi = miou_of(a, labels, C)
        out[dt] = (agree, mi - m32)
        print(f"  {tag:34s} {dt}: argmax agreement {agree:.5f}  mIoU {mi:.5f} (fp32 {m32:.5f}, "
              f"diff {mi - m32:+.2e})", flush=True)
    return out


def golden():
    print("1. golden cases (random-init weights)")
    for name in CASES:
        g = load(name)
        sd, pts, lab, _, masks = inputs(g)
        C = int(g["C"])
        train = bool(g["train"])
        x = torch.from_numpy(pts).to(DEV)
        y = torch.from_numpy(lab).to(DEV)
        bits = tuple(torch.from_numpy(np.packbits(m, axis=1, bitorder="little")).to(DEV) for m in masks)
        logits = {}
        for dt in DTYPES:
            m = model_from(sd, C, dt, train)
            if train:
                m.set_dropout_masks(*bits)
            with torch.no_grad():
                logits[dt] = m(x).float()
        compare(logits, y, C, name)


def train_curves(steps, dtypes=DTYPES):
    print(f"2. training {steps} steps from one init (cfg1-size scenes, C=2)")
    C, B, N = 2, 4, 4096
    torch.manual_seed(0)
    init = {k: v.clone() for k, v in PointNetSegmentation(C).state_dict().items()}
    trained = {}
    for dt in dtypes:
        m = model_from(init, C, dt, True)
        opt = FusedAdam(m, lr=1e-3, weight_decay=1e-4)
        losses = []
        for s in range(steps):
            pts, lab, _ = synthetic_batch(5000 + s, [N] * B, C, grid=32)
            w = class_weights([lab[b] for b in range(B)], num_classes=C)
            step = FusedTrainStep(m, opt, class_weight=w)
            loss = step(torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV))
            losses.append(float(loss))
        print(f"  {dt}: loss " + " ".join(f"{losses[i]:.4f}" for i in range(0, steps, max(1, steps // 10))) +
              f" ... {losses[-1]:.4f}", flush=True)
        trained[dt] = {k: v.detach().clone() for k, v in m.state_dict().items()}
    pts, lab, _ = synthetic_batch(99, [N] * B, C, grid=32)
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV)
    for dt in dtypes:
        for de in DTYPES:
            m = model_from(trained[dt], C, de, False)
            with torch.no_grad():
                mi_e = miou_of(m(x).float(), y, C)
            m.train(True)
            with torch.no_grad():
                mi_t = miou_of(m(x).float(), y, C)
            print(f"  held-out mIoU of the {dt}-trained model, {de}: eval BN {mi_e:.5f}, batch BN {mi_t:.5f}")
    return trained["fp32"]


def trained_eval(sd):
    print("3. fp32-trained weights, eval-mode BN")
    C = 2
    for tag, (n, grid, dense) in (("cfg1 held-out (4 x 4096)", (4096, 32, False)),
                                  ("cfg2 (4 x 128^3)", (128 ** 3, 128, True))):
        pts, lab, _ = synthetic_batch(4242, [n] * 4, C, grid=grid, dense=dense)
        x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV)
        del pts, lab
        logits = {}
        for dt in DTYPES:
            m = model_from(sd, C, dt, False)
            with torch.no_grad():
                logits[dt] = m(x).float()
            del m
        compare(logits, y, C, tag)
        del logits
        torch.cuda.empty_cache()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    if os.environ.get("FP8ACC_GOLDEN", "1") == "1":
        golden()
    sd = train_curves(steps, tuple(os.environ.get("FP8ACC_TRAIN", ",".join(DTYPES)).split(",")))
    trained_eval(sd)


if __name__ == "__main__":
    main()

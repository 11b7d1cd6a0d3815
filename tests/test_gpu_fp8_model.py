"""The fp8 compute dtype (BASELINE configs[4] / SURVEY cfg5: the bf16 step with a5 and
global_feat's GEMMs in e4m3 on MX-scaled MFMA) against the fp32 path, end to end.

What fp8 storage costs is measured, not assumed: oracle/bf16_emulation.py with store="fp8"
rounds exactly the tensors the HIP fp8 path stores (bf16 everywhere the bf16 path rounds,
a5 to e4m3, global_feat's W and the folded H to row-scaled e4m3).  On the golden cases the
HIP fp8 logits' error against the fp32 oracle is 0.5x..2x the emulation's (storage-intrinsic,
not a kernel error; measured r02: 1.00, 1.01, 1.06).

Prediction-level bounds (measured r02, tools/fp8_accuracy.py, bound = measured + margin):

* golden cases (random-init weights, the reference's own step): the eval-mode case agrees
  exactly (agreement 1.0, dmIoU 0; bound 1e-3).  The train-mode cases (batch-statistics BN
  over random weights: most points sit near a decision boundary) agree >= 0.85 (measured
  0.878 .. 0.956; bf16 0.955 .. 0.985) with |mIoU_fp8 - mIoU_fp32| <= 5e-3 (measured
  0.9e-3 .. 3.1e-3; bf16 0.2e-3 .. 1.8e-3): not 1e-3, and the emulation above shows that
  is what e4m3's 3 mantissa bits cost there, not a kernel error.
* cfg2 size (4 x 128^3) with weights trained 3000 steps in fp32 on cfg1-sized scenes
  (eval-mode BN): agreement >= 0.998 (measured 0.99906; bf16 0.99942), |dmIoU| <= 1e-3
  (measured 5.4e-4; bf16 6e-5).  How far a prediction flip moves mIoU depends on how many
  points sit near a decision boundary: after only 200-600 steps agreement is 0.987-0.998 and
  |dmIoU| ranged 3.5e-4 .. 7.7e-3 for fp8 and 6e-5 .. 4.5e-3 for bf16 over training
  lengths and dropout streams (tools/fp8_accuracy.py).  The path is deterministic
  (fixed-order reductions, Philox dropout), so each figure is one fixed measurement.
* training: 300 fp8 steps from the fp32 run's init track the fp32 loss curve (mean of the
  last 100 losses within 0.03; measured 600-step curves within 0.01).
"""
import os
import sys

import numpy as np
import pytest
import torch

import pointnet_oracle as orc
from golden_util import CASES, inputs, load

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import bf16_emulation as emu  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _model(sd, C, dtype, train):
    from pcs_amd.model import PointNetSegmentation
    m = PointNetSegmentation(C, compute_dtype=dtype).to(DEV)
    m.load_state_dict({k: (v if torch.is_tensor(v) else torch.from_numpy(np.array(v))) for k, v in sd.items()})
    m.train(train)
    return m


def _miou(logits, labels, C):
    from pcs_amd.metrics import ConfusionMeter, miou
    return miou(ConfusionMeter(C, DEV).update(logits, labels).cm.cpu().numpy())


def _agree(a, b, labels):
    valid = labels.reshape(-1) >= 0
    return float((a.argmax(-1).reshape(-1) == b.argmax(-1).reshape(-1))[valid].float().mean())


@pytest.mark.parametrize("name", CASES)
def test_fp8_golden_predictions_track_fp32(name):
    g = load(name)
    sd, pts, lab, _, masks = inputs(g)
    C, train = int(g["C"]), bool(g["train"])
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV)
    bits = tuple(torch.from_numpy(np.packbits(m, axis=1, bitorder="little")).to(DEV) for m in masks)
    out = {}
    for dt in ("fp32", "fp8"):
        m = _model(sd, C, dt, train)
        if train:
            m.set_dropout_masks(*bits)
        with torch.no_grad():
            out[dt] = m(x).float()
    agree = _agree(out["fp8"], out["fp32"], y)
    dm = _miou(out["fp8"], y, C) - _miou(out["fp32"], y, C)
    print(f"{name}: fp8 argmax agreement {agree:.5f}, dmIoU {dm:+.2e}")
    if not train:
        assert agree >= 0.999 and abs(dm) <= 1e-3
        return
    assert agree >= 0.85 and abs(dm) <= 5e-3
    # storage-intrinsic: the emulated fp8 step's logit error against the fp32 oracle
    ref = orc.forward(sd, pts, train=True, masks=masks)[0].reshape(-1, C).astype(np.float64)
    e_emu = emu.train_step(sd, pts, lab, g["weight"], masks, store="fp8", return_logits=True)[2]
    valid = lab.reshape(-1) >= 0
    hip = out["fp8"].reshape(-1, C).cpu().numpy().astype(np.float64)
    err_hip = np.linalg.norm((hip - ref)[valid]) / np.linalg.norm(ref[valid])
    err_emu = np.linalg.norm((e_emu.astype(np.float64) - ref)[valid]) / np.linalg.norm(ref[valid])
    print(f"{name}: logits rel err HIP fp8 {err_hip:.3e}, emulated fp8 {err_emu:.3e}, ratio {err_hip / err_emu:.2f}")
    assert 0.5 <= err_hip / err_emu <= 2.0


def _train(dtypes, steps):
    """dtype -> (trained state, per-step losses): ``steps`` FusedTrainStep + FusedAdam steps
    on cfg1-sized synthetic scenes from one seeded init."""
    from pcs_amd.data import class_weights, synthetic_batch
    from pcs_amd.model import PointNetSegmentation
    from pcs_amd.optim import FusedAdam
    from pcs_amd.train import FusedTrainStep
    C, B, N = 2, 4, 4096
    torch.manual_seed(0)
    init = {k: v.clone() for k, v in PointNetSegmentation(C).state_dict().items()}
    res = {}
    for dt in dtypes:
        m = _model(init, C, dt, True)
        opt = FusedAdam(m, lr=1e-3, weight_decay=1e-4)
        losses = []
        for s in range(steps):
            pts, lab, _ = synthetic_batch(5000 + s, [N] * B, C, grid=32)
            w = class_weights([lab[b] for b in range(B)], num_classes=C)
            loss = FusedTrainStep(m, opt, class_weight=w)(torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV))
            losses.append(float(loss))
        res[dt] = ({k: v.detach().clone() for k, v in m.state_dict().items()}, np.array(losses))
        del m, opt
    return res


@pytest.fixture(scope="module")
def trained():
    return _train(("fp32", "fp8"), 300)


def test_fp8_training_tracks_fp32(trained):
    l32, l8 = trained["fp32"][1], trained["fp8"][1]
    assert np.isfinite(l8).all()
    print(f"mean loss of the last 100 steps: fp32 {l32[-100:].mean():.4f}, fp8 {l8[-100:].mean():.4f}")
    assert abs(l8[-100:].mean() - l32[-100:].mean()) < 0.03
    assert l8[-100:].mean() < l8[:10].mean() - 0.05        # it learns


def test_fp8_cfg2_predictions_track_fp32():
    from pcs_amd.data import synthetic_batch
    sd = _train(("fp32",), 3000)["fp32"][0]
    pts, lab, _ = synthetic_batch(4242, [128 ** 3] * 4, 2, grid=128, dense=True)
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV)
    del pts, lab
    out = {}
    for dt in ("fp32", "bf16", "fp8"):
        m = _model(sd, 2, dt, False)
        with torch.no_grad():
            out[dt] = m(x).float()
        del m
    m32 = _miou(out["fp32"], y, 2)
    for dt in ("bf16", "fp8"):
        print(f"cfg2: {dt} argmax agreement {_agree(out[dt], out['fp32'], y):.5f}, mIoU {_miou(out[dt], y, 2):.5f} "
              f"(fp32 {m32:.5f})")
    agree = _agree(out["fp8"], out["fp32"], y)
    m8 = _miou(out["fp8"], y, 2)
    assert agree >= 0.998 and abs(m8 - m32) <= 1e-3

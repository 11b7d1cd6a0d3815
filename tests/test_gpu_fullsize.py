"""Full-size (BASELINE configs[1] / SURVEY §8(d) cfg2) checks on MI355X: 4 scenes x 128^3 points,
C=2, the bench's own workload.  The oracle cannot run this size (≈300 GB of fp64
activations), so the bf16 bench path is checked against the fp32 HIP path -- itself pinned to
the oracle at small sizes (test_gpu_parity) -- through size-independent properties:

* logits: argmax agreement > 95 % and norm-relative error < 0.1 (the bf16 bound of
  test_gpu_parity's bf16 case);
* one training step (same weights, same Philox dropout seed): losses within 1e-2, BN running
  statistics within 2e-2, and per-tensor gradient cosine similarity for every layer
  after the max-pool (seg_conv1..4, bn_seg1..3; 1 - cos <= 0.03, measured r02 0.0218).
  Layers before the pool get their gradient through per-scene sums of the dense
  BN-backward of seg_conv1 (and the sparse pool rows), which cancel to O(pool rows / points)
  of their size, so bf16 storage noise (2^-9 per element, growing ~sqrt(N)) dominates at
  2M points per scene: 1 - cos measured r02 up to 0.496 (conv2).  That this is what bf16
  storage costs and not a kernel error is shown at 4K-262K points per scene, where a numpy
  bf16-storage emulation can run: the HIP error / emulated error ratio is 0.88-1.11 for
  every tensor (test_gpu_bf16_storage.py, profiles/bf16_emulation_r02.md).  Bound: the
  measured value times 1.13, the top of that ratio spread: 1 - cos <= 0.56.  bn_global.bias is skipped: its
  gradient is W^T sum_b csum_b with sum_b csum_b = 0 (BN input gradients sum to zero),
  i.e. analytically ~0 like the BN-cancelled conv biases;
* the 2^21-row scenes exercise the chunk geometry, the 256-row tiles and the fused kernels at
  the row counts the bench uses.
"""
import numpy as np
import pytest
import torch

import pointnet_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.fixture(scope="module")
def cfg2_batch():
    from pcs_amd.data import class_weights, synthetic_batch
    B, G, C = 4, 128, 2
    pts, lab, _ = synthetic_batch(4321, [G ** 3] * B, C, grid=G, dense=True)
    w = class_weights([lab[b] for b in range(B)], num_classes=C)
    return torch.from_numpy(pts), torch.from_numpy(lab), w


def _model(sd, dtype):
    from pcs_amd.model import PointNetSegmentation
    m = PointNetSegmentation(2, compute_dtype=dtype).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
    return m


def test_cfg2_bf16_forward_tracks_fp32(cfg2_batch):
    pts, _, _ = cfg2_batch
    sd = orc.init_params(2, 2024, bn_affine_random=True)
    x = pts.to(DEV)
    out = {}
    for dt in ("fp32", "bf16"):
        m = _model(sd, dt)
        m.eval()
        with torch.no_grad():
            out[dt] = m(x).float().cpu()
        del m
        torch.cuda.empty_cache()
    a, b = out["bf16"], out["fp32"]
    assert torch.isfinite(a).all()
    rel = float((a - b).norm() / b.norm())
    agree = float((a.argmax(-1) == b.argmax(-1)).float().mean())
    print(f"cfg2 eval logits: rel err {rel:.3e}, argmax agreement {agree:.4f}")
    assert rel < 0.1 and agree > 0.95


def test_cfg2_bf16_train_step_tracks_fp32(cfg2_batch):
    """One reference-style step (forward, weighted CE, backward) per dtype with the same
    Philox dropout seed: loss, per-tensor gradient cosine (bounds: module docstring) and BN
    running statistics."""
    pts, lab, w = cfg2_batch
    sd = orc.init_params(2, 77)
    x, y = pts.to(DEV), lab.to(DEV).view(-1)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    res = {}
    for dt in ("fp32", "bf16"):
        m = _model(sd, dt)
        m.train()
        m.seed_dropout(99)
        loss = crit(m(x).contiguous().view(-1, 2), y)
        loss.backward()
        torch.cuda.synchronize()
        res[dt] = (float(loss.detach()), {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()},
                   {n: b.detach().cpu().clone() for n, b in m.named_buffers() if "running" in n})
        del m, loss
        torch.cuda.empty_cache()
    (l32, g32, b32), (l16, g16, b16) = res["fp32"], res["bf16"]
    print(f"cfg2 step loss fp32 {l32:.6f} bf16 {l16:.6f}")
    assert np.isfinite(l16) and abs(l16 - l32) < 1e-2 * max(1.0, abs(l32))
    worst = {}
    for n in g32:
        if (n.endswith(".bias") and not n.startswith(("bn", "seg_conv4"))) or n == "bn_global.bias":
            continue   # analytically ~0 gradients (module docstring): rounding noise in both paths
        a, b = g16[n].flatten().double(), g32[n].flatten().double()
        assert torch.isfinite(a).all(), n
        worst[n] = 1 - float(a @ b / (a.norm() * b.norm() + 1e-30))
    print("cfg2 bf16 gradient 1-cos:", {k: round(v, 4) for k, v in worst.items()})
    post_pool = ("seg_conv", "bn_seg")
    bad = {k: v for k, v in worst.items() if v > (0.03 if k.startswith(post_pool) else 0.56)}
    assert not bad, bad
    for n in b32:
        e = float((b16[n] - b32[n]).norm() / b32[n].norm())
        assert e < 2e-2, (n, e)


def test_cfg2_bf16_step_same_pool_rows_tight(cfg2_batch):
    """The pre-pool gradients at full size with the max-pool's rows held fixed: the bf16 step
    takes the fp32 forward's argmax rows (Engine.pool_rows_override), which removes the
    routing difference that dominates the bound above (profiles/bf16_ablation_r03.md: 728 of
    4096 pool rows move under bf16 rounding at 262K points per scene).  What is left is bf16
    arithmetic and storage, so every tensor, before and after the pool, is held to a tight
    cosine bound: a pre-pool kernel error at the bench size fails here."""
    pts, lab, w = cfg2_batch
    sd = orc.init_params(2, 77)
    x, y = pts.to(DEV), lab.to(DEV).view(-1)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    res, rows = {}, None
    for dt in ("fp32", "bf16"):
        m = _model(sd, dt)
        m.train()
        m.seed_dropout(99)
        eng = m._engine()
        if dt == "fp32":
            eng.record_pool_rows = True
        else:
            eng.pool_rows_override = rows
        loss = crit(m(x).contiguous().view(-1, 2), y)
        loss.backward()
        torch.cuda.synchronize()
        if dt == "fp32":
            rows = eng.last_pool_rows.clone()
        res[dt] = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
        eng.pool_rows_override, eng.record_pool_rows, eng.last_pool_rows = None, False, None
        del m, loss
        torch.cuda.empty_cache()
    g32, g16 = res["fp32"], res["bf16"]
    worst = {}
    for n in g32:
        if (n.endswith(".bias") and not n.startswith(("bn", "seg_conv4"))) or n == "bn_global.bias":
            continue   # analytically ~0 (module docstring)
        a, b = g16[n].flatten().double(), g32[n].flatten().double()
        assert torch.isfinite(a).all(), n
        worst[n] = 1 - float(a @ b / (a.norm() * b.norm() + 1e-30))
    print("cfg2 bf16 gradient 1-cos, fp32 pool rows:", {k: round(v, 5) for k, v in worst.items()})
    bad = {k: v for k, v in worst.items() if v > POOL_ROWS_TIGHT_BOUND}
    assert not bad, bad


# measured at the bench size with the fp32 forward's pool rows (r04, see the test's print), plus
# margin; the routing-dominated bound of test_cfg2_bf16_train_step_tracks_fp32 is 0.56
POOL_ROWS_TIGHT_BOUND = 0.15

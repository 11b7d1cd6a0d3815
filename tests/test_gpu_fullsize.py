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
    arithmetic and storage: every tensor, before and after the pool, within POOL_ROWS_TIGHT_BOUND.

    What this bound can and cannot see (negative controls, Engine.perturb on dz5's columns
    256..511 after global_feat's input gradient): a sign error in that column block fails it;
    a 1 % scale error does not -- 1 - cos is second order in a scale error (~1e-5 here), far
    below the ~0.1 that bf16 rounding noise leaves in the pre-pool layers, whose gradients come
    through per-scene sums that cancel to O(pool rows / points) of their terms (DESIGN.md
    section 4).  Errors of that size are caught by test_cfg2_bf16_prepool_kernels_same_operands,
    which checks those kernels against torch on their own operands."""
    pts, lab, w = cfg2_batch
    sd = orc.init_params(2, 77)
    x, y = pts.to(DEV), lab.to(DEV).view(-1)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    m = _model(sd, "fp32")
    m.train()
    m.seed_dropout(99)
    eng = m._engine()
    eng.record_pool_rows = True
    loss = crit(m(x).contiguous().view(-1, 2), y)
    loss.backward()
    torch.cuda.synchronize()
    rows = eng.last_pool_rows.clone()
    g32 = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
    del m, loss, eng
    torch.cuda.empty_cache()

    def cos_err(g16):
        worst = {}
        for n in g32:
            if (n.endswith(".bias") and not n.startswith(("bn", "seg_conv4"))) or n == "bn_global.bias":
                continue   # analytically ~0 (module docstring)
            a, b = g16[n].flatten().double(), g32[n].flatten().double()
            assert torch.isfinite(a).all(), n
            worst[n] = 1 - float(a @ b / (a.norm() * b.norm() + 1e-30))
        return worst

    out = {}
    for tag, pert in (("ship", None), ("dz5 x1.01 on 256 columns", {"dz5": (256, 512, 1.01)}),
                      ("dz5 x-1 on 256 columns", {"dz5": (256, 512, -1.0)})):
        g16, _ = _bf16_step(cfg2_batch, perturb=pert, pool_rows=rows)
        out[tag] = cos_err(g16)
        torch.cuda.empty_cache()
        print(f"cfg2 bf16 gradient 1-cos, fp32 pool rows, {tag}:", {k: round(v, 6) for k, v in out[tag].items()})
    bad = {k: v for k, v in out["ship"].items() if v > POOL_ROWS_TIGHT_BOUND}
    assert not bad, bad
    flipped = {k: v for k, v in out["dz5 x-1 on 256 columns"].items() if v > POOL_ROWS_TIGHT_BOUND}
    assert flipped, "the sign-flip control must fail the bound"
    # the 1 % control moves every tensor's 1 - cos by far less than the bf16 noise (recorded above)
    shift = max(abs(out["dz5 x1.01 on 256 columns"][k] - out["ship"][k]) for k in out["ship"])
    print(f"1 % control: largest change of 1 - cos {shift:.2e}")


# measured at the bench size with the fp32 forward's pool rows (r04, see the test's print), plus
# margin; the routing-dominated bound of test_cfg2_bf16_train_step_tracks_fp32 is 0.56
POOL_ROWS_TIGHT_BOUND = 0.15


def _bf16_step(cfg2_batch, capture=None, perturb=None, pool_rows=None, record_rows=False):
    """One bf16 reference-style step at cfg2; returns (gradients, engine hooks' results)."""
    pts, lab, w = cfg2_batch
    sd = orc.init_params(2, 77)
    x, y = pts.to(DEV), lab.to(DEV).view(-1)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    m = _model(sd, "bf16")
    m.train()
    m.seed_dropout(99)
    eng = m._engine()
    eng.capture, eng.perturb, eng.pool_rows_override = capture, perturb, pool_rows
    eng.record_pool_rows = record_rows
    loss = crit(m(x).contiguous().view(-1, 2), y)
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
    rows = eng.last_pool_rows.clone() if record_rows else None
    eng.capture = eng.perturb = eng.pool_rows_override = eng.last_pool_rows = None
    eng.record_pool_rows = False
    del m, loss
    return grads, rows


def _ulp_check(got, ref):
    """got (bf16) against ref (fp32, the same arithmetic in another order): the fraction of
    elements that differ at all, and of those off by more than one bf16 ulp of ref."""
    g = got.float()
    r = ref.to(torch.bfloat16).float()
    d = (g - r).abs()
    ulp = torch.clamp(r.abs(), min=1e-30) * 2.0 ** -7
    return float((d > 0).float().mean()), float((d > 1.0001 * ulp).float().mean())


def _check_prepool(cap):
    """Recompute the three pre-pool backward kernels' outputs with torch fp32 from the operands
    they read (cap: Engine.capture).  Returns {name: (fraction differing, fraction > 1 ulp)}
    for dz5 / dz4 and the relative L2 error of R."""
    torch.backends.cuda.matmul.allow_tf32 = False
    a5, H, cvec, dz5 = cap["a5"], cap["H"].float(), cap["cvec"], cap["dz5"]
    M = a5.shape[0]
    pool = torch.zeros(M, dtype=torch.bool, device=DEV)
    pool[cap["am"].flatten().long()] = True        # rows carrying max-pool terms: checked apart
    s4, t4 = cap["s4"], cap["t4"]
    y4 = cap["y4"]
    ws_t, h4, c5, dz4 = cap["ws_t"].float(), cap["h4"].float(), cap["c5"], cap["dz4"]
    n_dif = n_ulp = n_dif4 = n_ulp4 = 0.0
    R = torch.zeros(1024, 128, dtype=torch.float64, device=DEV)
    step = 1 << 20
    for i in range(0, M, step):
        a = a5[i:i + step].float()
        v = torch.where(a > 0, a @ H.T + cvec, torch.zeros((), device=DEV))
        keep = ~pool[i:i + step]
        f, u = _ulp_check(dz5[i:i + step][keep], v[keep])
        n_dif += f * int(keep.sum())
        n_ulp += u * int(keep.sum())
        z = y4[i:i + step].float() * s4 + t4
        a4 = torch.relu(z).to(torch.bfloat16).float()
        d5 = dz5[i:i + step].float()
        R += d5.double().T @ a4.double()    # fp64: the kernel's own fp32 sums are what is checked
        v4 = d5 @ ws_t.T + a4 @ h4.T + c5
        v4 = torch.where(z > 0, v4, torch.zeros((), device=DEV))
        f, u = _ulp_check(dz4[i:i + step], v4)
        n_dif4 += f * a.shape[0]
        n_ulp4 += u * a.shape[0]
    npool = int(pool.sum())
    r5 = cap["r5"].double()
    return {"dz5": (n_dif / (M - npool), n_ulp / (M - npool)), "dz4": (n_dif4 / M, n_ulp4 / M),
            "R": float((r5 - R).norm() / R.norm())}


def test_cfg2_bf16_prepool_kernels_same_operands(cfg2_batch):
    """Full-size guard for the pre-pool backward kernels, which the cosine bounds above cannot
    give (bf16 noise through the pool's cancelling sums sets those, see
    test_cfg2_bf16_step_same_pool_rows_tight): global_feat's folded input gradient (dz5 =
    relu mask * (a5 H + c), P:113 at P:254), conv5's R = dz5^T a4 and conv5's folded input
    gradient (dz4), each recomputed by torch in fp32 from the same bf16 operands the kernel read
    in the bench-size step.  Same arithmetic in another summation order: the bf16 outputs agree
    bit for bit except where the fp32 sums straddle a rounding boundary.  Negative control: a
    1 % scale of dz5's columns 256..511 after the kernel (Engine.perturb) must fail it."""
    res = {}
    for tag, pert in (("ship", None), ("dz5 x1.01 on 256 columns", {"dz5": (256, 512, 1.01)})):
        cap = {}
        _bf16_step(cfg2_batch, capture=cap, perturb=pert)
        res[tag] = _check_prepool(cap)
        del cap
        torch.cuda.empty_cache()
        print(f"cfg2 pre-pool kernels, {tag}: {res[tag]}")
    ok = res["ship"]
    # measured r05: dz5 1.1e-4 differing / 6.6e-6 beyond one ulp (values whose fp32 sums
    # cancel to far below their terms), dz4 3.2e-5 / 1.9e-6, R 6.8e-5 (fp32 sums over 8.4M rows)
    assert ok["dz5"][0] < 2e-3 and ok["dz5"][1] < 1e-4, ok
    assert ok["dz4"][0] < 2e-3 and ok["dz4"][1] < 1e-4, ok
    assert ok["R"] < 2e-4, ok
    bad = res["dz5 x1.01 on 256 columns"]
    assert bad["dz5"][1] > 0.05, bad   # the simulated 1 % error is caught

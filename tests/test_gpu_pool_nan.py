"""The global max-pool (P:114, ``torch.max(x, 2)``) on non-finite input.

torch.max over a dim propagates NaN: the value is NaN and the index is the first NaN's row.
The pool kernels (csrc/gemm_glds.hip forward epilogue, gemm_nt / gemm_big epilogues,
pcs_pool_finalize's merge) follow that order (common.h ``pool_max_wins``), and
pcs_pool_finalize never hands on the "no candidate" sentinel as a row: the backward's
pool kernels (pcs_pool_rows_add, pcs_gram_wgrad) read the row it names.

* kernel level: a5 with one NaN element (that row's y is NaN in every channel) or a NaN
  column (every row of the scene NaN), other scenes finite: values / rows against torch's
  own max / min over the same fp64 y, then pcs_pool_rows_add with those rows and with
  out-of-range rows (skipped, no fault);
* step level: a NaN written into a5 inside the training step (Engine.perturb): the step
  completes, the loss is NaN, and every argmax row is the scene's first row -- what the
  reference gives, since bn_global's batch statistics are NaN there and so is every x."""
import ctypes as ct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _variant(L, v):
    return {"glds": (L.BF16, torch.bfloat16, 0), "glds_signed": (L.BF16, torch.bfloat16, L.FLAG_POOL_SIGNED_W),
            "noglds": (L.BF16, torch.bfloat16, L.FLAG_NO_GLDS), "fp32": (L.F32, torch.float32, 0)}[v]


def _torch_pool(y, gamma, B, N):
    """torch.max / torch.min over each scene's rows (first NaN / first extremum), by gamma's sign."""
    yb = y.view(B, N, -1)
    mx, ix = torch.max(yb, 1)
    mn, jx = torch.min(yb, 1)
    pos = (gamma > 0)[None, :]
    val = torch.where(pos, mx, mn)
    row = torch.where(pos, ix, jx) + torch.arange(B)[:, None] * N
    return val, row


@pytest.mark.parametrize("variant", ["glds", "glds_signed", "noglds", "fp32"])
@pytest.mark.parametrize("where", ["element", "column"])
def test_pool_nan_propagates(variant, where):
    import pcs_amd._lib as L
    dt, tdt, flags = _variant(L, variant)
    B, N, K, cps = 3, 256 * 5 + 77, 512, 2
    g = torch.Generator().manual_seed(5)
    A = torch.relu(torch.randn(B * N, K, generator=g))
    if where == "element":
        A[N + 700, 33] = float("nan")          # scene 1, one row: y[row, :] is NaN
    else:
        A[N:2 * N, 33] = float("nan")          # scene 1, every row NaN
    A = A.to(tdt)
    W = (torch.randn(K, K, generator=g) * 0.05).to(tdt)
    gamma = torch.randn(K, generator=g)
    Wd = W.to(DEV)
    if flags & L.FLAG_POOL_SIGNED_W:
        Ws = torch.empty_like(Wd)
        L.call("pcs_sign_rows", L.ptr(Wd), dt, K, K, L.ptr(gamma.to(DEV)), L.ptr(Ws), L.stream_ptr())
        Wd = Ws
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=K, dtype=dt, prologue=L.PRO_RAW, epilogue=L.EPI_FWD,
                   chunks_per_scene=cps, flags=flags)
    assert L.load().pcs_gemm_geometry(ct.byref(a)) > 0
    Ad, gd = A.to(DEV), gamma.to(DEV)
    pool = torch.empty(B * a.chunks_per_scene, K, 4, device=DEV)
    a.A, a.W, a.C, a.pool, a.es = Ad.data_ptr(), Wd.data_ptr(), None, pool.data_ptr(), gd.data_ptr()
    s = L.stream_ptr()
    L.call("pcs_gemm", ct.byref(a), s)
    # finite BN coefficients (as if the statistics had come from elsewhere): the pool alone decides
    scale, shift = gd.clone(), torch.zeros(K, device=DEV)
    gp, ysel = torch.empty(B, K, device=DEV), torch.empty(B, K, device=DEV)
    am = torch.empty(B, K, dtype=torch.int32, device=DEV)
    L.call("pcs_pool_finalize", L.ptr(pool), B, N, K, a.chunks_per_scene, L.ptr(scale), L.ptr(shift),
           L.ptr(gp), L.ptr(am), L.ptr(ysel), s)
    torch.cuda.synchronize()
    y = A.double() @ W.double().T
    val, row = _torch_pool(y, gamma, B, N)
    got, rows = ysel.cpu().double(), am.cpu().long()
    nan_ref = torch.isnan(val)
    assert nan_ref[1].all() and not nan_ref[0].any() and not nan_ref[2].any()
    assert torch.equal(torch.isnan(got), nan_ref)
    assert torch.equal(rows[1], row[1]), (rows[1][:8], row[1][:8])        # the first NaN's row
    scl = y[torch.isfinite(y)].abs().max().item()
    tol = 4e-3 if variant == "noglds" else 1e-5
    fin = ~nan_ref
    assert float((got[fin] - val[fin]).abs().max()) < tol * scl
    assert torch.isnan(gp.cpu()[1]).all()                     # relu keeps the NaN, as torch.relu
    assert torch.isfinite(gp.cpu()[[0, 2]]).all()
    lo = (torch.arange(B) * N)[:, None]
    assert ((rows >= lo) & (rows < lo + N)).all()

    # the backward's sparse rows term on those rows, then on rows outside the scenes: no fault
    if variant == "fp32":
        dz = torch.zeros(B * N, K, device=DEV)
        dzt, ypt = L.F32, L.F32
    else:
        dz = torch.zeros(B * N, K, dtype=torch.bfloat16, device=DEV)
        dzt, ypt = L.BF16, L.BF16
    coef = torch.ones(B, K, device=DEV)
    Wp = (torch.randn(K, K, generator=g) * 0.05).to(DEV)
    for idx in (am, torch.full((B, K), 0x7fffffff, dtype=torch.int32, device=DEV),
                torch.full((B, K), -5, dtype=torch.int32, device=DEV)):
        L.call("pcs_pool_rows_add", L.ptr(dz), dzt, L.ptr(Ad), ypt, B, N, K, L.ptr(idx), L.ptr(coef),
               L.ptr(Wp), K, K, None, 0, s)
        torch.cuda.synchronize()
    assert torch.isfinite(dz.float()[:N]).all()


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp8"])
def test_step_with_nan_activation(dtype):
    from pcs_amd.model import PointNetSegmentation
    from pcs_amd.train import FusedTrainStep
    B, N, C = 2, 256 * 5 + 33, 2
    torch.manual_seed(3)
    m = PointNetSegmentation(C, compute_dtype=dtype).to(DEV)
    step = FusedTrainStep(m)
    x = torch.randn(B, N, 4, device=DEV)
    y = torch.randint(0, C, (B, N), device=DEV)
    eng = m._engine()
    eng.record_pool_rows = True
    eng.perturb = {"a5": (N + 400, 17, float("nan"))}
    try:
        loss = step(x, y)
        torch.cuda.synchronize()
        rows = eng.last_pool_rows.cpu().long()
    finally:
        eng.perturb, eng.record_pool_rows, eng.last_pool_rows = None, False, None
    assert torch.isnan(loss.cpu()).item()
    # the reference: bn_global's batch statistics are NaN, so is every x, and torch.max's
    # first NaN is each scene's first row
    assert torch.equal(rows, (torch.arange(B) * N)[:, None].expand(B, 1024))
    # a clean step afterwards on fresh weights runs (the device is healthy)
    m2 = PointNetSegmentation(C, compute_dtype=dtype).to(DEV)
    l2 = FusedTrainStep(m2)(x, y)
    torch.cuda.synchronize()
    assert np.isfinite(l2.item())

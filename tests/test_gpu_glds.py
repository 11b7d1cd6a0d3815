"""The global_feat GEMMs on the stored a5 = relu(bn5(y5)) (csrc/gemm_glds.hip: LDS-DMA
256x256 kernel; the generic kernel with FLAG_NO_GLDS / fp32) against torch fp32 on the same
operands, through the C ABI:

* forward epilogue: BN statistics + max-pool partials of y = a5 W^T with nothing stored,
  finalised by pcs_bn_fwd_finalize / pcs_pool_finalize (mean / variance / per-scene max);
* folded input-gradient epilogue: dz = (a5 > 0) * (a5 H + c + max-pool rows), S1 = sum dz;
* EPI_BNRELU (conv5's second pass): relu((A W^T + b) * s + t) stored.

Ragged scenes (the last row tile of a scene partial) and several tiles per workgroup chunk
exercise the cross-tile pipeline; duplicate max-pool rows exercise the sparse sums."""
import ctypes as ct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _args(L, B, N, K, Nc, dt, pro, epi, flags, cps=0):
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=dt, prologue=pro, epilogue=epi,
                   chunks_per_scene=cps, flags=flags)
    rpc = L.load().pcs_gemm_geometry(ct.byref(a))
    assert rpc > 0
    return a, rpc


def _variant(L, v):
    return {"glds": (L.BF16, torch.bfloat16, 0), "noglds": (L.BF16, torch.bfloat16, L.FLAG_NO_GLDS),
            "fp32": (L.F32, torch.float32, 0)}[v]


@pytest.mark.parametrize("variant", ["glds", "noglds", "fp32"])
@pytest.mark.parametrize("B,N,cps", [(2, 256 * 7 + 77, 2), (1, 200, 0), (3, 1024, 1)])
def test_forward_stats_and_pool(variant, B, N, cps):
    import pcs_amd._lib as L
    dt, tdt, flags = _variant(L, variant)
    K = Nc = 512
    g = torch.Generator().manual_seed(B * 1000 + N)
    A = torch.relu(torch.randn(B * N, K, generator=g)).to(tdt).to(DEV)
    W = (torch.randn(Nc, K, generator=g) * 0.05).to(tdt).to(DEV)
    a, rpc = _args(L, B, N, K, Nc, dt, L.PRO_RAW, L.EPI_FWD, flags, cps)
    nch = B * a.chunks_per_scene
    st = torch.empty(nch, Nc, 2, device=DEV)
    pool = torch.empty(nch, Nc, 4, device=DEV)
    gamma = torch.randn(Nc, generator=g).to(DEV)       # signs pick max or min in the pool
    a.A, a.W, a.C, a.stats, a.pool = A.data_ptr(), W.data_ptr(), None, st.data_ptr(), pool.data_ptr()
    a.es = gamma.data_ptr()                            # EPI_FWD: only sign(es) matters (pool side)
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    beta = torch.zeros(Nc, device=DEV)
    mean, rstd, scale, shift = (torch.empty(Nc, device=DEV) for _ in range(4))
    ssum = torch.empty(B, Nc, device=DEV)
    s = L.stream_ptr()
    L.call("pcs_bn_fwd_finalize", L.ptr(st), B, N, Nc, a.chunks_per_scene, rpc, L.ptr(gamma), L.ptr(beta),
           None, None, None, 0.1, 1e-5, 0, L.ptr(mean), L.ptr(rstd), L.ptr(scale), L.ptr(shift), L.ptr(ssum), s)
    gp = torch.empty(B, Nc, device=DEV)
    am = torch.empty(B, Nc, dtype=torch.int32, device=DEV)
    ysel = torch.empty(B, Nc, device=DEV)
    L.call("pcs_pool_finalize", L.ptr(pool), B, N, Nc, a.chunks_per_scene, L.ptr(scale), L.ptr(shift),
           L.ptr(gp), L.ptr(am), L.ptr(ysel), s)
    torch.cuda.synchronize()
    y = (A.double() @ W.double().T)
    ym, yv = y.mean(0), y.var(0, unbiased=False)
    scl = y.abs().max().item()
    # the 256x256 register-staged kernel (noglds) takes its statistics from the bf16-rounded
    # stored tile; the LDS-DMA and fp32 kernels from the fp32 accumulators
    mtol, vtol = (5e-4, 5e-3) if variant == "noglds" else (1e-5, 1e-4)
    err_m = float((mean.double() - ym).abs().max())
    assert err_m < mtol * scl, err_m
    var = 1.0 / rstd.double() ** 2 - 1e-5
    err_v = float(((var - yv).abs() / yv).max())
    assert err_v < vtol, err_v
    assert abs(ssum.double().sum().item() - y.sum().item()) < mtol * y.abs().sum().item()
    yb = y.view(B, N, Nc)
    sgn = torch.where(gamma > 0, 1.0, -1.0).double()
    ext = (yb * sgn).max(1).values * sgn                   # max for gamma > 0, min for gamma < 0
    ptol = 4e-3 if variant == "noglds" else 1e-5          # noglds: bf16-rounded candidates
    assert float((ysel.double() - ext).abs().max()) < ptol * scl
    rows = am.long() - (torch.arange(B, device=DEV) * N)[:, None]
    assert ((rows >= 0) & (rows < N)).all()
    at = yb.gather(1, rows[:, None, :]).squeeze(1)         # value at the reported row
    assert float((at - ext).abs().max()) < ptol * scl


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("B,N,cps", [(2, 256 * 7 + 77, 2), (3, 256 * 3, 1)])
def test_forward_pool_signed_w(fp8, B, N, cps):
    """PCS_FLAG_POOL_SIGNED_W: with W's rows multiplied by sign(gamma) (pcs_sign_rows, exact)
    the LDS-DMA forward's max-pool partials match the unsigned kernel's (which multiplies by
    the sign in its epilogue); a signed W with statistics is refused."""
    import pcs_amd._lib as L
    K = Nc = 512
    g = torch.Generator().manual_seed(31 + N)
    A = torch.relu(torch.randn(B * N, K, generator=g))
    W = torch.randn(Nc, K, generator=g) * 0.05
    gamma = torch.randn(Nc, generator=g).to(DEV)
    flags, extra = 0, {}
    if fp8:
        A = A.clamp(max=448.0).to(torch.float8_e4m3fn).view(torch.uint8).to(DEV)
        Wq = torch.empty(Nc, K, dtype=torch.uint8, device=DEV)
        wsc = torch.empty(Nc, dtype=torch.uint8, device=DEV)
        L.call("pcs_quant_fp8_rows", L.ptr(W.to(DEV)), Nc, K, K, L.ptr(Wq), L.ptr(wsc), None, L.stream_ptr())
        W, wdt, flags, extra = Wq, L.FP8, L.FLAG_AW_FP8, {"w_scale": wsc}
    else:
        A, W, wdt = A.to(torch.bfloat16).to(DEV), W.to(torch.bfloat16).to(DEV), L.BF16
    Ws = torch.empty_like(W)
    L.call("pcs_sign_rows", L.ptr(W), wdt, Nc, K, L.ptr(gamma), L.ptr(Ws), L.stream_ptr())
    flip = 0x80 if fp8 else -0x8000                      # the sign bit of a byte / an int16
    Wi = W.view(torch.uint8) if fp8 else W.view(torch.int16)
    Wsi = Ws.view(torch.uint8) if fp8 else Ws.view(torch.int16)
    ref = torch.where((gamma < 0)[:, None], Wi ^ flip, Wi)
    assert torch.equal(Wsi, ref)
    pools = []
    for w, fl in ((W, flags), (Ws, flags | L.FLAG_POOL_SIGNED_W)):
        a, _ = _args(L, B, N, K, Nc, L.BF16, L.PRO_RAW, L.EPI_FWD, fl, cps)
        pool = torch.full((B * a.chunks_per_scene, Nc, 4), float("nan"), device=DEV)
        a.A, a.W, a.C, a.pool, a.es = A.data_ptr(), w.data_ptr(), None, pool.data_ptr(), gamma.data_ptr()
        for k, v in extra.items():
            setattr(a, k, v.data_ptr())
        L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
        pools.append(pool)
    torch.cuda.synchronize()
    # bitwise (the untouched slots hold NaN-pattern argument sentinels)
    # the extremum pcs_pool_finalize reads (max where gamma > 0, min where gamma < 0) and its
    # row: the MFMA's fp32 sums of negated products are not always bitwise the negated sums
    # (measured: one value in 4096 off by 2 ulp), so values agree to 1e-6 relative, rows exactly
    val = torch.where(gamma[None, :] > 0, pools[0][..., 0], pools[0][..., 2])
    vals = torch.where(gamma[None, :] > 0, pools[1][..., 0], pools[1][..., 2])
    row = torch.where(gamma[None, :] > 0, pools[0][..., 1], pools[0][..., 3]).view(torch.int32)
    rows = torch.where(gamma[None, :] > 0, pools[1][..., 1], pools[1][..., 3]).view(torch.int32)
    assert torch.isfinite(val).all() and torch.equal(row, rows)
    assert float(((val - vals).abs() / val.abs()).max()) <= 1e-6
    st = torch.empty(B * a.chunks_per_scene, Nc, 2, device=DEV)
    a.stats = st.data_ptr()
    with pytest.raises(L.PcsError):
        L.call("pcs_gemm", ct.byref(a), L.stream_ptr())


@pytest.mark.parametrize("variant", ["glds", "noglds", "fp32"])
@pytest.mark.parametrize("B,N,cps", [(2, 256 * 5 + 33, 2), (1, 300, 0)])
def test_folded_dgrad_sparse_mask_s1(variant, B, N, cps):
    import pcs_amd._lib as L
    dt, tdt, flags = _variant(L, variant)
    K = 512
    g = torch.Generator().manual_seed(7 + N)
    A = torch.relu(torch.randn(B * N, K, generator=g)).to(tdt).to(DEV)
    H = (torch.randn(K, K, generator=g) * 0.05).to(tdt).to(DEV)
    c = (torch.randn(K, generator=g) * 0.1).to(DEV)
    Pc = 256
    Wsp = (torch.randn(Pc, K, generator=g) * 0.1).to(DEV)
    am = torch.randint(0, N, (B, Pc), generator=g)
    am[:, 1] = am[:, 0]                                   # two channels on one row
    am[:, 2] = N - 1                                      # the scene's last (ragged-tile) row
    am = (am + torch.arange(B)[:, None] * N).int().to(DEV)
    sp = torch.randn(B, Pc, generator=g).to(DEV)
    a, rpc = _args(L, B, N, K, K, dt, L.PRO_RAW, L.EPI_DGRAD, flags, cps)
    nch = B * a.chunks_per_scene
    st = torch.empty(nch, K, 2, device=DEV)
    out = torch.empty(B * N, K, dtype=tdt, device=DEV)
    a.A, a.W, a.C, a.Yp, a.bias = A.data_ptr(), H.data_ptr(), out.data_ptr(), A.data_ptr(), c.data_ptr()
    a.stats = st.data_ptr()
    if variant == "glds":
        # the LDS-DMA kernel leaves the max-pool rows to pcs_pool_rows_add
        L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
        L.call("pcs_pool_rows_add", L.ptr(out), dt, L.ptr(A), dt, B, N, K, L.ptr(am), L.ptr(sp), L.ptr(Wsp), K, Pc,
               L.ptr(st), a.chunks_per_scene, L.stream_ptr())
    else:
        a.pool_idx, a.pool_coef, a.pool_w, a.pool_ldw, a.pool_c = am.data_ptr(), sp.data_ptr(), Wsp.data_ptr(), K, Pc
        L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    v = A.double() @ H.double().T + c.double()
    for b in range(B):
        for q in range(Pc):
            v[am[b, q].long()] += sp[b, q].double() * Wsp[q].double()
    dz = torch.where(A.double() > 0, v, torch.zeros_like(v))
    tol = 1e-5 if variant == "fp32" else 1e-2
    err = float((out.double() - dz).abs().max())
    assert err < tol * dz.abs().max().item(), err
    s1 = st[..., 0].double().sum(0)
    err = float((s1 - dz.sum(0)).abs().max())
    assert err < (1e-5 if variant == "fp32" else 1e-3) * dz.abs().sum(0).max().item(), err


@pytest.mark.parametrize("variant", ["big", "fp32"])
def test_bnrelu_epilogue(variant):
    import pcs_amd._lib as L
    dt, tdt = (L.BF16, torch.bfloat16) if variant == "big" else (L.F32, torch.float32)
    B, N, K, Nc = 2, 700, 128, 1024
    g = torch.Generator().manual_seed(3)
    Y = torch.randn(B * N, K, generator=g).to(tdt).to(DEV)
    ps = (torch.rand(K, generator=g) + 0.5).to(DEV)
    pt = (torch.randn(K, generator=g) * 0.2).to(DEV)
    W = (torch.randn(Nc, K, generator=g) * 0.1).to(tdt).to(DEV)
    bias = (torch.randn(Nc, generator=g) * 0.1).to(DEV)
    es = torch.randn(Nc, generator=g).to(DEV)
    et = (torch.randn(Nc, generator=g) * 0.3).to(DEV)
    a, _ = _args(L, B, N, K, Nc, dt, L.PRO_BNRELU, L.EPI_BNRELU, 0)
    out = torch.empty(B * N, Nc, dtype=tdt, device=DEV)
    a.A, a.W, a.C, a.pa, a.pb, a.bias, a.es, a.et = (Y.data_ptr(), W.data_ptr(), out.data_ptr(), ps.data_ptr(),
                                                      pt.data_ptr(), bias.data_ptr(), es.data_ptr(), et.data_ptr())
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    x = torch.relu(Y.float() * ps + pt).to(tdt).double()     # the prologue rounds to dtype
    ref = torch.relu((x @ W.double().T + bias.double()) * es.double() + et.double())
    tol = 1e-5 if variant == "fp32" else 1e-2
    err = float((out.double() - ref).abs().max())
    assert err < tol * ref.abs().max().item(), err


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_bn_stats_from_gram(dtype):
    """bn5 statistics of y = a W^T from the Gram of a (bf16 path): the per-scene partials
    finalise to the batch mean / biased variance of y."""
    import pcs_amd._lib as L
    dt, tdt = (L.BF16, torch.bfloat16) if dtype == "bf16" else (L.F32, torch.float32)
    g = torch.Generator().manual_seed(5)
    B, N, Cin, C = 3, 1000, 128, 512
    a = torch.relu(torch.randn(B * N, Cin, generator=g) + 0.3).to(tdt).to(DEV)
    W = (torch.randn(C, Cin, generator=g) * 0.08).to(tdt).to(DEV)
    ad = a.double()
    G = (ad.T @ ad).float()
    S = ad.sum(0).float()
    st = torch.empty(B, C, 2, device=DEV)
    L.call("pcs_bn_stats_from_gram", L.ptr(G), L.ptr(S), B * N, L.ptr(W), dt, Cin, C, Cin, B, L.ptr(st),
           L.stream_ptr())
    mean, rstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    ones, zeros = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    L.call("pcs_bn_fwd_finalize", L.ptr(st), B, N, C, 1, N, L.ptr(ones), L.ptr(zeros), None, None, None,
           0.1, 1e-5, 0, L.ptr(mean), L.ptr(rstd), L.ptr(scale), L.ptr(shift), None, L.stream_ptr())
    torch.cuda.synchronize()
    y = ad @ W.double().T
    err_m = float((mean.double() - y.mean(0)).abs().max() / y.std(0).min())
    var = 1.0 / rstd.double() ** 2 - 1e-5
    err_v = float(((var - y.var(0, unbiased=False)) / y.var(0, unbiased=False)).abs().max())
    assert err_m < 1e-5 and err_v < 1e-4, (err_m, err_v)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_bn_stats_from_gram_scenes(dtype):
    """bn_global statistics of y = a W^T (bf16 / fp8 path) from the Gram of a and per-scene
    column sums: the partials finalise to the batch mean / biased variance and to exact
    per-scene sums of y, with scenes of deliberately different means."""
    import pcs_amd._lib as L
    dt, tdt = (L.BF16, torch.bfloat16) if dtype == "bf16" else (L.F32, torch.float32)
    g = torch.Generator().manual_seed(6)
    B, N, C = 3, 1000, 256
    shift_b = torch.tensor([0.0, 0.5, -0.2]).repeat_interleave(N)[:, None]
    a = torch.relu(torch.randn(B * N, C, generator=g) + 0.3 + shift_b).to(tdt).to(DEV)
    W = (torch.randn(C, C, generator=g) * 0.06).to(tdt).to(DEV)
    ad = a.double()
    G = (ad.T @ ad).float()
    Sb = ad.reshape(B, N, C).sum(1).float().contiguous()
    nbytes = L.load().pcs_bn_stats_from_gram_scenes_workspace(C, C)
    assert nbytes >= (C // 64) * C * 8
    ws = torch.empty(nbytes // 8, dtype=torch.float64, device=DEV)
    st = torch.empty(B, C, 2, device=DEV)
    L.call("pcs_bn_stats_from_gram_scenes", L.ptr(G), L.ptr(Sb), N, L.ptr(W), dt, C, C, C, B, L.ptr(ws), nbytes,
           L.ptr(st), L.stream_ptr())
    mean, rstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    ssum = torch.empty(B, C, device=DEV)
    ones, zeros = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    L.call("pcs_bn_fwd_finalize", L.ptr(st), B, N, C, 1, N, L.ptr(ones), L.ptr(zeros), None, None, None,
           0.1, 1e-5, 0, L.ptr(mean), L.ptr(rstd), L.ptr(scale), L.ptr(shift), L.ptr(ssum), L.stream_ptr())
    torch.cuda.synchronize()
    y = ad @ W.double().T
    sd = y.std(0).min()
    err_m = float((mean.double() - y.mean(0)).abs().max() / sd)
    var = 1.0 / rstd.double() ** 2 - 1e-5
    err_v = float(((var - y.var(0, unbiased=False)) / y.var(0, unbiased=False)).abs().max())
    err_s = float((ssum.double() - y.reshape(B, N, C).sum(1)).abs().max() / (N * sd))
    assert err_m < 1e-5 and err_v < 1e-4 and err_s < 1e-5, (err_m, err_v, err_s)
    with pytest.raises(L.PcsError):
        L.call("pcs_bn_stats_from_gram_scenes", L.ptr(G), L.ptr(Sb), N, L.ptr(W), dt, C, C, C, B, L.ptr(ws),
               nbytes - 8, L.ptr(st), L.stream_ptr())


def test_bn_s2_from_r():
    """S2 = rstd (sum_k W R - mean S1), rewritten into the (S1, S2) partials (chunk 0 total)."""
    import pcs_amd._lib as L
    g = torch.Generator().manual_seed(11)
    C, Cin, nch = 256, 128, 5
    R = torch.randn(C, Cin, generator=g).to(DEV)
    W = torch.randn(C, Cin, generator=g).to(DEV)
    mean = torch.randn(C, generator=g).to(DEV)
    rstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
    st = torch.randn(nch, C, 2, generator=g).to(DEV)
    s1 = st[..., 0].double().sum(0)
    L.call("pcs_bn_s2_from_r", L.ptr(st), nch, C, L.ptr(R), L.ptr(W), L.F32, Cin, Cin, L.ptr(mean), L.ptr(rstd),
           L.stream_ptr())
    torch.cuda.synchronize()
    ref = rstd.double() * ((W.double() * R.double()).sum(1) - mean.double() * s1)
    err = float((st[0, :, 1].double() - ref).abs().max())
    assert err < 1e-5 * ref.abs().max().item(), err
    assert (st[1:, :, 1] == 0).all()
    assert torch.equal(st[..., 0].double().sum(0), s1)


@pytest.mark.parametrize("mode", ["fwd", "dgrad"])
def test_glds_deterministic_and_tail_exact(mode):
    """The LDS-DMA kernel at the bench shape (K = Ncols = 1024), several row tiles per chunk
    and a ragged last tile: repeated launches on identical inputs are bitwise identical, and
    the chunk's last row tile (the one whose final K-tiles run with no loads left to issue,
    where the pipeline's counted waits shrink) matches torch like every other tile."""
    import pcs_amd._lib as L
    B, N, K = 2, 256 * 9 + 50, 1024
    g = torch.Generator().manual_seed(404)
    A = torch.relu(torch.randn(B * N, K, generator=g)).to(torch.bfloat16).to(DEV)
    W = (torch.randn(K, K, generator=g) * 0.03).to(torch.bfloat16).to(DEV)
    epi = L.EPI_FWD if mode == "fwd" else L.EPI_DGRAD
    a, _ = _args(L, B, N, K, K, L.BF16, L.PRO_RAW, epi, 0, 2)
    nch = B * a.chunks_per_scene
    runs = []
    for _ in range(12):
        st = torch.full((nch, K, 2), float("nan"), device=DEV)
        a.A, a.W, a.stats = A.data_ptr(), W.data_ptr(), st.data_ptr()
        if mode == "fwd":
            pool = torch.full((nch, K, 4), float("nan"), device=DEV)
            gamma = torch.ones(K, device=DEV)
            a.C, a.pool, a.es = None, pool.data_ptr(), gamma.data_ptr()
            L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
            runs.append((st, pool))
        else:
            out = torch.full((B * N, K), float("nan"), dtype=torch.bfloat16, device=DEV)
            a.C, a.Yp = out.data_ptr(), A.data_ptr()
            L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
            runs.append((st, out))
    torch.cuda.synchronize()
    for r in runs[1:]:
        for x, y in zip(runs[0], r):
            assert torch.equal(x.view(torch.int32) if x.dtype == torch.float32 else x.view(torch.int16),
                               y.view(torch.int32) if y.dtype == torch.float32 else y.view(torch.int16))
    y = A.double() @ W.double().T
    if mode == "fwd":
        st, pool = runs[0]
        yb = y.view(B, N, K)
        ext = yb.max(1).values
        # per-chunk maxima: the chunk holding each scene's last tile is the last one
        cps = a.chunks_per_scene
        pmax = pool.view(B, cps, K, 4)[..., 0].max(1).values.double()
        assert float((pmax - ext).abs().max()) < 1e-5 * y.abs().max().item()
    else:
        st, out = runs[0]
        dz = torch.where(A.double() > 0, y, torch.zeros_like(y))
        for b in range(B):   # every scene's last (ragged) row tile, then the whole output
            sl = slice(b * N + (N // 256) * 256, (b + 1) * N)
            err = float((out[sl].double() - dz[sl]).abs().max())
            assert err < 1e-2 * dz.abs().max().item(), (b, err)
        err = float((out.double() - dz).abs().max())
        assert err < 1e-2 * dz.abs().max().item(), err


@pytest.mark.parametrize("signed", [False, True])
@pytest.mark.parametrize("data", ["ties", "trend"])
def test_forward_pool_strided_tile_order(signed, data):
    """Chunks of more than 97 row tiles visit their tiles in a strided order (gemm_glds.hip): the
    max-pool must still report the first maximum in row order.  'ties': 37 distinct rows repeated
    across the scene (every maximum is tied hundreds of times, identical bits); 'trend': values
    rising along the rows (the spatially ordered case the order is for)."""
    import pcs_amd._lib as L
    B, N, K, cps = 1, 256 * 100 + 51, 512, 1
    g = torch.Generator().manual_seed(11)
    if data == "ties":
        # tile 0 (visited first) holds zero rows, the first occurrences of the 37 rows sit in tile 1
        # (visited late), duplicates in every later tile (tile P is visited second)
        base = torch.relu(torch.randn(37, K, generator=g))
        A = base[(torch.arange(N) * 7) % 37]
        A[:256] = 0
    else:
        A = torch.relu(torch.randn(N, K, generator=g) + torch.linspace(0, 3, N)[:, None])
    A = A.to(torch.bfloat16)
    W = (torch.randn(K, K, generator=g) * 0.05).to(torch.bfloat16)
    gamma = torch.randn(K, generator=g)
    Wd = W.to(DEV)
    if signed:
        Ws = torch.empty_like(Wd)
        L.call("pcs_sign_rows", L.ptr(Wd), L.BF16, K, K, L.ptr(gamma.to(DEV)), L.ptr(Ws), L.stream_ptr())
        Wd = Ws
    a, rpc = _args(L, B, N, K, K, L.BF16, L.PRO_RAW, L.EPI_FWD, L.FLAG_POOL_SIGNED_W if signed else 0, cps)
    assert rpc // 256 > 97                                   # the strided order is in use
    Ad, gd = A.to(DEV), gamma.to(DEV)
    pool = torch.empty(B * a.chunks_per_scene, K, 4, device=DEV)
    a.A, a.W, a.C, a.pool, a.es = Ad.data_ptr(), Wd.data_ptr(), None, pool.data_ptr(), gd.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    y = A.double() @ W.double().T
    sgn = torch.where(gamma > 0, 1.0, -1.0).double()
    pl = pool.cpu()
    val = torch.where(gamma > 0, pl[0, :, 0], pl[0, :, 2]).double()
    row = torch.where(gamma > 0, pl[0, :, 1], pl[0, :, 3]).view(torch.int32).long()
    ext = (y * sgn).max(0).values * sgn
    scl = y.abs().max().item()
    assert float((val - ext).abs().max()) < 1e-5 * scl
    at = y.gather(0, row[None, :]).squeeze(0)
    assert float((at - ext).abs().max()) < 1e-5 * scl
    if data == "ties":   # exact: the first row, in row order, holding the extremum
        yb = y * sgn
        first = (yb == yb.max(0).values).double().argmax(0)   # argmax returns the first maximum
        assert torch.equal(row, first)

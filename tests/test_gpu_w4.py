"""The four-wave 32x32x16 LDS-DMA kernel for global_feat's bf16 GEMMs (csrc/gemm_w4.hip) through
the C ABI, against torch fp64 on the same bf16 operands and against the 8-wave kernel
(gemm_glds.hip, the default; w4 is opt-in by PCS_FLAG_W4) on identical inputs:

* folded input gradient (P:113 at P:254): dz = (a5 > 0) * (a5 H + c), bf16, the row tile's
  stores deferred into the next tile's K-tiles 1..4, the ragged last tile of a scene;
* forward max-pool on sign-folded W rows (P:113-114, PCS_FLAG_POOL_SIGNED_W): per-chunk
  (max, first argmax row) of sgn * y, strided tile order, several tiles per chunk;
* bitwise repeatability, and the applicability rules (statistics / fp8 go elsewhere)."""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _args(L, B, N, K, Nc, epi, flags, cps=0):
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=L.PRO_RAW, epilogue=epi,
                   chunks_per_scene=cps, flags=flags)
    rpc = L.load().pcs_gemm_geometry(ct.byref(a))
    assert rpc > 0
    return a, rpc


def _dgrad(L, A, H, c, B, N, flags, cps):
    K = A.shape[1]
    a, _ = _args(L, B, N, K, K, L.EPI_DGRAD, flags, cps)
    out = torch.full((B * N, K), float("nan"), dtype=torch.bfloat16, device=DEV)
    a.A, a.W, a.C, a.Yp, a.bias = A.data_ptr(), H.data_ptr(), out.data_ptr(), A.data_ptr(), c.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    return out


@pytest.mark.parametrize("B,N,K,cps", [(2, 256 * 5 + 33, 512, 2), (1, 300, 512, 0), (2, 256 * 9, 1024, 3),
                                       (1, 256 * 3 + 255, 384, 1)])
def test_dgrad_masked_bias(B, N, K, cps):
    import pcs_amd._lib as L
    g = torch.Generator().manual_seed(11 + N + K)
    A = torch.relu(torch.randn(B * N, K, generator=g)).to(torch.bfloat16)
    A[::7, 3] = -0.0                                  # -0 is not > 0 (the mask is a5 > 0)
    A = A.to(DEV)
    H = (torch.randn(K, K, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    c = (torch.randn(K, generator=g) * 0.1 + 1e-3 * torch.rand(K, generator=g)).to(DEV)
    out = _dgrad(L, A, H, c, B, N, L.FLAG_W4, cps)
    old = _dgrad(L, A, H, c, B, N, 0, cps)
    torch.cuda.synchronize()
    v = A.double() @ H.double().T + c.double()
    dz = torch.where(A.double() > 0, v, torch.zeros_like(v))
    assert torch.isfinite(out.float()).all()
    err = float((out.double() - dz).abs().max())
    assert err < 1e-2 * dz.abs().max().item(), err
    # masked entries are exact zeros; the bf16 rounding of the fp32 sums matches the 8-wave
    # kernel's except where the two MFMA shapes' fp32 sums straddle a rounding boundary
    assert torch.equal(out[A <= 0].float(), torch.zeros_like(out[A <= 0].float()))
    same = (out.view(torch.int16) == old.view(torch.int16)).double().mean().item()
    assert same > 0.97, same


def test_dgrad_bias_exact():
    """The accumulators start from the bias through an MFMA of its three-way bf16 split against
    ones: with H = 0 the output is round_bf16(c) exactly on every unmasked entry."""
    import pcs_amd._lib as L
    B, N, K = 1, 256 * 2 + 17, 512
    g = torch.Generator().manual_seed(5)
    A = torch.relu(torch.randn(B * N, K, generator=g)).to(torch.bfloat16).to(DEV)
    H = torch.zeros(K, K, dtype=torch.bfloat16, device=DEV)
    c = (torch.randn(K, generator=g) * 3.0).to(DEV)
    out = _dgrad(L, A, H, c, B, N, L.FLAG_W4, 0)
    torch.cuda.synchronize()
    ref = torch.where(A > 0, c.to(torch.bfloat16)[None, :].expand(B * N, K), torch.zeros_like(A))
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))


def _pool(L, A, Ws, gamma, B, N, flags, cps):
    K, Nc = A.shape[1], Ws.shape[0]
    a, rpc = _args(L, B, N, K, Nc, L.EPI_FWD, flags | L.FLAG_POOL_SIGNED_W, cps)
    pool = torch.full((B * a.chunks_per_scene, Nc, 4), float("nan"), device=DEV)
    a.A, a.W, a.C, a.pool, a.es = A.data_ptr(), Ws.data_ptr(), None, pool.data_ptr(), gamma.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    _pool.rpc = rpc   # rows per chunk (whole row tiles: pcs_gemm_geometry)
    return pool


@pytest.mark.parametrize("B,N,K,cps", [(2, 256 * 7 + 77, 512, 2), (3, 256 * 3, 512, 1),
                                       (1, 256 * 120 + 5, 1024, 1)])
def test_forward_pool_signed(B, N, K, cps):
    import pcs_amd._lib as L
    Nc = 512
    g = torch.Generator().manual_seed(31 + N)
    A = torch.relu(torch.randn(B * N, K, generator=g)).to(torch.bfloat16).to(DEV)
    W = (torch.randn(Nc, K, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    gamma = torch.randn(Nc, generator=g).to(DEV)
    Ws = torch.empty_like(W)
    L.call("pcs_sign_rows", L.ptr(W), L.BF16, Nc, K, L.ptr(gamma), L.ptr(Ws), L.stream_ptr())
    new = _pool(L, A, Ws, gamma, B, N, L.FLAG_W4, cps)
    old = _pool(L, A, Ws, gamma, B, N, 0, cps)
    torch.cuda.synchronize()
    pos = gamma[None, :] > 0
    val = torch.where(pos, new[..., 0], new[..., 2])
    row = torch.where(pos, new[..., 1], new[..., 3]).view(torch.int32)
    # against fp64: the extremum of each chunk and the value at the reported row
    y = (A.double() @ W.double().T)
    sgn = torch.where(gamma > 0, 1.0, -1.0).double()
    nch = new.shape[0]
    cps_ = nch // B
    rpc = _pool.rpc
    scl = y.abs().max().item()
    for ch in range(nch):
        b, ci = divmod(ch, cps_)
        lo, hi = b * N + ci * rpc, b * N + min((ci + 1) * rpc, N)
        if lo >= hi:
            continue
        ext = (y[lo:hi] * sgn).max(0).values * sgn
        assert float((val[ch].double() - ext).abs().max()) < 1e-5 * scl
        r = row[ch].long()
        assert ((r >= lo) & (r < hi)).all()
        at = y[r, torch.arange(Nc, device=DEV)]
        assert float((at - ext).abs().max()) < 1e-5 * scl
    # the 8-wave kernel: the same rows except where two candidates tie within fp32 rounding
    vold = torch.where(pos, old[..., 0], old[..., 2])
    rold = torch.where(pos, old[..., 1], old[..., 3]).view(torch.int32)
    assert float(((val - vold).abs() / vold.abs().clamp_min(1e-30)).max()) < 1e-5
    assert (row == rold).double().mean().item() > 0.995


def test_forward_pool_first_row_ties():
    """Repeated rows: every maximum occurs on many rows of the chunk (across tiles visited out of
    order); the reported row is the first, as torch.max's first-index rule on the reference."""
    import pcs_amd._lib as L
    B, K, Nc = 1, 512, 256
    base = torch.relu(torch.randn(37, K, generator=torch.Generator().manual_seed(3)))
    N = 256 * 100
    A = base.repeat(N // 37 + 1, 1)[:N].to(torch.bfloat16).to(DEV)
    W = (torch.randn(Nc, K, generator=torch.Generator().manual_seed(4)) * 0.05).to(torch.bfloat16).to(DEV)
    gamma = torch.ones(Nc, device=DEV)
    pool = _pool(L, A, W, gamma, B, N, L.FLAG_W4, 1)
    torch.cuda.synchronize()
    y = A.double() @ W.double().T
    first = y.argmax(0).int()
    assert torch.equal(pool[0, :, 1].view(torch.int32), first)


def test_bitwise_repeatable_and_applicability():
    import pcs_amd._lib as L
    B, N, K = 2, 256 * 6 + 100, 1024
    g = torch.Generator().manual_seed(9)
    A = torch.relu(torch.randn(B * N, K, generator=g)).to(torch.bfloat16).to(DEV)
    H = (torch.randn(K, K, generator=g) * 0.03).to(torch.bfloat16).to(DEV)
    c = torch.randn(K, generator=g).to(DEV)
    outs = [_dgrad(L, A, H, c, B, N, L.FLAG_W4, 2) for _ in range(4)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o.view(torch.int16), outs[0].view(torch.int16))
    lib = L.load()
    a, _ = _args(L, B, N, K, K, L.EPI_DGRAD, L.FLAG_W4)
    a.A, a.Yp, a.W = A.data_ptr(), A.data_ptr(), H.data_ptr()
    assert lib.pcs_gemm_w4_selected(ct.byref(a)) == 1
    st = torch.empty(B * a.chunks_per_scene, K, 2, device=DEV)
    a.stats = st.data_ptr()                           # statistics: the 8-wave kernel's epilogue
    assert lib.pcs_gemm_w4_selected(ct.byref(a)) == 0
    a.stats = None
    a.flags = 0                                       # the default: the 8-wave kernel
    assert lib.pcs_gemm_w4_selected(ct.byref(a)) == 0

"""The fp8 wide-layer kernels (compute dtype "fp8", BASELINE configs[4]) against torch on the
same e4m3 operands, through the C ABI:

* pcs_quant_fp8_rows: e4m3 bytes and E8M0 row scales bit-exact against torch's float8_e4m3fn
  cast of W * 2^-e (e = ceil(log2(row max / 448))), and the dequantized copy;
* conv5's BN+ReLU epilogue storing fp8 (PCS_FLAG_C_FP8): every stored byte within one e4m3
  rounding of the fp64 value, column sums equal to the sums of the stored bytes;
* the LDS-DMA global_feat kernel on MX-scaled fp8 MFMA (PCS_FLAG_AW_FP8): forward BN
  statistics / max-pool and the folded input gradient (+ pcs_pool_rows_add on fp8 Yp) against
  fp64 products of the dequantized operands -- e4m3 x e4m3 products are exact in the fp32
  accumulators, so only the summation order differs;
* pcs_gram_raw on fp8 rows (ragged M: the reduce kernel's tail rows) and pcs_gram_wgrad's
  max-pool term reading e4m3 a5.
"""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _e4m3(x):
    """fp32 tensor -> e4m3 bytes (uint8), round to nearest even."""
    return x.to(torch.float8_e4m3fn).view(torch.uint8)


def _dec(b):
    """e4m3 bytes -> fp64 (decoded on the host, returned on b's device)."""
    return b.cpu().view(torch.float8_e4m3fn).to(torch.float64).to(b.device)


def _quant(L, W):
    rows, cols = W.shape
    Wq = torch.empty(rows, cols, dtype=torch.uint8, device=DEV)
    sc = torch.empty(rows, dtype=torch.uint8, device=DEV)
    deq = torch.empty(rows, cols, device=DEV)
    L.call("pcs_quant_fp8_rows", L.ptr(W), rows, cols, W.stride(0), L.ptr(Wq), L.ptr(sc), L.ptr(deq), L.stream_ptr())
    return Wq, sc, deq


def _args(L, B, N, K, Nc, pro, epi, flags, cps=0):
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=pro, epilogue=epi,
                   chunks_per_scene=cps, flags=flags)
    rpc = L.load().pcs_gemm_geometry(ct.byref(a))
    assert rpc > 0
    return a, rpc


def _fp8_act(g, M, K):
    """A post-ReLU activation stored as e4m3 (about half the entries zero)."""
    return _e4m3(torch.relu(torch.randn(M, K, generator=g)) * 2.0).to(DEV)


def test_quant_fp8_rows_bit_exact():
    import pcs_amd._lib as L
    g = torch.Generator().manual_seed(1)
    W = torch.randn(96, 520, generator=g) * torch.logspace(-6, 3, 96)[:, None]
    W[5] = 0.0                                            # zero row: scale 127, zero bytes
    W[7, 3] = 448.0 * 2 ** 10                             # a row whose max sits on a power of two
    Wd = torch.zeros(96, 640)
    Wd[:, :520] = W                                       # row stride 640 > cols
    Wq, sc, deq = _quant(L, Wd.to(DEV)[:, :520])
    torch.cuda.synchronize()
    mx = W.abs().amax(1)
    e = torch.where(mx > 0, torch.ceil(torch.log2(mx / 448.0)), torch.zeros_like(mx)).clamp(-126, 127)
    assert torch.equal(sc.cpu().long(), (127 + e).long())
    ref = _e4m3(W * torch.exp2(-e)[:, None])
    assert torch.equal(Wq.cpu(), ref)
    assert torch.equal(deq.cpu().double(), _dec(ref) * torch.exp2(e.double())[:, None])


@pytest.mark.parametrize("B,N", [(2, 700), (3, 64 * 37 + 5), (1, 64 * 64)])
def test_bnrelu_epilogue_fp8_store_and_colsums(B, N):
    import pcs_amd._lib as L
    K, Nc = 128, 1024
    g = torch.Generator().manual_seed(3 + N)
    Y = torch.randn(B * N, K, generator=g).to(torch.bfloat16).to(DEV)
    ps = (torch.rand(K, generator=g) + 0.5).to(DEV)
    pt = (torch.randn(K, generator=g) * 0.2).to(DEV)
    W = (torch.randn(Nc, K, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    es = torch.randn(Nc, generator=g).to(DEV)
    et = (torch.randn(Nc, generator=g) * 0.3).to(DEV)
    a, _ = _args(L, B, N, K, Nc, L.PRO_BNRELU, L.EPI_BNRELU, L.FLAG_C_FP8)
    out = torch.empty(B * N, Nc, dtype=torch.uint8, device=DEV)
    st = torch.empty(B * a.chunks_per_scene, Nc, 2, device=DEV)
    a.A, a.W, a.C, a.pa, a.pb, a.es, a.et, a.stats = (Y.data_ptr(), W.data_ptr(), out.data_ptr(), ps.data_ptr(),
                                                       pt.data_ptr(), es.data_ptr(), et.data_ptr(), st.data_ptr())
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    x = torch.relu(Y.float() * ps + pt).to(torch.bfloat16).double()
    ref = torch.relu((x @ W.double().T) * es.double() + et.double())
    got = _dec(out)
    # one e4m3 rounding (3 mantissa bits: half-ulp 2^-4 relative) of a value within fp32
    # accumulation noise of ref; subnormals (< 2^-6) have an absolute half-ulp of 2^-10
    err = (got - ref).abs() - (ref.abs() * 2.0 ** -4 + 2.0 ** -10)
    assert float(err.max()) < 1e-4 * float(ref.abs().max()), float(err.max())
    cs = st[..., 0].double().sum(0)
    assert float((cs - got.sum(0)).abs().max()) < 1e-5 * float(got.sum(0).abs().max())


@pytest.mark.parametrize("B,N,cps", [(2, 256 * 7 + 77, 2), (1, 200, 0), (2, 256 * 9 + 50, 2)])
def test_fp8_forward_stats_and_pool(B, N, cps):
    import pcs_amd._lib as L
    K = Nc = 512 if N < 2000 else 1024
    g = torch.Generator().manual_seed(B * 1000 + N)
    A = _fp8_act(g, B * N, K)
    Wf = (torch.randn(Nc, K, generator=g) * 0.05).to(DEV)
    Wq, sc, Wd = _quant(L, Wf)
    a, rpc = _args(L, B, N, K, Nc, L.PRO_RAW, L.EPI_FWD, L.FLAG_AW_FP8, cps)
    nch = B * a.chunks_per_scene
    runs = []
    gamma = torch.randn(Nc, generator=g).to(DEV)
    for _ in range(3):   # repeated launches are bitwise identical
        st = torch.full((nch, Nc, 2), float("nan"), device=DEV)
        pool = torch.full((nch, Nc, 4), float("nan"), device=DEV)
        a.A, a.W, a.C, a.stats, a.pool, a.es, a.w_scale = (A.data_ptr(), Wq.data_ptr(), None, st.data_ptr(),
                                                           pool.data_ptr(), gamma.data_ptr(), sc.data_ptr())
        L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
        runs.append((st, pool))
    torch.cuda.synchronize()
    for r in runs[1:]:
        assert torch.equal(r[0].view(torch.int32), runs[0][0].view(torch.int32))
        assert torch.equal(r[1].view(torch.int32), runs[0][1].view(torch.int32))
    st, pool = runs[0]
    beta = torch.zeros(Nc, device=DEV)
    mean, rstd, scale, shift = (torch.empty(Nc, device=DEV) for _ in range(4))
    s = L.stream_ptr()
    L.call("pcs_bn_fwd_finalize", L.ptr(st), B, N, Nc, a.chunks_per_scene, rpc, L.ptr(gamma), L.ptr(beta),
           None, None, None, 0.1, 1e-5, 0, L.ptr(mean), L.ptr(rstd), L.ptr(scale), L.ptr(shift), None, s)
    gp = torch.empty(B, Nc, device=DEV)
    am = torch.empty(B, Nc, dtype=torch.int32, device=DEV)
    ysel = torch.empty(B, Nc, device=DEV)
    L.call("pcs_pool_finalize", L.ptr(pool), B, N, Nc, a.chunks_per_scene, L.ptr(scale), L.ptr(shift),
           L.ptr(gp), L.ptr(am), L.ptr(ysel), s)
    torch.cuda.synchronize()
    y = _dec(A) @ Wd.double().T
    scl = y.abs().max().item()
    assert float((mean.double() - y.mean(0)).abs().max()) < 1e-5 * scl
    var = 1.0 / rstd.double() ** 2 - 1e-5
    assert float(((var - y.var(0, unbiased=False)).abs() / y.var(0, unbiased=False)).max()) < 1e-4
    yb = y.view(B, N, Nc)
    sgn = torch.where(gamma > 0, 1.0, -1.0).double()
    ext = (yb * sgn).max(1).values * sgn
    # per-element error of y: fp32 sums of 128-product MFMA blocks (measured 1.3e-5 of max|y|
    # at K = 512); a near-tie extremum may be reported at another row within that error
    err = float((ysel.double() - ext).abs().max())
    print(f"fp8 pool extremum err / max|y| = {err / scl:.2e}")
    assert err < 5e-5 * scl
    rows = am.long() - (torch.arange(B, device=DEV) * N)[:, None]
    assert ((rows >= 0) & (rows < N)).all()
    at = yb.gather(1, rows[:, None, :]).squeeze(1)
    assert float((at - ext).abs().max()) < 1e-4 * scl


@pytest.mark.parametrize("B,N,cps", [(2, 256 * 5 + 33, 2), (1, 300, 0), (2, 256 * 9 + 50, 2)])
def test_fp8_folded_dgrad(B, N, cps):
    import pcs_amd._lib as L
    K = 512 if N < 2000 else 1024
    g = torch.Generator().manual_seed(7 + N)
    A = _fp8_act(g, B * N, K)
    Hf = torch.randn(K, K, generator=g) * 0.05
    Hf = ((Hf + Hf.T) / 2).to(DEV)                         # symmetric, like W^T diag(gamma) W
    Hq, hs, Hd = _quant(L, Hf)
    c = (torch.randn(K, generator=g) * 0.1).to(DEV)
    Pc = 256
    Wsp = (torch.randn(Pc, K, generator=g) * 0.1).to(DEV)
    am = torch.randint(0, N, (B, Pc), generator=g)
    am[:, 1] = am[:, 0]
    am[:, 2] = N - 1
    am = (am + torch.arange(B)[:, None] * N).int().to(DEV)
    sp = torch.randn(B, Pc, generator=g).to(DEV)
    a, _ = _args(L, B, N, K, K, L.PRO_RAW, L.EPI_DGRAD, L.FLAG_AW_FP8, cps)
    st = torch.empty(B * a.chunks_per_scene, K, 2, device=DEV)
    out = torch.full((B * N, K), float("nan"), dtype=torch.bfloat16, device=DEV)
    a.A, a.W, a.C, a.Yp, a.bias, a.w_scale = (A.data_ptr(), Hq.data_ptr(), out.data_ptr(), A.data_ptr(),
                                              c.data_ptr(), hs.data_ptr())
    a.stats = st.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    L.call("pcs_pool_rows_add", L.ptr(out), L.BF16, L.ptr(A), L.FP8, B, N, K, L.ptr(am), L.ptr(sp), L.ptr(Wsp), K,
           Pc, L.ptr(st), a.chunks_per_scene, L.stream_ptr())
    torch.cuda.synchronize()
    Ad = _dec(A)
    v = Ad @ Hd.double() + c.double()                     # H symmetric: row n = column n
    for b in range(B):
        for q in range(Pc):
            v[am[b, q].long()] += sp[b, q].double() * Wsp[q].double()
    dz = torch.where(Ad > 0, v, torch.zeros_like(v))
    err = float((out.double() - dz).abs().max())
    assert err < 1e-2 * dz.abs().max().item(), err      # bf16 output rounding
    s1 = st[..., 0].double().sum(0)
    err = float((s1 - dz.sum(0)).abs().max())
    assert err < 1e-3 * dz.abs().sum(0).max().item(), err


@pytest.mark.parametrize("M", [128 * 300, 128 * 257 + 77])
def test_gram_raw_fp8(M):
    import pcs_amd._lib as L
    C = 1024
    g = torch.Generator().manual_seed(M)
    A = _fp8_act(g, M, C)
    nbytes = L.load().pcs_gram_raw_workspace(M, C)
    assert nbytes > 0
    ws = torch.empty(nbytes // 4, device=DEV)
    G = torch.full((C, C), float("nan"), device=DEV)
    L.call("pcs_gram_raw", L.ptr(A), M, C, L.FP8, L.ptr(ws), nbytes, L.ptr(G), L.stream_ptr())
    torch.cuda.synchronize()
    Ad = _dec(A)
    ref = Ad.T @ Ad
    err = float((G.double() - ref).abs().max())
    assert err < 1e-5 * float(ref.abs().max()), err
    assert torch.equal(G, G.T)


def test_gram_wgrad_fp8_pool_rows():
    """pcs_gram_wgrad's max-pool term reads the e4m3 a5 rows (s = 1, t = 0)."""
    import pcs_amd._lib as L
    B, N, Cin, Cout = 2, 500, 256, 128
    g = torch.Generator().manual_seed(9)
    A = _fp8_act(g, B * N, Cin)
    Ad = _dec(A)
    G = (Ad.T @ Ad).float().to(DEV)
    S = Ad.sum(0).float().to(DEV)
    W = (torch.randn(Cout, Cin, generator=g) * 0.1).to(DEV)
    beta = torch.randn(Cout, generator=g).to(DEV)
    gamma = torch.randn(Cout, generator=g).to(DEV)
    sp = torch.randn(B, Cout, generator=g).to(DEV)
    am = (torch.randint(0, N, (B, Cout), generator=g) + torch.arange(B)[:, None] * N).int().to(DEV)
    ones, zeros = torch.ones(Cin, device=DEV), torch.zeros(Cin, device=DEV)
    dW = torch.empty(Cout, Cin, device=DEV)
    L.call("pcs_gram_wgrad", L.ptr(G), L.ptr(S), L.ptr(W), Cin, L.ptr(beta), L.ptr(gamma), L.ptr(sp), L.ptr(am),
           L.ptr(A), L.ptr(ones), L.ptr(zeros), B, Cout, Cin, L.FP8, None, None, L.ptr(dW), Cin, L.stream_ptr())
    torch.cuda.synchronize()
    ref = beta.double()[:, None] * S.double()[None] + gamma.double()[:, None] * (W.double() @ G.double())
    for b in range(B):
        ref += sp[b].double()[:, None] * Ad[am[b].long().cpu()].to(DEV)
    err = float((dW.double() - ref).abs().max())
    assert err < 1e-5 * float(ref.abs().max()), err

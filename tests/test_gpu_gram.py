"""pcs_gram / pcs_gram_wgrad (global_feat weight gradient from the Gram of its input)
against torch fp32 on the same operands: G = a^T a, colsum = sum_m a, and
dW = beta S^T... + diag(gamma) W G + the max-pool rows (see csrc/gram.hip)."""
import ctypes as ct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _case(B, N, C, dtype, seed=0):
    import pcs_amd._lib as L
    g = torch.Generator().manual_seed(seed)
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    Y = (torch.randn(B * N, C, generator=g) * 0.7).to(tdt).to(DEV)
    s = (torch.rand(C, generator=g) + 0.5).to(DEV)
    t = (torch.randn(C, generator=g) * 0.3).to(DEV)
    a = torch.relu(Y.float() * s + t)
    dt = L.BF16 if dtype == "bf16" else L.F32
    sps = ct.c_int32(0)
    nbytes = L.load().pcs_gram_workspace(B, N, C, dt, ct.byref(sps))
    assert nbytes > 0 and sps.value > 0
    ws = torch.empty(nbytes // 4, device=DEV)
    G = torch.empty(C, C, device=DEV)
    S = torch.empty(C, device=DEV)
    L.call("pcs_gram", L.ptr(Y), L.ptr(s), L.ptr(t), B, N, C, dt, sps.value, L.ptr(ws), L.ptr(G), L.ptr(S),
           L.stream_ptr())
    torch.cuda.synchronize()
    return L, dt, Y, s, t, a, G, S


@pytest.mark.parametrize("B,N,C,dtype", [(2, 700, 256, "bf16"),   # 256x256 kernel (upper tiles)
                                         (3, 333, 128, "bf16"),   # one-pass 128 kernel (wgrad_c5.hip)
                                         (2, 70005, 128, "bf16"),  # ... several slices, ragged tail
                                         (51, 3000, 128, "bf16"),  # ... an empty trailing slice
                                         (2, 300, 192, "bf16"),   # generic bf16 kernel
                                         (2, 257, 128, "fp32")])
def test_gram_matches_torch(B, N, C, dtype):
    L, dt, Y, s, t, a, G, S = _case(B, N, C, dtype)
    ab = a.to(torch.bfloat16).float() if dtype == "bf16" else a   # MFMA operands are rounded
    ref = (ab.double().T @ ab.double()).float()
    err = (G - ref).abs().max().item() / ref.abs().max().item()
    assert err < (2e-5 if dtype == "fp32" else 1e-4), err
    assert torch.equal(G, G.T)
    serr = (S.double() - a.double().sum(0)).abs().max().item() / a.sum(0).abs().max().item()
    assert serr < 1e-5, serr


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_gram_wgrad_matches_direct(dtype):
    B, N, C = 2, 500, 256
    L, dt, Y, s, t, a, G, S = _case(B, N, C, dtype, seed=1)
    g = torch.Generator().manual_seed(7)
    W = (torch.randn(C, C, generator=g) * 0.05).to(DEV)
    beta = (torch.randn(C, generator=g) * 1e-2).to(DEV)
    gamma = (torch.randn(C, generator=g) * 1e-2).to(DEV)
    sp = torch.randn(B, C, generator=g).to(DEV)
    am = (torch.randint(0, N, (B, C), generator=g) + torch.arange(B)[:, None] * N).int().to(DEV)
    dW = torch.empty(C, C, device=DEV)
    L.call("pcs_gram_wgrad", L.ptr(G), L.ptr(S), L.ptr(W), C, L.ptr(beta), L.ptr(gamma), L.ptr(sp), L.ptr(am),
           L.ptr(Y), L.ptr(s), L.ptr(t), B, C, C, dt, None, None, L.ptr(dW), C, L.stream_ptr())
    torch.cuda.synchronize()
    # direct: dy = beta + gamma * (a W^T) + max-pool rows, dW = dy^T a  (float64)
    ad, Wd = a.double(), W.double()
    dy = beta.double() + gamma.double() * (ad @ Wd.T)
    rows = am.long()
    for b in range(B):
        dy[rows[b], torch.arange(C, device=DEV)] += sp[b].double()
    ref = dy.T @ ad
    err = (dW.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < (1e-5 if dtype == "fp32" else 5e-3), err


@pytest.mark.parametrize("B,N,C", [(2, 700, 256), (4, 1000, 1024)])
def test_raw_gram_of_stored_activations(B, N, C):
    """s = t = NULL: the Gram of Y itself (the stored a5 >= 0), no transform pass; equals
    torch on the same bf16 values (and the ragged row tail past each slice is excluded)."""
    import pcs_amd._lib as L
    g = torch.Generator().manual_seed(C + N)
    A = torch.relu(torch.randn(B * N, C, generator=g)).to(torch.bfloat16).to(DEV)
    sps = ct.c_int32(0)
    nbytes = L.load().pcs_gram_workspace(B, N, C, L.BF16, ct.byref(sps))
    ws = torch.empty(nbytes // 4, device=DEV)
    G = torch.empty(C, C, device=DEV)
    S = torch.empty(C, device=DEV)
    L.call("pcs_gram", L.ptr(A), None, None, B, N, C, L.BF16, sps.value, L.ptr(ws), L.ptr(G), L.ptr(S),
           L.stream_ptr())
    torch.cuda.synchronize()
    af = A.float()
    ref = af.t() @ af
    assert float((G - ref).norm() / ref.norm()) < 1e-5
    assert float((S - af.sum(0)).norm() / af.sum(0).norm()) < 1e-5
    with pytest.raises(L.PcsError):   # the identity form needs the 256x256 kernel
        L.call("pcs_gram", L.ptr(A), None, None, B, N, 128, L.BF16, sps.value, L.ptr(ws), L.ptr(G),
               L.ptr(S), L.stream_ptr())


@pytest.mark.parametrize("M", [8 * 128 ** 2 + 37, 1000, 64 * 3])
def test_gram_raw_lds_dma_matches_torch(M):
    """pcs_gram_raw (csrc/gram_glds.hip): the LDS-DMA Gram of a stored bf16 activation, over
    balanced (tile, 64-row step) ranges (ranges spanning two tiles, fewer steps than
    workgroups, a tail of M % 64 rows), is a^T a of the bf16 values; repeated launches are
    bitwise identical."""
    import pcs_amd._lib as L
    C = 1024
    g = torch.Generator().manual_seed(M)
    A = torch.relu(torch.randn(M, C, generator=g)).to(torch.bfloat16).to(DEV)
    A[:, 5] = 0   # an all-zero column
    nbytes = L.load().pcs_gram_raw_workspace(M, C)
    assert nbytes > 0
    ws = torch.empty(nbytes // 4, device=DEV)
    outs = []
    for _ in range(3):
        G = torch.full((C, C), float("nan"), device=DEV)
        L.call("pcs_gram_raw", L.ptr(A), M, C, L.BF16, L.ptr(ws), nbytes, L.ptr(G), L.stream_ptr())
        outs.append(G)
    torch.cuda.synchronize()
    ref = A.double().T @ A.double()
    G = outs[0]
    assert torch.isfinite(G).all()
    err = float((G.double() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err
    assert torch.equal(G, G.T)
    for o in outs[1:]:
        assert torch.equal(o, G)

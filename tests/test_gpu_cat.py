"""PCS_PRO_CAT (csrc/gemm_nt.hip): conv5's folded input gradient in one pass,
    v   = [dz | relu(Y s + t)] [W ; W2]^T + c        (the operand concatenated along k)
    dz' = (Y es + et > 0) * v,   S1 = sum dz',   S2 = sum dz' (Y - mean) rstd
against torch fp64 on the same (bf16-rounded) operands, through the C ABI.  Ragged scenes
exercise the clamped tail rows; K1 = 1024 is conv5's shape, K1 = 256 a short one."""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("B,N,K1", [(2, 700, 256), (3, 128 * 9 + 5, 1024)])
def test_cat_prologue_dgrad(dtype, B, N, K1):
    import pcs_amd._lib as L
    dt, tdt = (L.BF16, torch.bfloat16) if dtype == "bf16" else (L.F32, torch.float32)
    g = torch.Generator().manual_seed(K1 + N)
    M, K2, Nc = B * N, 128, 128
    dz = (torch.randn(M, K1, generator=g) * 0.1).to(tdt).to(DEV)
    Y = torch.randn(M, K2, generator=g).to(tdt).to(DEV)
    s, t = (torch.rand(K2, generator=g) + 0.5).to(DEV), (torch.randn(K2, generator=g) * 0.2).to(DEV)
    W = (torch.randn(Nc, K1, generator=g) * 0.05).to(tdt).to(DEV)
    W2 = (torch.randn(Nc, K2, generator=g) * 0.05).to(tdt).to(DEV)
    c = (torch.randn(Nc, generator=g) * 0.1).to(DEV)
    mean, rstd = (torch.randn(Nc, generator=g) * 0.1).to(DEV), (torch.rand(Nc, generator=g) + 0.5).to(DEV)
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K1 + K2, Ncols=Nc, dtype=dt, prologue=L.PRO_CAT,
                   epilogue=L.EPI_DGRAD, chunks_per_scene=0, K1=K1)
    assert L.load().pcs_gemm_geometry(ct.byref(a)) > 0
    st = torch.empty(B * a.chunks_per_scene, Nc, 2, device=DEV)
    out = torch.empty(M, Nc, dtype=tdt, device=DEV)
    a.A, a.A2, a.W, a.W2, a.C = dz.data_ptr(), Y.data_ptr(), W.data_ptr(), W2.data_ptr(), out.data_ptr()
    a.pa, a.pb, a.bias, a.Yp, a.es, a.et = L.ptr(s), L.ptr(t), L.ptr(c), Y.data_ptr(), L.ptr(s), L.ptr(t)
    a.emean, a.erstd, a.stats = L.ptr(mean), L.ptr(rstd), st.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    x = torch.relu(Y.float() * s + t).to(tdt).double()
    v = dz.double() @ W.double().T + x @ W2.double().T + c.double()
    y = Y.double()
    keep = (y * s.double() + t.double()) > 0
    ref = torch.where(keep, v, torch.zeros_like(v))
    tol = 1e-2 if dtype == "bf16" else 1e-5
    err = float((out.double() - ref).norm() / ref.norm())
    assert err < tol, err
    s1 = st[..., 0].double().sum(0)
    assert float((s1 - ref.sum(0)).abs().max()) < (1e-3 if dtype == "bf16" else 1e-5) * float(ref.abs().sum(0).max())
    s2 = st[..., 1].double().sum(0)
    r2 = (ref * (y - mean.double()) * rstd.double()).sum(0)
    assert float((s2 - r2).abs().max()) < (2e-3 if dtype == "bf16" else 1e-5) * float(r2.abs().max())
    a.K1 = K1 + 3            # not a k-step multiple: refused
    with pytest.raises(L.PcsError):
        L.call("pcs_gemm", ct.byref(a), L.stream_ptr())

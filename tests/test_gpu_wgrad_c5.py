"""conv5's R = dz5^T relu(bn4(y4)) (pcs_wgrad with dy_mode RAW, x_mode BNRELU, Cin 128: the
LDS-DMA stream of csrc/wgrad_c5.hip) against torch fp64 on the same bf16 operands and against
the register-staged kernel (PCS_FLAG_GENERIC), on ragged scenes (rows not a multiple of the
32-row step, a slice shorter than one step) and at a size with many steps per slice.

    R[n, k] = sum_m dz5[m, n] x[m, k],  x = relu(y4 s + t) rounded to bf16 as staged"""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _run(B, N, Cout, seed, generic=False):
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(seed)
    M = B * N
    dz = (torch.randn(M, Cout, generator=g) * 0.1).to(torch.bfloat16)
    y4 = torch.randn(M, 128, generator=g).to(torch.bfloat16)
    s, t = torch.rand(128, generator=g) + 0.5, torch.randn(128, generator=g) * 0.3
    T = {k: v.to(DEV).contiguous() for k, v in dict(dz=dz, y4=y4, s=s, t=t).items()}
    R = torch.empty(Cout, 128, device=DEV)
    a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=Cout, Cin=128, dtype=L.BF16, splits_per_scene=0,
                    dy_mode=L.PRO_RAW, x_mode=L.PRO_BNRELU, x_keep_scale=1.0, dW=R.data_ptr(), ldw=0,
                    flags=L.FLAG_GENERIC if generic else 0)
    a.dZ, a.X, a.s, a.t = (T[k].data_ptr() for k in ("dz", "y4", "s", "t"))
    nbytes = L.load().pcs_wgrad_workspace(ct.byref(a))
    ws = torch.empty(nbytes // 4, device=DEV)
    a.partial = ws.data_ptr()
    L.call("pcs_wgrad", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    x = torch.relu(y4.double() * s.double() + t.double()).to(torch.bfloat16).double()
    return R.double().cpu(), dz.double().T @ x


@pytest.mark.parametrize("B,N,Cout", [(2, 70000 + 5, 1024), (3, 1000, 1024), (1, 31, 1024), (2, 5000 + 3, 512)])
def test_wgrad_c5_matches_fp64(B, N, Cout):
    R, ref = _run(B, N, Cout, 5 + N)
    assert float((R - ref).abs().max() / ref.abs().max()) < 1e-4


def test_wgrad_c5_agrees_with_generic_kernel():
    R, _ = _run(2, 20000 + 3, 1024, 9)
    Rg, _ = _run(2, 20000 + 3, 1024, 9, generic=True)
    assert float((R - Rg).abs().max() / Rg.abs().max()) < 1e-4


@pytest.mark.parametrize("B,N", [(2, 70000 + 5), (1, 31), (3, 1000)])
def test_wgrad_c5_dy_colsum(B, N):
    """dy_colsum: bn5's S1 = sum over rows of dz5 (as stored) from a ones fragment beside R's
    MFMAs; rows past a slice (clamped DMA rows) add nothing; R itself is unchanged."""
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(N)
    M, Cout = B * N, 1024
    dz = (torch.randn(M, Cout, generator=g) * 0.1 + 0.01).to(torch.bfloat16).to(DEV)
    y4 = torch.randn(M, 128, generator=g).to(torch.bfloat16).to(DEV)
    s, t = (torch.rand(128, generator=g) + 0.5).to(DEV), (torch.randn(128, generator=g) * 0.3).to(DEV)
    outs = []
    for colsum in (False, True):
        R = torch.empty(Cout, 128, device=DEV)
        s1 = torch.full((Cout,), float("nan"), device=DEV)
        a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=Cout, Cin=128, dtype=L.BF16, splits_per_scene=0,
                        dy_mode=L.PRO_RAW, x_mode=L.PRO_BNRELU, x_keep_scale=1.0, dW=R.data_ptr(), ldw=0, flags=0)
        a.dZ, a.X, a.s, a.t = dz.data_ptr(), y4.data_ptr(), s.data_ptr(), t.data_ptr()
        if colsum:
            a.dy_colsum = s1.data_ptr()
        ws = torch.empty(L.load().pcs_wgrad_workspace(ct.byref(a)) // 4, device=DEV)
        a.partial = ws.data_ptr()
        L.call("pcs_wgrad", ct.byref(a), L.stream_ptr())
        outs.append((R, s1))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    ref = dz.double().sum(0)
    err = float((outs[1][1].double() - ref).abs().max())
    assert err < 1e-5 * dz.double().abs().sum(0).max().item(), err
    # another kernel refuses dy_colsum
    a.flags = L.FLAG_GENERIC
    with pytest.raises(L.PcsError):
        L.call("pcs_wgrad", ct.byref(a), L.stream_ptr())

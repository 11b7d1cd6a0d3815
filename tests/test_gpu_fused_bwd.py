"""pcs_dgrad_wgrad (csrc/fused_bwd.hip): seg_conv1's fused input + weight gradient against a
plain PyTorch fp32 reference of the same op on bf16 inputs.

    dy  = alpha * dZ + beta + gamma * Y            (bn_seg1 backward coefficients)
    dX  = dy @ W_l                                 (dA2, no epilogue)
    dW  = dy^T @ relu(X * s + t)                   (written into a row-stride-1088 buffer)

dy and x are rounded to bf16 on the reference side exactly as the kernel stages them; the
tolerance covers fp32 accumulation order and the bf16 rounding of dX (1e-2 norm-relative
for dX, 1e-4 for dW, whose fp32 partials are summed in a fixed order).  Scene lengths that
are not multiples of the 64-row step exercise the clamped tail rows.
"""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("B,N", [(3, 1000), (4, 4096), (1, 70), (2, 64 * 300 + 17)])
def test_dgrad_wgrad_matches_torch(B, N):
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(B * 7919 + N)
    M = B * N
    dZ = (torch.randn(M, 512, generator=g) * 0.1).to(DEV, torch.bfloat16)
    Y = torch.randn(M, 512, generator=g).to(DEV, torch.bfloat16)
    X = torch.randn(M, 64, generator=g).to(DEV, torch.bfloat16)
    alpha, beta, gamma = (torch.randn(512, generator=g).to(DEV) * s for s in (1.0, 0.01, 0.05))
    sx, tx = torch.rand(64, generator=g).to(DEV) + 0.5, torch.randn(64, generator=g).to(DEV) * 0.2
    W = torch.randn(512, 64, generator=g).to(DEV) * 0.05
    Wt = W.t().contiguous().to(torch.bfloat16)            # [64, 512]
    dW = torch.full((512, 1088), 7.0, device=DEV)          # columns 64.. must stay untouched
    dX = torch.empty(M, 64, device=DEV, dtype=torch.bfloat16)
    a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=512, Cin=64, dtype=L.BF16, splits_per_scene=0,
                    dy_mode=L.PRO_BWD, x_mode=L.PRO_BNRELU, x_keep_scale=1.0, dW=dW.data_ptr(), ldw=1088,
                    dZ=dZ.data_ptr(), Y=Y.data_ptr(), alpha=alpha.data_ptr(), beta=beta.data_ptr(),
                    gamma=gamma.data_ptr(), X=X.data_ptr(), s=sx.data_ptr(), t=tx.data_ptr())
    nbytes = L.load().pcs_dgrad_wgrad_workspace(ct.byref(a))
    assert nbytes > 0
    ws = torch.empty(nbytes // 4, device=DEV)
    a.partial = ws.data_ptr()
    L.call("pcs_dgrad_wgrad", ct.byref(a), Wt.data_ptr(), dX.data_ptr(), L.stream_ptr())
    torch.cuda.synchronize()
    dy = (alpha * dZ.float() + (gamma * Y.float() + beta)).to(torch.bfloat16).float()
    x = torch.relu(X.float() * sx + tx).to(torch.bfloat16).float()
    ref_dx = dy @ Wt.float().t()
    ref_dw = dy.t() @ x
    assert _rel(dX.float(), ref_dx) < 1e-2
    assert _rel(dW[:, :64], ref_dw) < 1e-4
    assert torch.all(dW[:, 64:] == 7.0)


@pytest.mark.parametrize("B,N", [(3, 1000), (4, 4096), (1, 70), (2, 64 * 300 + 17)])
def test_dgrad_wgrad_folded_matches_torch(B, N):
    """pcs_dgrad_wgrad_folded: the same two gradients from dz and x alone (bn_seg1's stored
    Y' = x W^T + sbias[b] is never read), against torch fp64 of the unfolded definition:
    dy = alpha dz + beta + gamma Y', dX = dy W, dW = dy^T x.  dX carries the bf16 rounding of
    the folded operands (diag(alpha) W)^T and H = W^T diag(gamma) W and of dX itself (1e-2
    norm-relative, as the unfolded kernel's bf16 dy); dW is assembled in fp32 from exact
    bf16 products (2e-4)."""
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(B * 7907 + N)
    M = B * N
    dZ = (torch.randn(M, 512, generator=g) * 0.1).to(DEV, torch.bfloat16)
    X = torch.randn(M, 64, generator=g).to(DEV, torch.bfloat16)
    alpha, beta, gamma = (torch.randn(512, generator=g).to(DEV) * s for s in (1.0, 0.01, 0.05))
    sx, tx = torch.rand(64, generator=g).to(DEV) + 0.5, torch.randn(64, generator=g).to(DEV) * 0.2
    Wf = torch.zeros(512, 1088, device=DEV)
    Wf[:, :64] = (torch.randn(512, 64, generator=g) * 0.05).to(torch.bfloat16).float().to(DEV)
    sbias = torch.randn(B, 512, generator=g).to(DEV) * 0.5
    WaT = torch.empty(64, 512, dtype=torch.bfloat16, device=DEV)
    H = torch.empty(64, 64, dtype=torch.bfloat16, device=DEV)
    c = torch.empty(64, device=DEV)
    L.call("pcs_bn_fold", L.ptr(Wf), 512, 64, 1088, L.ptr(alpha), L.ptr(beta), L.ptr(gamma), L.BF16, L.ptr(WaT),
           L.ptr(c), L.ptr(H), L.stream_ptr())
    dW = torch.full((512, 1088), 7.0, device=DEV)
    dX = torch.empty(M, 64, device=DEV, dtype=torch.bfloat16)
    a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=512, Cin=64, dtype=L.BF16, splits_per_scene=0,
                    dy_mode=L.PRO_RAW, x_mode=L.PRO_BNRELU, x_keep_scale=1.0, dW=dW.data_ptr(), ldw=1088,
                    dZ=dZ.data_ptr(), alpha=alpha.data_ptr(), beta=beta.data_ptr(), gamma=gamma.data_ptr(),
                    X=X.data_ptr(), s=sx.data_ptr(), t=tx.data_ptr())
    nbytes = L.load().pcs_dgrad_wgrad_folded_workspace(ct.byref(a))
    assert nbytes > 0
    ws = torch.empty(nbytes // 4, device=DEV)
    a.partial = ws.data_ptr()
    L.call("pcs_dgrad_wgrad_folded", ct.byref(a), L.ptr(WaT), L.ptr(H), L.ptr(Wf), L.ptr(sbias), L.ptr(dX),
           L.stream_ptr())
    torch.cuda.synchronize()
    x = torch.relu(X.float() * sx + tx).to(torch.bfloat16).double()
    Wl = Wf[:, :64].double()
    Yp = x @ Wl.t() + sbias.double().repeat_interleave(N, dim=0)
    dy = alpha.double() * dZ.double() + beta.double() + gamma.double() * Yp
    ref_dx, ref_dw = dy @ Wl, dy.t() @ x
    print(f"dX rel {_rel(dX.double(), ref_dx):.2e}  dW rel {_rel(dW[:, :64].double(), ref_dw):.2e}")
    assert _rel(dX.double(), ref_dx) < 1e-2
    assert _rel(dW[:, :64].double(), ref_dw) < 2e-4
    assert torch.all(dW[:, 64:] == 7.0)
    a.dy_mode = L.PRO_BWD
    assert L.load().pcs_dgrad_wgrad_folded_workspace(ct.byref(a)) < 0


def test_dgrad_wgrad_rejects_other_shapes():
    import pcs_amd._lib as L
    a = L.WgradArgs(num_scenes=1, scene_rows=128, Cout=256, Cin=64, dtype=L.BF16, dy_mode=L.PRO_BWD,
                    x_mode=L.PRO_BNRELU)
    assert L.load().pcs_dgrad_wgrad_workspace(ct.byref(a)) < 0


@pytest.mark.parametrize("cout,cin,variant,B,N", [
    (64, 64, "plain", 3, 1000), (64, 64, "addend", 2, 4096 + 33), (128, 64, "plain", 4, 4096),
    (128, 64, "plain", 1, 64 * 40 + 5), (128, 64, "mask", 3, 777),
    # seg_conv2 / seg_conv3 (LDS-DMA streams, csrc/fused_seg4.hip): ragged slices, one-step slices
    (256, 512, "mask", 2, 4096 + 33), (256, 512, "plain", 1, 70), (256, 512, "mask", 4, 65536 + 100),
    (128, 256, "mask", 3, 1000), (128, 256, "plain", 2, 64 * 40 + 5), (128, 256, "mask", 1, 31)])
def test_dgrad_wgrad_bn_matches_torch(cout, cin, variant, B, N):
    """pcs_dgrad_wgrad_bn (conv2/3/4, seg_conv2/3) vs torch fp32 on the same bf16 inputs:
    dz' = (es*Yp + et > 0) * keep * ks * (dy W + addend), its per-chunk S1 / S2 statistics
    (S2 = rstd * (sum dz' Yp - mean * S1)) and dW = dy^T x.  seg_conv2 / seg_conv3 run the
    4-wave 256-column kernel (csrc/fused_seg4.hip) by default."""
    _check_bn(cout, cin, variant, B, N, 0)


def _check_bn(cout, cin, variant, B, N, flags):
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(cout * 31 + cin + N)
    M = B * N
    bf = lambda t: t.to(DEV, torch.bfloat16)   # noqa: E731
    dZ, Y = bf(torch.randn(M, cout, generator=g) * 0.1), bf(torch.randn(M, cout, generator=g))
    Yp = bf(torch.randn(M, cin, generator=g))
    al, be, ga = (torch.randn(cout, generator=g).to(DEV) * s for s in (1.0, 0.01, 0.05))
    es, et = torch.rand(cin, generator=g).to(DEV) + 0.5, torch.randn(cin, generator=g).to(DEV) * 0.3
    emean, erstd = torch.randn(cin, generator=g).to(DEV) * 0.1, torch.rand(cin, generator=g).to(DEV) + 0.5
    W = torch.randn(cout, cin, generator=g).to(DEV) * 0.05
    Wt = W.t().contiguous().to(torch.bfloat16)          # [cin, cout] = the dgrad GEMM's W
    add = bf(torch.randn(M, cin, generator=g) * 0.1) if variant == "addend" else None
    keep = (torch.rand(M, cin, generator=g) < 0.7) if variant == "mask" else None
    ks = 1.0 / 0.7 if keep is not None else 1.0
    bits = None
    if keep is not None:
        w8 = (1 << torch.arange(8)).to(torch.uint8)
        bits = (keep.view(M, cin // 8, 8).to(torch.uint8) * w8).sum(-1).to(torch.uint8).to(DEV)
    out = torch.empty(M, cin, device=DEV, dtype=torch.bfloat16)
    dW = torch.zeros(cout, cin, device=DEV)
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=cout, Ncols=cin, dtype=L.BF16, prologue=L.PRO_BWD,
                   epilogue=L.EPI_DGRAD, chunks_per_scene=0, A=dZ.data_ptr(), W=Wt.data_ptr(), C=out.data_ptr(),
                   a_keep_scale=1.0, c_keep_scale=ks, flags=flags)
    for k, v in dict(A2=Y, pa=al, pb=be, pc=ga, Yp=Yp, es=es, et=et, emean=emean, erstd=erstd,
                     c_mask=bits, addend=add).items():
        setattr(a, k, L.ptr(v))
    nbytes = L.load().pcs_dgrad_wgrad_bn_workspace(ct.byref(a))
    assert nbytes > 0
    cps = a.chunks_per_scene
    st = torch.empty(B * cps, cin, 2, device=DEV)
    ws = torch.empty(nbytes // 4, device=DEV)
    a.stats = st.data_ptr()
    L.call("pcs_dgrad_wgrad_bn", ct.byref(a), ws.data_ptr(), dW.data_ptr(), 0, L.stream_ptr())
    torch.cuda.synchronize()

    dy = (al * dZ.float() + (ga * Y.float() + be)).to(torch.bfloat16).float()
    yp = Yp.float()
    kf = keep.to(DEV).float() if keep is not None else torch.ones_like(yp)
    x = (torch.relu(yp * es + et) * kf * ks).to(torch.bfloat16).float()
    gv = dy @ Wt.float().t()
    if add is not None:
        gv = gv + add.float()
    dz = torch.where(yp * es + et > 0, gv * kf * ks, torch.zeros_like(gv))
    assert _rel(out.float(), dz) < 1e-2
    assert _rel(dW, dy.t() @ x) < 1e-4
    # statistics: per scene sums over the chunks equal the per-scene sums of dz (fp32)
    s1 = st[..., 0].view(B, cps, cin).sum(1)
    s2 = st[..., 1].view(B, cps, cin).sum(1)
    dzs = dz.view(B, N, cin)
    r1 = dzs.sum(1)
    r2 = erstd * ((dzs * yp.view(B, N, cin)).sum(1) - emean * r1)
    assert _rel(s1, r1) < 1e-3 and _rel(s2, r2) < 1e-3

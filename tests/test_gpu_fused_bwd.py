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


def test_dgrad_wgrad_rejects_other_shapes():
    import pcs_amd._lib as L
    a = L.WgradArgs(num_scenes=1, scene_rows=128, Cout=256, Cin=64, dtype=L.BF16, dy_mode=L.PRO_BWD,
                    x_mode=L.PRO_BNRELU)
    assert L.load().pcs_dgrad_wgrad_workspace(ct.byref(a)) < 0

"""The streamed CE head (csrc/head_stream.hip: pcs_head PCS_HEAD_CE, bf16, C <= 4, no logits out,
the fused train step's head) against torch fp64 on the same bf16 rows and against the register-
resident head_small_kernel (the same call with a logits buffer), on ragged scenes (rows not a
multiple of the 64-row step, a chunk shorter than one step), ignored (-1) labels and the CE
denominator.  Reductions are compared after summing the per-chunk partials (the two kernels
chunk the rows differently)."""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _run(B, N, C, seed, with_logits=False):
    import pcs_amd._lib as L
    g = torch.Generator().manual_seed(seed)
    M = B * N
    Y = (torch.randn(M, 128, generator=g) * 1.5 + 0.2).to(torch.bfloat16)
    v = lambda n, sc=1.0, o=0.0: torch.randn(n, generator=g) * sc + o   # noqa: E731
    s, t, mean, rstd = v(128, 0.5, 1.0), v(128, 0.5), v(128, 0.3), v(128, 0.1, 1.0).abs()
    W, b = v(C * 128, 0.1).reshape(C, 128), v(C, 0.2)
    lab = torch.randint(-1, C, (M,), generator=g, dtype=torch.int64)
    cw = torch.rand(C, generator=g) + 0.5
    wsum = torch.tensor([float(cw[lab.clamp(min=0)][lab >= 0].sum())])
    T = {k: x.to(DEV).contiguous() for k, x in dict(Y=Y, s=s, t=t, mean=mean, rstd=rstd, W=W, b=b, lab=lab,
                                                     cw=cw, wsum=wsum).items()}
    logits = torch.empty(M, C, device=DEV) if with_logits else None
    a = L.HeadArgs(num_scenes=B, scene_rows=N, Cin=128, num_classes=C, dtype=L.BF16, mode=L.HEAD_CE,
                   chunks_per_scene=0, Y=T["Y"].data_ptr(), s=T["s"].data_ptr(), t=T["t"].data_ptr(),
                   W=T["W"].data_ptr(), bias=T["b"].data_ptr(),
                   logits=logits.data_ptr() if with_logits else None)
    L.load().pcs_head_geometry(ct.byref(a))
    nch = B * a.chunks_per_scene
    dZ = torch.full((M, 128), float("nan"), dtype=torch.bfloat16, device=DEV)
    stats = torch.empty(nch, 128, 2, device=DEV)
    wpart = torch.empty(nch, C * 129, device=DEV)
    lpart = torch.empty(nch, device=DEV)
    a.labels, a.class_weight, a.wsum = T["lab"].data_ptr(), T["cw"].data_ptr(), T["wsum"].data_ptr()
    a.dZ, a.mean, a.rstd = dZ.data_ptr(), T["mean"].data_ptr(), T["rstd"].data_ptr()
    a.stats, a.wpartial, a.loss_partial = stats.data_ptr(), wpart.data_ptr(), lpart.data_ptr()
    L.call("pcs_head", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    out = dict(dZ=dZ.double().cpu(), S=stats.double().sum(0).cpu(), Wp=wpart.double().sum(0).cpu(),
               loss=float(lpart.double().sum()))
    # fp64 reference from the same bf16 rows
    y = Y.double()
    av = torch.relu(y * s.double() + t.double())
    lg = av @ W.double().T + b.double()
    valid = lab >= 0
    li = lab.clamp(min=0)
    wt = torch.where(valid, cw.double()[li], torch.zeros((), dtype=torch.float64))
    lse = torch.logsumexp(lg, 1)
    loss = float((wt * (lse - lg.gather(1, li[:, None])[:, 0])).sum())
    dl = wt[:, None] / float(wsum) * (torch.softmax(lg, 1) - torch.nn.functional.one_hot(li, C).double())
    dz = (dl @ W.double()) * (av > 0)
    xh = (y - mean.double()) * rstd.double()
    ref = dict(dZ=dz, S=torch.stack([dz.sum(0), (dz * xh).sum(0)], 1),
               Wp=torch.cat([(dl.T @ av).reshape(-1), dl.sum(0)]), loss=loss)
    return out, ref, a.chunks_per_scene


@pytest.mark.parametrize("C", [1, 2, 3, 4])
@pytest.mark.parametrize("B,N", [(2, 70000 + 5), (3, 1000), (1, 31)])
def test_head_stream_matches_fp64(C, B, N):
    out, ref, _ = _run(B, N, C, 100 * C + N)
    assert torch.isfinite(out["dZ"]).all()
    sc = ref["dZ"].abs().max() + 1e-30
    assert float((out["dZ"] - ref["dZ"]).abs().max() / sc) < 8e-3   # one bf16 rounding of dz
    for k in ("S", "Wp"):
        assert float((out[k] - ref[k]).abs().max() / (ref[k].abs().max() + 1e-30)) < 1e-4, k
    assert abs(out["loss"] - ref["loss"]) <= 1e-5 * abs(ref["loss"]) + 1e-6


@pytest.mark.parametrize("C", [2, 3])
def test_head_stream_agrees_with_register_kernel(C):
    B, N = 2, 20000 + 3
    out, _, _ = _run(B, N, C, 9)
    reg, _, _ = _run(B, N, C, 9, with_logits=True)   # logits out: the register-resident kernel
    # (with a logits buffer pcs_head takes the register kernel: pcs_head_stream_class needs no logits out)
    assert torch.equal(out["dZ"], reg["dZ"])   # the same per-row arithmetic
    for k in ("S", "Wp"):
        assert float((out[k] - reg[k]).abs().max() / reg[k].abs().max()) < 1e-5, k
    assert abs(out["loss"] - reg["loss"]) <= 1e-6 * abs(reg["loss"])

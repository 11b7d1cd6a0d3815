"""conv5's folded input gradient (pcs_gemm PRO_CAT / EPI_DGRAD at K1 = 1024, K - K1 = 128, 128
columns: the LDS-DMA stream of csrc/fused_c5.hip) against torch fp64 on the same bf16 operands
and against the generic kernel (PCS_FLAG_GENERIC), on ragged scenes (rows not a multiple of the
32-row step) and at a size with several steps per chunk.

    g   = dz5 Ws^T + relu(pa y4 + pb) H4^T + c5        (relu(...) rounded to bf16 as staged)
    dA4 = [es y4 + et > 0] g                            (stored bf16)
    S1  = sum dA4,  S2 = sum dA4 (y4 - emean) erstd     (per column, summed over the chunks)"""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _run(B, N, seed, generic=False):
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(seed)
    M = B * N
    bf = lambda t: t.to(torch.bfloat16)   # noqa: E731
    dz5 = bf(torch.randn(M, 1024, generator=g) * 0.1)
    y4 = bf(torch.randn(M, 128, generator=g))
    Ws = bf(torch.randn(128, 1024, generator=g) * 0.03)
    H4 = bf(torch.randn(128, 128, generator=g) * 0.05)
    v = lambda n, s=1.0, o=0.0: torch.randn(n, generator=g) * s + o   # noqa: E731
    pa, pb, c5 = v(128, 0.5, 1.0), v(128, 0.3), v(128, 0.2)
    es, et, em, er = v(128, 0.5, 1.0), v(128, 0.3), v(128, 0.2), v(128, 0.1, 1.0).abs()
    d = lambda t: t.to(DEV).contiguous()   # noqa: E731
    T = {k: d(t) for k, t in dict(dz5=dz5, y4=y4, Ws=Ws, H4=H4, pa=pa, pb=pb, c5=c5, es=es, et=et, em=em, er=er).items()}
    out = torch.empty(M, 128, dtype=torch.bfloat16, device=DEV)
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=1152, Ncols=128, dtype=L.BF16, prologue=L.PRO_CAT,
                   epilogue=L.EPI_DGRAD, chunks_per_scene=0, A=T["dz5"].data_ptr(), W=T["Ws"].data_ptr(),
                   C=out.data_ptr(), a_keep_scale=1.0, c_keep_scale=1.0)
    a.K1 = 1024
    a.A2, a.W2, a.pa, a.pb, a.bias = (T[k].data_ptr() for k in ("y4", "H4", "pa", "pb", "c5"))
    a.Yp, a.es, a.et, a.emean, a.erstd = (T[k].data_ptr() for k in ("y4", "es", "et", "em", "er"))
    if generic:
        a.flags |= L.FLAG_GENERIC
    L.load().pcs_gemm_geometry(ct.byref(a))
    stats = torch.zeros(B * a.chunks_per_scene, 128, 2, device=DEV)
    a.stats = stats.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    # reference (fp64 on the host, from the bf16 operands)
    a4 = torch.relu(y4.double() * pa.double() + pb.double()).to(torch.bfloat16).double()
    gg = dz5.double() @ Ws.double().T + a4 @ H4.double().T + c5.double()
    keep = (y4.double() * es.double() + et.double()) > 0
    ref = torch.where(keep, gg, torch.zeros_like(gg))
    S1 = ref.sum(0)
    S2 = (ref * (y4.double() - em.double()) * er.double()).sum(0)
    return out.double().cpu(), stats.sum(0).double().cpu(), ref, S1, S2


@pytest.mark.parametrize("B,N", [(2, 1000), (3, 4096 + 17), (1, 31), (2, 65536 + 5)])
def test_c5_dgrad_matches_fp64(B, N):
    out, st, ref, S1, S2 = _run(B, N, 7 + N)
    scale = ref.abs().max()
    assert float((out - ref).abs().max() / scale) < 8e-3            # one bf16 rounding of the output
    assert float((st[:, 0] - S1).abs().max() / S1.abs().max()) < 2e-3
    assert float((st[:, 1] - S2).abs().max() / S2.abs().max()) < 2e-3


def test_c5_dgrad_agrees_with_generic_kernel():
    out, st, _, _, _ = _run(2, 20000 + 3, 3)
    out_g, st_g, _, _, _ = _run(2, 20000 + 3, 3, generic=True)
    assert float((out - out_g).abs().max() / out_g.abs().max()) < 8e-3
    assert float((st - st_g).abs().max() / st_g.abs().max()) < 2e-3

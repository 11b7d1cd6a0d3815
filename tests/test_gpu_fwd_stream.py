"""The streaming forward kernel (csrc/fwd_stream.hip: pcs_gemm PRO_BNRELU with EPI_FWD on the
narrow-K layers seg_conv1 / seg_conv2 / seg_conv3 / conv4 / conv2-3, EPI_BNRELU on conv5) against torch
fp64 on the same bf16 operands and against the generic kernel (PCS_FLAG_GENERIC), on ragged
scenes (rows not a multiple of the step, several chunks, a slice shorter than one step).

    x  = relu(Yp pa + pb) [* keep / (1 - p)]         (rounded to bf16 as staged; P:106-127)
    y  = x W^T (+ bias | + per-scene bias)           stored bf16, per-chunk (mean, M2) of the stored
                                                      values (EPI_FWD)
    a  = relu(y es + et)                             stored bf16, per-chunk column sums (EPI_BNRELU)"""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")

SHAPES = [(64, 512, "scene"), (512, 256, "mask"), (256, 128, "mask"), (64, 128, "bias"), (64, 64, "bias"),
          (128, 1024, "bnrelu")]


def _run(B, N, K, C, kind, seed, generic=False, nomask=False):
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(seed)
    M = B * N
    bf = lambda t: t.to(torch.bfloat16)   # noqa: E731
    yp = bf(torch.randn(M, K, generator=g) * 2.0 + 0.3)
    W = bf(torch.randn(C, K, generator=g) * (1.0 / K ** 0.5))
    v = lambda n, s=1.0, o=0.0: torch.randn(n, generator=g) * s + o   # noqa: E731
    pa, pb = v(K, 0.5, 1.0), v(K, 0.5)
    mask = kind == "mask" and not nomask
    bits = torch.randint(0, 256, (M, K // 8), generator=g, dtype=torch.uint8) if mask else None
    ks = 1.0 / 0.7
    d = lambda t: t.to(DEV).contiguous()   # noqa: E731
    out = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    epi = L.EPI_BNRELU if kind == "bnrelu" else L.EPI_FWD
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=C, dtype=L.BF16, prologue=L.PRO_BNRELU,
                   epilogue=epi, chunks_per_scene=0, A=0, W=0, C=out.data_ptr(),
                   a_keep_scale=ks if mask else 1.0, c_keep_scale=1.0)
    if generic:
        a.flags |= L.FLAG_GENERIC
    T = dict(yp=d(yp), W=d(W), pa=d(pa), pb=d(pb))
    a.A, a.W, a.pa, a.pb = (T[k].data_ptr() for k in ("yp", "W", "pa", "pb"))
    bias = sbias = es = et = None
    if kind == "scene":
        sbias = v(B * C, 0.7).reshape(B, C)
        T["sb"] = d(sbias)
        a.scene_bias = T["sb"].data_ptr()
    if kind in ("bias", "bnrelu"):
        bias = v(C, 0.3)
        T["b"] = d(bias)
        a.bias = T["b"].data_ptr()
    if kind == "bnrelu":
        es, et = v(C, 0.5, 0.8), v(C, 0.4)
        T["es"], T["et"] = d(es), d(et)
        a.es, a.et = T["es"].data_ptr(), T["et"].data_ptr()
    if mask:
        T["bits"] = d(bits)
        a.a_mask = T["bits"].data_ptr()
    rpc = L.load().pcs_gemm_geometry(ct.byref(a))
    cps = a.chunks_per_scene
    stats = torch.full((B * cps, C, 2), float("nan"), device=DEV)
    # (the generic kernel keeps no column sums for EPI_BNRELU)
    a.stats = 0 if (generic and kind == "bnrelu") else stats.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    # reference (fp64 on the host, from the bf16 operands; x rounded to bf16 as staged)
    x = torch.relu(yp.double() * pa.double() + pb.double())
    if mask:
        keep = ((bits.long().unsqueeze(-1) >> torch.arange(8)) & 1).reshape(M, K).double()
        x = x * ks * keep
    x = x.to(torch.bfloat16).double()
    y = x @ W.double().T
    if sbias is not None:
        y = y + sbias.double().repeat_interleave(N, 0)
    if bias is not None:
        y = y + bias.double()
    if kind == "bnrelu":
        y = torch.relu(y * es.double() + et.double())
    counts = torch.tensor([min(rpc, N - c * rpc) for c in range(cps)] * B, dtype=torch.float64)
    return out.double().cpu(), stats.double().cpu(), y, counts


def _merged(stats, counts):
    """Chan merge of per-chunk (mean, M2) partials -> (mean, var) per column."""
    n = counts[:, None]
    mean = (stats[..., 0] * n).sum(0) / n.sum()
    m2 = stats[..., 1].sum(0) + (n * (stats[..., 0] - mean) ** 2).sum(0)
    return mean, m2 / n.sum()


@pytest.mark.parametrize("K,C,kind", SHAPES)
@pytest.mark.parametrize("B,N", [(2, 70000 + 5), (3, 1000), (1, 31)])
def test_fwd_stream_matches_fp64(K, C, kind, B, N):
    out, st, ref, counts = _run(B, N, K, C, kind, 11 + N + K)
    scale = ref.abs().max()
    assert float((out - ref).abs().max() / scale) < 8e-3            # one bf16 rounding of the output
    if kind == "bnrelu":
        S = ref.sum(0)
        assert float((st[..., 0].sum(0) - S).abs().max() / S.abs().max()) < 2e-3
        assert float(st[..., 1].abs().max()) == 0.0
    else:
        mean, var = _merged(st, counts)
        rmean, rvar = ref.mean(0), ref.var(0, unbiased=False)
        assert float((mean - rmean).abs().max() / rvar.sqrt().max()) < 5e-3
        assert float(((var - rvar).abs() / rvar).max()) < 2e-2


@pytest.mark.parametrize("K,C,kind", SHAPES)
def test_fwd_stream_agrees_with_generic_kernel(K, C, kind):
    B, N = 2, 20000 + 3
    out, st, _, counts = _run(B, N, K, C, kind, 5)
    out_g, st_g, _, counts_g = _run(B, N, K, C, kind, 5, generic=True)
    assert float((out - out_g).abs().max() / out_g.abs().max()) < 8e-3
    if kind != "bnrelu":
        m, v = _merged(st, counts)
        mg, vg = _merged(st_g, counts_g)
        assert float((m - mg).abs().max() / vg.sqrt().max()) < 5e-3
        assert float(((v - vg).abs() / vg).max()) < 2e-2


def test_fwd_stream_seg_conv2_without_dropout():
    out, st, ref, counts = _run(2, 9000 + 7, 512, 256, "mask", 3, nomask=True)
    assert float((out - ref).abs().max() / ref.abs().max()) < 8e-3


@pytest.mark.parametrize("B,N", [(2, 70000 + 5), (1, 31)])
def test_fwd_stream_conv5_fp8_store(B, N):
    """cfg5's a5 (PCS_FLAG_C_FP8): e4m3 bytes staged through LDS as 64-B wave rows; every stored
    byte within one e4m3 rounding of the fp64 value, column sums equal to the stored bytes' sums."""
    import pcs_amd._lib as L
    K, C = 128, 1024
    g = torch.Generator(device="cpu").manual_seed(17 + N)
    M = B * N
    yp = (torch.randn(M, K, generator=g) * 2.0).to(torch.bfloat16)
    W = (torch.randn(C, K, generator=g) * 0.1).to(torch.bfloat16)
    pa, pb = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.2
    es, et = torch.randn(C, generator=g), torch.randn(C, generator=g) * 0.3
    T = {k: t.to(DEV).contiguous() for k, t in dict(yp=yp, W=W, pa=pa, pb=pb, es=es, et=et).items()}
    out = torch.empty(M, C, dtype=torch.uint8, device=DEV)
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=C, dtype=L.BF16, prologue=L.PRO_BNRELU,
                   epilogue=L.EPI_BNRELU, chunks_per_scene=0, A=T["yp"].data_ptr(), W=T["W"].data_ptr(),
                   C=out.data_ptr(), a_keep_scale=1.0, c_keep_scale=1.0, flags=L.FLAG_C_FP8)
    a.pa, a.pb, a.es, a.et = (T[k].data_ptr() for k in ("pa", "pb", "es", "et"))
    L.load().pcs_gemm_geometry(ct.byref(a))
    st = torch.empty(B * a.chunks_per_scene, C, 2, device=DEV)
    a.stats = st.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    x = torch.relu(yp.double() * pa.double() + pb.double()).to(torch.bfloat16).double()
    ref = torch.relu((x @ W.double().T) * es.double() + et.double())
    got = out.cpu().view(torch.float8_e4m3fn).double()
    err = (got - ref).abs() - (ref.abs() * 2.0 ** -4 + 2.0 ** -10)
    assert float(err.max()) < 1e-4 * float(ref.abs().max())
    cs = st[..., 0].double().cpu().sum(0)
    assert float((cs - got.sum(0)).abs().max()) < 1e-5 * float(got.sum(0).abs().max())

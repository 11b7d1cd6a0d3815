"""The fused seg_conv1 + seg_conv2 forward (csrc/fwd_s12.hip, pcs_fwd_seg12; P:117-125) and
bn_seg1's statistics from the Gram of a2 (pcs_bn_stats_gram_sbias):

* the fused pass against the two streaming passes it replaces (pcs_gemm FWD for seg_conv1 with
  the scene bias, then for seg_conv2 with bn_seg1 + ReLU + dropout in its prologue) on the same
  operands and coefficients: Y1 and Y2 bit for bit (same bf16 operands, same fp32 summation
  order), bn_seg2's statistics merged per scene within 1e-5;
* the Gram statistics against torch fp64 of the same y = a W^T + sbias;
* one bf16 training step with the fused pass against the same step with the two passes."""
import ctypes as ct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ops(B, N, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    M = B * N
    r = lambda *s: torch.randn(*s, generator=g)   # noqa: E731
    y2 = r(M, 64).to(torch.bfloat16).to(DEV)
    s2, t2 = (r(64) * 0.5 + 1.0).to(DEV), (r(64) * 0.3).to(DEV)
    W1 = (r(512, 64) * 0.15).to(torch.bfloat16).to(DEV)
    sbias = (r(B, 512) * 0.2).to(DEV)
    s1, t1 = (r(512) * 0.3 + 0.8).to(DEV), (r(512) * 0.2).to(DEV)
    bits = torch.randint(0, 256, (M, 64), generator=g, dtype=torch.uint8).to(DEV)
    W2 = (r(256, 512) * 0.05).to(torch.bfloat16).to(DEV)
    return y2, s2, t2, W1, sbias, s1, t1, bits, W2


def _two_pass(L, B, N, y2, s2, t2, W1, sbias, s1, t1, bits, W2, ks):
    lib = L.load()
    M = B * N
    y1 = torch.empty(M, 512, dtype=torch.bfloat16, device=DEV)
    out = torch.empty(M, 256, dtype=torch.bfloat16, device=DEV)
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=64, Ncols=512, dtype=L.BF16, prologue=L.PRO_BNRELU,
                   epilogue=L.EPI_FWD, chunks_per_scene=0, A=y2.data_ptr(), W=W1.data_ptr(), C=y1.data_ptr(),
                   pa=s2.data_ptr(), pb=t2.data_ptr(), scene_bias=sbias.data_ptr(), a_keep_scale=1.0, c_keep_scale=1.0)
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    b = L.GemmArgs(num_scenes=B, scene_rows=N, K=512, Ncols=256, dtype=L.BF16, prologue=L.PRO_BNRELU,
                   epilogue=L.EPI_FWD, chunks_per_scene=0, A=y1.data_ptr(), W=W2.data_ptr(), C=out.data_ptr(),
                   pa=s1.data_ptr(), pb=t1.data_ptr(), a_mask=L.ptr(bits), a_keep_scale=ks, c_keep_scale=1.0)
    lib.pcs_gemm_geometry(ct.byref(b))
    st = torch.empty(B * b.chunks_per_scene, 256, 2, device=DEV)
    b.stats = st.data_ptr()
    L.call("pcs_gemm", ct.byref(b), L.stream_ptr())
    return y1, out, st


def _fused(L, B, N, y2, s2, t2, W1, sbias, s1, t1, bits, W2, ks):
    lib = L.load()
    M = B * N
    y1 = torch.empty(M, 512, dtype=torch.bfloat16, device=DEV)
    out = torch.empty(M, 256, dtype=torch.bfloat16, device=DEV)
    a = L.Seg12Args(num_scenes=B, scene_rows=N, chunks_per_scene=0, y2=y2.data_ptr(), s2=s2.data_ptr(),
                    t2=t2.data_ptr(), W1=W1.data_ptr(), sbias=sbias.data_ptr(), Y1=y1.data_ptr(),
                    s1=s1.data_ptr(), t1=t1.data_ptr(), keep1=L.ptr(bits), keep_scale=ks, W2=W2.data_ptr(),
                    Y2=out.data_ptr())
    rpc = lib.pcs_fwd_seg12_geometry(ct.byref(a))
    assert rpc > 0 and rpc % 32 == 0
    st = torch.empty(B * a.chunks_per_scene, 256, 2, device=DEV)
    a.stats = st.data_ptr()
    L.call("pcs_fwd_seg12", ct.byref(a), L.stream_ptr())
    return y1, out, st, rpc


@pytest.mark.parametrize("B,N,mask", [(2, 3000, True), (3, 4097, True), (1, 100, False), (4, 2 ** 16, True),
                                      (1, 20, True), (2, 33, True)])
def test_fused_matches_two_passes(B, N, mask):
    import pcs_amd._lib as L
    ops = list(_ops(B, N, seed=B * 7 + N))
    if not mask:
        ops[7] = None
    ks = 1.0 / 0.7 if mask else 1.0
    ry1, ry2, rst = _two_pass(L, B, N, *ops, ks)
    fy1, fy2, fst, rpc = _fused(L, B, N, *ops, ks)
    torch.cuda.synchronize()
    assert torch.equal(ry1.view(torch.int16), fy1.view(torch.int16)), "Y1 differs"
    neq = int((ry2.view(torch.int16) != fy2.view(torch.int16)).sum())
    print(f"B={B} N={N}: Y2 elements differing {neq} of {fy2.numel()}")
    assert neq == 0
    # bn_seg2's statistics: the fused pass's chunk partials merged per scene against fp64
    # statistics of the stored Y2
    y = fy2.float().view(B, N, 256).double()
    ref_mean, ref_m2 = y.mean(1), ((y - y.mean(1, keepdim=True)) ** 2).sum(1)
    cps = fst.shape[0] // B
    rows = [min(rpc, N - c * rpc) for c in range(cps)]
    st = fst.double().view(B, cps, 256, 2)
    n = torch.tensor(rows, dtype=torch.float64, device=DEV)[None, :, None]
    mean = (st[..., 0] * n).sum(1) / N
    m2 = st[..., 1].sum(1) + (n * (st[..., 0] - mean[:, None, :]) ** 2).sum(1)
    assert torch.allclose(mean, ref_mean, rtol=1e-5, atol=1e-5)
    assert torch.allclose(m2, ref_m2, rtol=1e-4, atol=1e-4 * float(ref_m2.abs().max()))


def test_bn_stats_from_gram_of_a2():
    import pcs_amd._lib as L
    B, N = 3, 5000
    y2, s2, t2, W1, sbias, *_ = _ops(B, N, seed=5)
    a2 = torch.relu(y2.float() * s2 + t2).to(torch.bfloat16).float()
    G = (a2.double().T @ a2.double()).float()
    Sb = a2.view(B, N, 64).double().sum(1).float()
    W = W1.float().contiguous()
    st = torch.empty(B, 512, 2, device=DEV)
    L.call("pcs_bn_stats_gram_sbias", L.ptr(G), L.ptr(Sb), B, N, L.ptr(W), 64, 64, 512, L.ptr(sbias), L.ptr(st),
           L.stream_ptr())
    torch.cuda.synchronize()
    y = (a2.double() @ W.double().T).view(B, N, 512) + sbias.double()[:, None, :]
    mean_b = y.mean(1)
    m2w = ((y - mean_b[:, None, :]) ** 2).sum((0, 1))
    assert torch.allclose(st[..., 0].double(), mean_b, rtol=1e-5, atol=1e-5)
    assert torch.allclose(st[..., 1].double().sum(0), m2w, rtol=1e-4)


def test_train_step_fused_vs_two_passes():
    """A bf16 training step (replayed dropout masks) with the fused pass and with the two passes:
    same loss and gradients up to the Gram statistics' rounding (bn_seg1 from the Gram of a2 in
    fp32 instead of the stored Y1's own statistics)."""
    from pcs_amd.data import class_weights, synthetic_batch
    from pcs_amd.model import PointNetSegmentation
    import pointnet_oracle as orc
    B, G, C = 2, 24, 2
    pts, lab, _ = synthetic_batch(99, [G ** 3] * B, C, grid=G, dense=True)
    w = class_weights([lab[b] for b in range(B)], num_classes=C)
    sd = orc.init_params(C, 3)
    M = B * G ** 3
    gen = torch.Generator().manual_seed(1)
    m1 = torch.randint(0, 256, (M, 64), generator=gen, dtype=torch.uint8).to(DEV)
    m2 = torch.randint(0, 256, (M, 32), generator=gen, dtype=torch.uint8).to(DEV)
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV).view(-1)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    res = {}
    for fused in (True, False):
        m = PointNetSegmentation(C, compute_dtype="bf16").to(DEV)
        m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
        m.train()
        m._engine().fused_seg12 = fused
        m.set_dropout_masks(m1, m2)
        loss = crit(m(x).contiguous().view(-1, C), y)
        loss.backward()
        torch.cuda.synchronize()
        res[fused] = (float(loss), {n: p.grad.detach().double().flatten() for n, p in m.named_parameters()},
                      {n: b.detach().double() for n, b in m.named_buffers() if "running" in n})
    (lf, gf, bf), (lt, gt, bt) = res[True], res[False]
    print(f"loss fused {lf:.6f} two-pass {lt:.6f}")
    assert abs(lf - lt) < 2e-3 * max(1.0, abs(lt))
    worst = {}
    for n in gt:
        if (n.endswith(".bias") and not n.startswith(("bn", "seg_conv4"))) or n == "bn_global.bias":
            continue
        a, b = gf[n], gt[n]
        worst[n] = 1 - float(a @ b / (a.norm() * b.norm() + 1e-30))
    print("1 - cos fused vs two-pass:", {k: round(v, 6) for k, v in worst.items()})
    assert max(worst.values()) < 1e-3   # measured r05: 8e-5
    for n in bt:
        e = float((bf[n] - bt[n]).norm() / bt[n].norm())
        assert e < 1e-3, (n, e)


@pytest.mark.parametrize("B,N", [(2, 3000), (3, 4097), (1, 100), (1, 20), (2, 65)])
def test_conv3_forward_gram_of_its_operand(B, N):
    """conv3's streaming forward with the gram record (the Gram of a2 = relu(bn2(y2)) that
    bn_seg1's statistics use): y3 bit-identical to the pass without it, and the per-chunk
    [G | S] records sum to the fp64 Gram and per-scene column sums of the bf16 a2 (rows past
    each chunk's slice excluded: ragged N, one chunk smaller than a step)."""
    import pcs_amd._lib as L
    g = torch.Generator(device="cpu").manual_seed(B * 31 + N)
    M = B * N
    y2 = torch.randn(M, 64, generator=g).to(torch.bfloat16).to(DEV)
    s2, t2 = (torch.randn(64, generator=g) * 0.5 + 1.0).to(DEV), (torch.randn(64, generator=g) * 0.3).to(DEV)
    W3 = (torch.randn(64, 64, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    outs = []
    for with_gram in (False, True):
        y3 = torch.empty(M, 64, dtype=torch.bfloat16, device=DEV)
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=64, Ncols=64, dtype=L.BF16, prologue=L.PRO_BNRELU,
                       epilogue=L.EPI_FWD, chunks_per_scene=0, A=y2.data_ptr(), W=W3.data_ptr(), C=y3.data_ptr(),
                       pa=s2.data_ptr(), pb=t2.data_ptr(), a_keep_scale=1.0, c_keep_scale=1.0)
        L.load().pcs_gemm_geometry(ct.byref(a))
        cps = a.chunks_per_scene
        st = torch.empty(B * cps, 64, 2, device=DEV)
        a.stats = st.data_ptr()
        gr = torch.full((B * cps, 64 * 64 + 64), float("nan"), device=DEV)
        if with_gram:
            a.gram = gr.data_ptr()
        L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
        torch.cuda.synchronize()
        outs.append((y3, st, gr, cps))
    (y3a, sta, _, _), (y3b, stb, gr, cps) = outs
    assert torch.equal(y3a.view(torch.int16), y3b.view(torch.int16))
    assert torch.equal(sta, stb)
    assert not torch.isnan(gr).any()
    a2 = torch.relu(y2.float() * s2 + t2).to(torch.bfloat16).double()
    G = gr[:, :4096].double().sum(0).view(64, 64)
    Gref = a2.T @ a2
    err = float((G - Gref).abs().max() / Gref.abs().max())
    S = gr[:, 4096:].double().view(B, cps, 64).sum(1)
    Sref = a2.view(B, N, 64).sum(1)
    serr = float((S - Sref).abs().max() / Sref.abs().max())
    print(f"B={B} N={N}: Gram rel err {err:.2e}, column sums {serr:.2e}")
    assert err < 1e-4 and serr < 1e-4


@pytest.mark.parametrize("offset", [0.0, 2.0, 8.0])
def test_bn_seg1_gram_stats_offset_operand(offset):
    """bn_seg1's variance from the Gram route (uncentred: w (G - S S^T / N) w^T) on conv3's own
    fp32 Gram records, with a2 = relu(s2 y2 + t2) pushed away from zero by `offset` so that the
    channels of y1 = a2 W1^T have |mean| / std up to ~180: against fp64 statistics of the same
    y1, and against the direct per-chunk (mean, M2) of seg_conv1's forward GEMM (shifted sums,
    Chan merge).  The Gram route's variance error must stay below 1e-3 and within the direct
    route's error plus 2e-4 relative (a quarter of a bf16 half-ulp in the BN scale), at every
    ratio.  Measured r06 (|mean|/std 9 / 47 / 184): Gram route 4.3e-7 / 3.8e-5 / 4.7e-4, direct
    route 3.2e-4 / 7.2e-3 / 0.11 (it takes the statistics of the bf16-stored outputs, whose
    rounding noise grows with |mean|)."""
    import pcs_amd._lib as L
    lib = L.load()
    B, N = 2, 2 ** 17
    M = B * N
    g = torch.Generator(device="cpu").manual_seed(11)
    y2 = torch.randn(M, 64, generator=g).to(torch.bfloat16).to(DEV)
    s2 = (torch.rand(64, generator=g) * 0.3 + 0.1).to(DEV)
    t2 = (torch.randn(64, generator=g) * 0.1 + offset).to(DEV)
    W3 = (torch.randn(64, 64, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    W1 = (torch.randn(512, 64, generator=g) * 0.05 + 0.03).to(torch.bfloat16).to(DEV)
    sbias = (torch.randn(B, 512, generator=g) * 0.2).to(DEV)
    # conv3's forward with the gram record, reduced as the engine does (engine._seg12)
    y3 = torch.empty(M, 64, dtype=torch.bfloat16, device=DEV)   # (held: the kernel writes it)
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=64, Ncols=64, dtype=L.BF16, prologue=L.PRO_BNRELU,
                   epilogue=L.EPI_FWD, chunks_per_scene=0, A=y2.data_ptr(), W=W3.data_ptr(), C=y3.data_ptr(),
                   pa=s2.data_ptr(), pb=t2.data_ptr(), a_keep_scale=1.0, c_keep_scale=1.0)
    lib.pcs_gemm_geometry(ct.byref(a))
    cps = a.chunks_per_scene
    st3 = torch.empty(B * cps, 64, 2, device=DEV)
    rec = 64 * 64 + 64
    gr = torch.empty(B * cps, rec, device=DEV)
    a.stats, a.gram = st3.data_ptr(), gr.data_ptr()
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    per_scene = torch.empty(B, rec, device=DEV)
    L.call("pcs_reduce_partials_grouped", L.ptr(gr), B, cps, rec, 1.0, L.ptr(per_scene), L.stream_ptr())
    tot = torch.empty(rec, device=DEV)
    L.call("pcs_reduce_partials", L.ptr(per_scene), B, rec, 1.0, L.ptr(tot), 1, rec, L.stream_ptr())
    Wf = W1.float().contiguous()
    stg = torch.empty(B, 512, 2, device=DEV)
    L.call("pcs_bn_stats_gram_sbias", L.ptr(tot[:4096]), L.ptr(per_scene[:, 4096:].contiguous()), B, N, L.ptr(Wf),
           64, 64, 512, L.ptr(sbias), L.ptr(stg), L.stream_ptr())
    # the direct route: seg_conv1's forward GEMM with per-chunk statistics of its fp32 outputs
    y1 = torch.empty(M, 512, dtype=torch.bfloat16, device=DEV)
    b = L.GemmArgs(num_scenes=B, scene_rows=N, K=64, Ncols=512, dtype=L.BF16, prologue=L.PRO_BNRELU,
                   epilogue=L.EPI_FWD, chunks_per_scene=0, A=y2.data_ptr(), W=W1.data_ptr(), C=y1.data_ptr(),
                   pa=s2.data_ptr(), pb=t2.data_ptr(), scene_bias=sbias.data_ptr(), a_keep_scale=1.0, c_keep_scale=1.0)
    lib.pcs_gemm_geometry(ct.byref(b))
    cpd = b.chunks_per_scene
    std = torch.empty(B * cpd, 512, 2, device=DEV)
    b.stats = std.data_ptr()
    L.call("pcs_gemm", ct.byref(b), L.stream_ptr())
    torch.cuda.synchronize()
    a2 = torch.relu(y2.float() * s2 + t2).to(torch.bfloat16).double()
    y = (a2 @ W1.double().T).view(B, N, 512) + sbias.double()[:, None, :]
    mean_b = y.mean(1)
    var = ((y - y.mean((0, 1))) ** 2).mean((0, 1))
    ratio = float((y.mean((0, 1)).abs() / var.sqrt()).max())

    def total_var(mb, m2b):   # per-scene (mean, M2) pairs -> the batch variance (Chan)
        mu = mb.mean(0)
        return (m2b.sum(0) + N * ((mb - mu) ** 2).sum(0)) / M

    vg = total_var(stg[..., 0].double(), stg[..., 1].double())
    sd = std.double().view(B, cpd, 512, 2)
    rps = lib.pcs_gemm_geometry(ct.byref(b))
    rows = torch.tensor([min(rps, N - c * rps) for c in range(cpd)], dtype=torch.float64, device=DEV)[None, :, None]
    md = (sd[..., 0] * rows).sum(1) / N
    m2d = sd[..., 1].sum(1) + (rows * (sd[..., 0] - md[:, None, :]) ** 2).sum(1)
    vd = total_var(md, m2d)
    eg = float(((vg - var).abs() / var).max())
    ed = float(((vd - var).abs() / var).max())
    emg = float(((stg[..., 0].double() - mean_b).abs() / var.sqrt()).max())
    print(f"offset {offset}: max |mean|/std {ratio:.1f}; variance rel err Gram route {eg:.2e}, direct route "
          f"{ed:.2e}; Gram-route mean err / std {emg:.2e}")
    assert emg < 1e-4
    assert eg < 1e-3 and eg <= ed + 2e-4

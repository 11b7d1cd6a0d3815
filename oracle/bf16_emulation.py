"""bf16-storage emulation of the PointNetSegmentation training step (numpy float32).

TEST / ANALYSIS INFRASTRUCTURE ONLY (same rule as pointnet_oracle.py: never imported by the
product path).  It answers one question about the bf16 bench path: is its gradient error at
large scenes a property of storing activations and gradients in bf16, or of a kernel?

``train_step(sd, x, labels, weight, masks, store)`` runs the reference step (forward P:98-133,
weighted CE P:216/251, backward P:254) in float32 arithmetic.  With ``store="fp32"`` nothing
is rounded (a plain fp32 restatement).  With ``store="bf16"`` every tensor the HIP bf16 path
keeps in bf16 is rounded to bf16 (round-to-nearest-even) at the point the HIP path rounds it
(point-cloud-cnn-segmentation_amd/engine.py), everything else stays fp32:

* forward: GEMM weights (conv2..conv5, global_feat, seg_conv1's local half, seg_conv2/3;
  conv1, seg_conv4 and seg_conv1's global half stay fp32); every stored pre-BN output Y_l
  (BN statistics from the stored values, as the GEMM epilogues compute them); every GEMM
  input activation a_l = relu(bn(Y_l)) [* dropout]; a5 = relu(bn5(y5)) (conv5's statistics
  and global_feat's statistics / max-pool from fp32 accumulators, as the Gram-derived bn5
  statistics and the LDS-DMA epilogue do); the head works in fp32;
* backward: every stored dZ_l (the BN-output gradient after ReLU / dropout; its sums S1 / S2
  from the fp32 values, as the producing epilogues form them); every GEMM operand dy_l; the
  folded global_feat / conv5 operands H and diag(alpha) W (the Gram-form weight gradients,
  the pool rows and the per-scene sums csum_b stay fp32).

With ``store="fp8"`` the bf16 rounding above applies and, as the HIP fp8 path (compute dtype
"fp8") stores them, a5 is rounded to e4m3 (OCP e4m3fn, nearest-even, saturating at 448) and
global_feat's weight and the folded H are e4m3 rows with one power-of-two scale each
(pcs_quant_fp8_rows: scale 2^ceil(log2(row max / 448))); the max-pool rows and the
Gram-form weight gradient use the dequantized global_feat weight, as the HIP path does.
``return_logits=True`` also returns the logits (float32 [M, C]).

``eval_logits(sd, x, sites)`` is the EVAL forward (BatchNorm running statistics, no dropout;
P:98-133 under model.eval(), P:313) in float32 with a chosen set of bf16 rounding sites, as
the HIP bf16 eval path (engine.Engine.forward, train=False) rounds them; ``eval_sites(trunk)``
names the sites of that path with ``eval_trunk`` = "bf16" or "fp32" (tools/miou_attr.py
attributes the eval logit error site by site).

Memory is kept to the tensors the backward needs (about 9 KB per point plus a few [M, 1024]
temporaries), so 4 scenes x 64^3 points run on a 64 GB host.
"""
from __future__ import annotations

import numpy as np

from pointnet_oracle import BN_EPS, DROPOUT_P, _w

F32 = np.float32


def round_bf16(a):
    """float32 -> nearest-even bf16, returned as float32 (finite inputs)."""
    a = np.ascontiguousarray(a, dtype=F32)
    u = a.view(np.uint32)
    r = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) & np.uint32(0xFFFF0000)
    return r.view(F32)


def round_e4m3(a):
    """float32 -> nearest-even e4m3fn (4 significant bits, subnormal step 2^-9, |x| <= 448),
    returned as float32."""
    a = np.asarray(a, dtype=np.float64)
    _, e = np.frexp(a)                                    # |a| in [2^(e-1), 2^e)
    q = np.exp2(np.maximum(e - 4, -9).astype(np.float64))  # quantum of a's binade
    r = np.round(a / q) * q                              # np.round: half to even
    return np.clip(r, -448.0, 448.0).astype(F32)


def quant_rows_e4m3(W):
    """Row-scaled e4m3 copy of W (dequantized float32), as pcs_quant_fp8_rows."""
    W = np.asarray(W, dtype=F32)
    mx = np.abs(W).max(axis=1).astype(np.float64)
    e = np.where(mx > 0, np.ceil(np.log2(np.where(mx > 0, mx, 1.0) / 448.0)), 0.0)
    e = np.clip(e, -126, 127)
    return (round_e4m3(W * np.exp2(-e)[:, None].astype(F32)).astype(np.float64) * np.exp2(e)[:, None]).astype(F32)


def _stats(Y):
    """Batch mean and biased variance per column, fp64 accumulation (the HIP finalisation
    merges fp32 partials in fp64)."""
    mean = Y.mean(axis=0, dtype=np.float64)
    var = np.zeros(Y.shape[1], np.float64)
    step = 1 << 18
    for i in range(0, Y.shape[0], step):
        d = Y[i:i + step].astype(np.float64) - mean
        var += (d * d).sum(axis=0)
    return mean, var / Y.shape[0]


def train_step(sd, x, labels, weight, masks, store="bf16", p=DROPOUT_P, return_logits=False, exact=(), pool_idx=None, info=None):
    """One reference training step (without the optimizer).  Returns (loss, grads) with
    grads keyed by state-dict parameter name (float64 arrays); conv biases that BN cancels
    are returned as zeros (analytically ~0 in every path).

    ``exact``: names of rounding sites left in fp32 (the ablation of tools/bf16_ablation.py):
    "W" (every GEMM weight), "Y" (stored pre-BN outputs), "A" (GEMM input activations except
    a5), "a5", "dz" (stored BN-output gradients), "dy" (GEMM operands dy), "DZ5", "H" (folded
    global_feat H), "fold5" (conv5's folded operands), "dA2", "dA4".  ``pool_idx`` [B, 1024]
    replaces the max-pool's argmax rows (the value pooled is still this path's own); a dict
    ``info`` receives this step's own argmax rows under "pool_idx"."""
    R0 = round_bf16 if store in ("bf16", "fp8") else (lambda a: np.ascontiguousarray(a, dtype=F32))
    exact = set(exact)

    def R(a, site=None):
        return np.ascontiguousarray(a, dtype=F32) if site in exact else R0(a)
    fp8 = store == "fp8"
    B, N, D = x.shape
    M = B * N
    X = x.reshape(M, D).astype(F32)
    W = {n: _w(sd, n, F32) for n in ("conv1", "conv2", "conv3", "conv4", "conv5", "global_feat",
                                    "seg_conv1", "seg_conv2", "seg_conv3", "seg_conv4")}
    Wr = {n: R(W[n], "W") for n in ("conv2", "conv3", "conv4", "conv5", "global_feat", "seg_conv2", "seg_conv3")}
    Wr["seg_conv1_l"] = R(W["seg_conv1"][:, :64], "W")
    if fp8:
        Wr["global_feat"] = quant_rows_e4m3(W["global_feat"])
    Wg1 = np.ascontiguousarray(W["seg_conv1"][:, 64:])     # global half: fp32 (pcs_scene_gemv)
    gam = {bn: sd[f"{bn}.weight"].astype(np.float64) for bn in
           ("bn1", "bn2", "bn3", "bn4", "bn5", "bn_global", "bn_seg1", "bn_seg2", "bn_seg3")}
    bet = {bn: sd[f"{bn}.bias"].astype(np.float64) for bn in gam}
    keep = 1.0 / (1.0 - p)
    k1 = masks[0].astype(F32) * F32(keep)
    k2 = masks[1].astype(F32) * F32(keep)
    cache = {}

    def bn_coef(bn, mean, var):
        rstd = 1.0 / np.sqrt(var + BN_EPS)
        scale = gam[bn] * rstd
        shift = bet[bn] - mean * scale
        cache[bn] = (mean, rstd)
        return scale.astype(F32), shift.astype(F32)

    def act(Y, bn, k=None):
        s, t = cache[bn + "_st"]
        a = np.maximum(Y * s + t, F32(0))
        return a * k if k is not None else a

    def layer(A, bn, Wt):
        Y = R(A @ Wt.T, "Y")                                  # stored pre-BN (bias cancels in BN)
        cache[bn + "_st"] = bn_coef(bn, *_stats(Y))
        return Y

    # ---------------- forward (P:103-131)
    Y1 = R(X @ W["conv1"].T, "Y")
    cache["bn1_st"] = bn_coef("bn1", *_stats(Y1))
    Y2 = layer(R(act(Y1, "bn1"), "A"), "bn2", Wr["conv2"])
    A2 = R(act(Y2, "bn2"), "A")                               # point_feat (conv3 / seg_conv1 input)
    Y3 = layer(A2, "bn3", Wr["conv3"])
    A3 = R(act(Y3, "bn3"), "A")
    Y4 = layer(A3, "bn4", Wr["conv4"])
    A4 = R(act(Y4, "bn4"), "A")
    y5 = A4 @ Wr["conv5"].T                              # fp32 accumulators
    cache["bn5_st"] = bn_coef("bn5", *_stats(y5))
    a5 = round_e4m3(act(y5, "bn5")) if fp8 else R(act(y5, "bn5"), "a5")
    del y5
    yg = a5 @ Wr["global_feat"].T
    mg, vg = _stats(yg)
    sg, tg = bn_coef("bn_global", mg, vg)
    cache["bn_global_st"] = (sg, tg)
    zg = (yg * sg + tg).reshape(B, N, -1)
    idx = zg.argmax(axis=1) if pool_idx is None else np.asarray(pool_idx)   # first max (P:114)
    if info is not None:
        info["pool_idx"] = zg.argmax(axis=1)
    g = np.maximum(np.take_along_axis(zg, idx[:, None, :], 1)[:, 0, :], 0).astype(np.float64)
    ysel = np.take_along_axis(yg.reshape(B, N, -1), idx[:, None, :], 1)[:, 0, :].astype(np.float64)
    del yg, zg
    sb = g @ Wg1.T.astype(np.float64)                    # per-scene bias (P:117-123), centred
    sb -= sb.mean(axis=0)
    Ys1 = R((A2 @ Wr["seg_conv1_l"].T).reshape(B, N, -1) + sb[:, None, :].astype(F32), "Y").reshape(M, -1)
    cache["bn_seg1_st"] = bn_coef("bn_seg1", *_stats(Ys1))
    As1 = R(act(Ys1, "bn_seg1", k1), "A")
    Ys2 = layer(As1, "bn_seg2", Wr["seg_conv2"])
    As2 = R(act(Ys2, "bn_seg2", k2), "A")
    Ys3 = layer(As2, "bn_seg3", Wr["seg_conv3"])
    as3 = act(Ys3, "bn_seg3")                            # head: fp32
    logits = as3 @ W["seg_conv4"].T + sd["seg_conv4.bias"].astype(F32)

    # ---------------- weighted CE (P:216, P:251)
    y = labels.reshape(-1)
    valid = y >= 0
    ys = np.where(valid, y, 0)
    z = logits.astype(np.float64)
    mx = z.max(axis=1, keepdims=True)
    e = np.exp(z - mx)
    se = e.sum(axis=1, keepdims=True)
    wv = np.where(valid, np.asarray(weight, np.float64)[ys], 0.0)
    den = wv.sum()
    loss = float((wv * (mx[:, 0] + np.log(se[:, 0]) - z[np.arange(M), ys])).sum() / den)
    dl = e / se
    dl[np.arange(M), ys] -= 1.0
    dl = (dl * (wv / den)[:, None]).astype(F32)
    del e, z

    # ---------------- backward (P:254)
    grads = {}
    grads["seg_conv4.weight"] = (dl.T.astype(np.float64) @ as3)[:, :, None]
    grads["seg_conv4.bias"] = dl.sum(axis=0, dtype=np.float64)
    dA = dl @ W["seg_conv4"]

    def bn_back(dA, Y, bn, k=None):
        """dZ after ReLU (and dropout) -> stored R(dZ); S1/S2 from fp32; dy = R(alpha dZ + beta
        + gamma Y) in the GEMM operand dtype.  Also returns dy before rounding (pool sums)."""
        mean, rstd = cache[bn]
        s, t = cache[bn + "_st"]
        pos = (Y * s + t) > 0
        dz = np.where(pos, dA * k if k is not None else dA, F32(0))
        xh = ((Y.astype(np.float64) - mean) * rstd)
        S1 = dz.sum(axis=0, dtype=np.float64)
        S2 = (dz * xh).sum(axis=0)
        grads[f"{bn}.weight"], grads[f"{bn}.bias"] = S2, S1
        al = gam[bn] * rstd
        dy = (al * (R(dz, "dz").astype(np.float64) - S1 / M - xh * (S2 / M))).astype(F32)
        return dy, S1, S2

    def conv_back(conv, dy, Ain, Wt, need_dx=True):
        dyr = R(dy, "dy")
        grads[f"{conv}.weight"] = (dyr.T.astype(np.float64) @ Ain)[:, :, None]
        grads[f"{conv}.bias"] = np.zeros(dy.shape[1])
        return dyr @ Wt if need_dx else None

    dy, _, _ = bn_back(dA, Ys3, "bn_seg3")
    dA = conv_back("seg_conv3", dy, As2, Wr["seg_conv3"])
    dy, _, _ = bn_back(dA, Ys2, "bn_seg2", k2)
    dA = conv_back("seg_conv2", dy, As1, Wr["seg_conv2"])
    dys1, _, _ = bn_back(dA, Ys1, "bn_seg1", k1)
    del dA
    # seg_conv1 = local GEMM + per-scene global GEMV: dW = [dy^T A2 | sum_b csum_b g_b^T]
    dyr = R(dys1, "dy")
    dWl = dyr.T.astype(np.float64) @ A2
    csum = dys1.reshape(B, N, -1).sum(axis=1, dtype=np.float64)    # fp32 sums (pcs_pool_bwd)
    grads["seg_conv1.weight"] = np.concatenate([dWl, csum.T @ g], axis=1)[:, :, None]
    grads["seg_conv1.bias"] = np.zeros(dys1.shape[1])
    dA2 = R(dyr @ Wr["seg_conv1_l"], "dA2")                                  # stored (conv3 addend)
    del dys1, dyr
    # max-pool + bn_global backward (sparse rows), folded dA5 = a5 H + c + sparse
    dg = csum @ Wg1.astype(np.float64)                                # [B, 1024]
    mean, rstd = cache["bn_global"]
    sgl, tgl = cache["bn_global_st"]
    dzs = np.where(ysel * sgl + tgl > 0, dg, 0.0)
    xs = (ysel - mean) * rstd
    S1 = dzs.sum(axis=0)
    S2 = (dzs * xs).sum(axis=0)
    grads["bn_global.weight"], grads["bn_global.bias"] = S2, S1
    al = gam["bn_global"] * rstd
    gc = -al * rstd * S2 / M
    bc = -al * S1 / M - gc * mean
    Wgr = Wr["global_feat"].astype(np.float64)
    H = quant_rows_e4m3((Wgr.T * gc) @ Wgr) if fp8 else R((Wgr.T * gc) @ Wgr, "H")
    cvec = (Wgr.T @ bc).astype(F32)
    dA5 = a5 @ H + cvec
    rows = idx + (np.arange(B) * N)[:, None]
    sp = al * dzs                                                     # [B, 1024]
    Wg32 = Wgr if fp8 else W["global_feat"].astype(np.float64)
    for b in range(B):
        np.add.at(dA5, rows[b], (sp[b][:, None] * Wg32).astype(F32))
    dz5 = np.where(a5 > 0, dA5, F32(0))
    del dA5
    S1_5 = dz5.sum(axis=0, dtype=np.float64)
    DZ5 = R(dz5, "DZ5")
    del dz5
    G5 = (a5.T @ a5).astype(np.float64)                               # fp32 accumulation
    S5 = a5.sum(axis=0, dtype=np.float64)
    dWg = np.outer(bc, S5) + (gc[:, None] * Wgr) @ G5
    for b in range(B):                                                # the max-pool rows
        dWg += sp[b][:, None] * a5[rows[b]].astype(np.float64)
    grads["global_feat.weight"] = dWg[:, :, None]
    grads["global_feat.bias"] = np.zeros(1024)
    del G5
    # conv5 folded backward (R = dz5^T a4 gives S2 and the alpha term of dW5)
    mean, rstd = cache["bn5"]
    Rm = DZ5.T.astype(np.float64) @ A4                                 # [1024, 128]
    W5r = Wr["conv5"].astype(np.float64)
    mu_y = mean
    S2_5 = rstd * ((W5r * Rm).sum(axis=1) - mu_y * S1_5)
    grads["bn5.weight"], grads["bn5.bias"] = S2_5, S1_5
    al5 = gam["bn5"] * rstd
    ga5 = -al5 * rstd * S2_5 / M
    be5 = -al5 * S1_5 / M - ga5 * mean
    Ws = R(al5[:, None] * W5r, "fold5")
    h4 = R((W5r.T * ga5) @ W5r, "fold5")
    c5 = (W5r.T @ be5).astype(F32)
    dA4 = R(DZ5 @ Ws + c5, "dA4") + A4 @ h4
    del DZ5
    G4 = A4.T.astype(np.float64) @ A4
    S4 = A4.sum(axis=0, dtype=np.float64)
    grads["conv5.weight"] = (al5[:, None] * Rm + np.outer(be5, S4) + (ga5[:, None] * W5r) @ G4)[:, :, None]
    grads["conv5.bias"] = np.zeros(1024)
    dy, _, _ = bn_back(dA4, Y4, "bn4")
    dA = conv_back("conv4", dy, A3, Wr["conv4"])
    dy, _, _ = bn_back(dA, Y3, "bn3")
    dA = conv_back("conv3", dy, A2, Wr["conv3"]) + dA2
    dy, _, _ = bn_back(dA, Y2, "bn2")
    A1 = R(act(Y1, "bn1"), "A")
    dA = conv_back("conv2", dy, A1, Wr["conv2"])
    mean, rstd = cache["bn1"]
    s, t = cache["bn1_st"]
    dz = np.where((Y1 * s + t) > 0, dA, F32(0))
    xh = (Y1.astype(np.float64) - mean) * rstd
    S1 = dz.sum(axis=0, dtype=np.float64)
    S2 = (dz * xh).sum(axis=0)
    grads["bn1.weight"], grads["bn1.bias"] = S2, S1
    dy = gam["bn1"] * rstd * (R(dz, "dz").astype(np.float64) - S1 / M - xh * (S2 / M))   # conv1 wgrad: fp32 dy
    grads["conv1.weight"] = (dy.T @ X.astype(np.float64))[:, :, None]
    grads["conv1.bias"] = np.zeros(64)
    if return_logits:
        return loss, grads, logits
    return loss, grads


# ------------------------------------------------------------------ eval forward
EVAL_LAYERS = ("conv1", "conv2", "conv3", "conv4", "seg_conv1", "seg_conv2", "seg_conv3")
_TRUNK = ("conv1", "conv2", "conv3", "conv4")


def eval_sites(trunk="bf16"):
    """bf16 rounding sites of the HIP eval forward.  Names: W<l> (GEMM weight), Y<l> (stored
    pre-BN output), A<l> (relu(bn(Y_l)) as the next GEMM's operand; "Aconv2s" is seg_conv1's
    copy of a2), "a5" (stored relu(bn5(y5))), "Asplit4" (conv5's operand as the 16-bit split
    [hi | lo] of pcs_bnrelu_bf16: hi = bf16(a4), lo = bf16(a4 - hi), so conv5 sees hi + lo).
    trunk="fp32": conv1..conv4 stored and computed in fp32, seg_conv1 fed a bf16 a2, conv5 fed
    the split of a4."""
    s = {"a5", "Wglobal_feat", "Wconv5", "Aconv2s"}
    for l in EVAL_LAYERS:
        s |= {f"Y{l}", f"A{l}"}
        if l != "conv1":
            s.add(f"W{l}")
    s.discard("Aseg_conv3")           # the head reads bn_seg3's output in fp32
    if trunk == "fp32":
        s -= {f"{k}{l}" for l in _TRUNK for k in "YAW"}
        s.add("Asplit4")
    return frozenset(s)


def eval_logits(sd, x, sites, fp8=False, sums="f32"):
    """float32 eval forward with the bf16 rounding ``sites`` (eval_sites); logits [B, N, C].
    Stored pre-BN outputs omit the conv bias as the HIP path's do (seg_conv1's per-scene bias
    centred over the scenes).  fp8=True: a5 in e4m3 and global_feat's weight as e4m3 rows with
    one power-of-two scale each (the compute dtype "fp8"), whatever ``sites`` holds for them.
    relu(bn(y)) = max(fma(y, s, t), 0) with one rounding, as the kernels' fmaf.
    ``sums``: "f32" sums every GEMM in float32 (BLAS order), "f64" in float64 rounded once to
    float32 -- another valid order of the same arithmetic, whose distance from the "f32" result
    is the rounding-order noise floor a device-vs-emulation comparison cannot go below."""
    def R(a, site):
        if fp8 and site == "a5":
            return round_e4m3(a)
        if fp8 and site == "Wglobal_feat":
            return quant_rows_e4m3(a)
        return round_bf16(a) if site in sites else np.ascontiguousarray(a, dtype=F32)
    B, N, D = x.shape
    M = B * N
    X = x.reshape(M, D).astype(F32)
    W = {n: _w(sd, n, F32) for n in ("conv1", "conv2", "conv3", "conv4", "conv5", "global_feat",
                                    "seg_conv1", "seg_conv2", "seg_conv3", "seg_conv4")}

    def coefs(bn, off):
        g = sd[f"{bn}.weight"].astype(np.float64)
        rm = sd[f"{bn}.running_mean"].astype(np.float64)
        sc = g / np.sqrt(sd[f"{bn}.running_var"].astype(np.float64) + BN_EPS)
        return sc.astype(F32), (sd[f"{bn}.bias"].astype(np.float64) - (rm - off) * sc).astype(F32)

    def mm(A, Wt):   # A @ Wt.T
        if sums == "f64":
            return (np.asarray(A, np.float64) @ np.asarray(Wt, np.float64).T).astype(F32)
        return A @ Wt.T

    def layer(A, conv, bn, Wt):
        Y = R(mm(A, Wt), f"Y{conv}")
        return Y, *coefs(bn, sd[f"{conv}.bias"].astype(np.float64))

    def relu_bn(Y, s, t):   # fma: the product and sum of two float32 are exact in float64
        return np.maximum((Y.astype(np.float64) * s + t).astype(F32), F32(0))

    Y, s, t = layer(X, "conv1", "bn1", W["conv1"])
    Y, s, t = layer(R(relu_bn(Y, s, t), "Aconv1"), "conv2", "bn2", R(W["conv2"], "Wconv2"))
    A2 = relu_bn(Y, s, t)
    Y, s, t = layer(R(A2, "Aconv2"), "conv3", "bn3", R(W["conv3"], "Wconv3"))
    Y, s, t = layer(R(relu_bn(Y, s, t), "Aconv3"), "conv4", "bn4", R(W["conv4"], "Wconv4"))
    A4 = R(relu_bn(Y, s, t), "Aconv4")
    if "Asplit4" in sites:   # engine.Engine.forward's bridge("conv4", "bn4", 128, True)
        hi = round_bf16(A4)
        A4 = hi + round_bf16(A4 - hi)   # exact in fp32 (16 significant bits)
    s5, t5 = coefs("bn5", sd["conv5.bias"].astype(np.float64))
    a5 = R(relu_bn(mm(A4, R(W["conv5"], "Wconv5")), s5, t5), "a5")          # fp32 accumulators
    sg, tg = coefs("bn_global", sd["global_feat.bias"].astype(np.float64))
    zg = (mm(a5, R(W["global_feat"], "Wglobal_feat")).astype(np.float64) * sg + tg).astype(F32).reshape(B, N, -1)
    g = np.maximum(zg.max(axis=1), 0).astype(np.float64)                   # P:114
    del zg
    sb = g @ W["seg_conv1"][:, 64:].T.astype(np.float64) + sd["seg_conv1.bias"]   # [B, 512]
    soff = sb.mean(axis=0)
    a2s = R(A2, "Aconv2" if "Aconv2" in sites else "Aconv2s")
    Ys1 = R(mm(a2s, R(W["seg_conv1"][:, :64], "Wseg_conv1")).reshape(B, N, -1)
            + (sb - soff)[:, None, :].astype(F32), "Yseg_conv1").reshape(M, -1)
    s, t = coefs("bn_seg1", soff)
    Y, s, t = layer(R(relu_bn(Ys1, s, t), "Aseg_conv1"), "seg_conv2", "bn_seg2", R(W["seg_conv2"], "Wseg_conv2"))
    Y, s, t = layer(R(relu_bn(Y, s, t), "Aseg_conv2"), "seg_conv3", "bn_seg3", R(W["seg_conv3"], "Wseg_conv3"))
    return (mm(relu_bn(Y, s, t), W["seg_conv4"]) + sd["seg_conv4.bias"].astype(F32)).reshape(B, N, -1)

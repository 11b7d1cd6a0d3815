"""CPU oracle: numpy restatement of the reference PointNetSegmentation training step.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker
(or as the timed CPU baseline).  The product path (``pcs_amd``) never calls it and
fails loudly when its HIP library is missing.

Every function restates the reference algorithm of
``/root/reference/point_cloud_segmentation.py`` (cited below as ``P:<line>``) with
explicit formulas: forward in train/eval mode, weighted cross-entropy with
``ignore_index=-1``, a hand-written backward (no autograd), BatchNorm running-stat
updates and the L2-weight-decay Adam step.  Arithmetic runs in the dtype passed in
(float64 by default, which is what the parity tests use).

Parity pinning: ``tests/test_oracle_golden.py`` checks this oracle against golden
vectors produced by the imported reference itself (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import numpy as np

BN_EPS = 1e-5          # nn.BatchNorm1d default (P:86-94)
BN_MOMENTUM = 0.1      # nn.BatchNorm1d default
DROPOUT_P = 0.3        # nn.Dropout(0.3) (P:96)

# (conv name, Cin, Cout, bn name or None) in registration order (P:70-94).
# Cin of conv1 / Cout of seg_conv4 are filled in by layer_table().
_LAYERS = [
    ("conv1", None, 64, "bn1"),
    ("conv2", 64, 64, "bn2"),
    ("conv3", 64, 64, "bn3"),
    ("conv4", 64, 128, "bn4"),
    ("conv5", 128, 1024, "bn5"),
    ("global_feat", 1024, 1024, "bn_global"),
    ("seg_conv1", 1088, 512, "bn_seg1"),
    ("seg_conv2", 512, 256, "bn_seg2"),
    ("seg_conv3", 256, 128, "bn_seg3"),
    ("seg_conv4", 128, None, None),
]


def layer_table(num_classes: int, input_dim: int = 4):
    """[(conv, Cin, Cout, bn)] for PointNetSegmentation(num_classes, input_dim) (P:66-96)."""
    out = []
    for conv, cin, cout, bn in _LAYERS:
        out.append((conv, input_dim if cin is None else cin,
                    num_classes if cout is None else cout, bn))
    return out


def state_dict_keys(num_classes: int, input_dim: int = 4):
    """The 65 state-dict keys in registration order: 10 convs then 9 BNs (P:70-94)."""
    keys = []
    for conv, _, _, _ in layer_table(num_classes, input_dim):
        keys += [f"{conv}.weight", f"{conv}.bias"]
    for _, _, cout, bn in layer_table(num_classes, input_dim):
        if bn:
            keys += [f"{bn}.weight", f"{bn}.bias", f"{bn}.running_mean",
                     f"{bn}.running_var", f"{bn}.num_batches_tracked"]
    return keys


def init_params(num_classes: int, seed: int, input_dim: int = 4, bn_affine_random: bool = False):
    """Seeded parameters in the reference state-dict layout (numpy PCG64).

    Conv weights/biases follow the distribution of torch's default Conv1d init
    (kaiming_uniform(a=sqrt 5) => U(+-1/sqrt(fan_in)); bias U(+-1/sqrt(fan_in))) but are
    drawn from numpy so fixtures need not carry 7.7 MB of weights.  BN gamma=1, beta=0,
    running_mean=0, running_var=1 unless ``bn_affine_random`` (then gamma in
    +-[0.5,1.5] with random sign, beta ~ U(-0.5,0.5), running stats random positive),
    which exercises the negative-scale branch of the max-pool.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for conv, cin, cout, bn in layer_table(num_classes, input_dim):
        bound = 1.0 / np.sqrt(cin)
        sd[f"{conv}.weight"] = rng.uniform(-bound, bound, size=(cout, cin, 1)).astype(np.float32)
        sd[f"{conv}.bias"] = rng.uniform(-bound, bound, size=(cout,)).astype(np.float32)
    for conv, cin, cout, bn in layer_table(num_classes, input_dim):
        if not bn:
            continue
        if bn_affine_random:
            mag = rng.uniform(0.5, 1.5, size=(cout,))
            sign = np.where(rng.uniform(size=(cout,)) < 0.3, -1.0, 1.0)
            sd[f"{bn}.weight"] = (mag * sign).astype(np.float32)
            sd[f"{bn}.bias"] = rng.uniform(-0.5, 0.5, size=(cout,)).astype(np.float32)
            sd[f"{bn}.running_mean"] = rng.uniform(-0.5, 0.5, size=(cout,)).astype(np.float32)
            sd[f"{bn}.running_var"] = rng.uniform(0.5, 2.0, size=(cout,)).astype(np.float32)
        else:
            sd[f"{bn}.weight"] = np.ones(cout, np.float32)
            sd[f"{bn}.bias"] = np.zeros(cout, np.float32)
            sd[f"{bn}.running_mean"] = np.zeros(cout, np.float32)
            sd[f"{bn}.running_var"] = np.ones(cout, np.float32)
        sd[f"{bn}.num_batches_tracked"] = np.array(0, np.int64)
    return sd


def dropout_masks(seed: int, M: int, p: float = DROPOUT_P):
    """Two independent Bernoulli(1-p) keep masks [M,512] and [M,256] (uint8).

    The reference reuses one nn.Dropout module twice (P:124, P:126), so there are two
    independent masks per forward.  Tests replay these into the reference and into the
    HIP path so that train-mode outputs are comparable.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    m1 = (rng.uniform(size=(M, 512)) >= p).astype(np.uint8)
    m2 = (rng.uniform(size=(M, 256)) >= p).astype(np.uint8)
    return m1, m2


# --------------------------------------------------------------------------------------
# data layout (P:44-63)
# --------------------------------------------------------------------------------------

def collate(points_list, labels_list):
    """Pad a ragged list of clouds to the batch max (P:44-63).

    Pads are (0,0,0,0) points with label -1 and mask False; the model sees them.
    """
    B = len(points_list)
    N = max(p.shape[0] for p in points_list)
    pts = np.zeros((B, N, 4), np.float32)
    lab = np.full((B, N), -1, np.int64)
    msk = np.zeros((B, N), bool)
    for i, (p, l) in enumerate(zip(points_list, labels_list)):
        n = p.shape[0]
        pts[i, :n] = p
        lab[i, :n] = l
        msk[i, :n] = True
    return pts, lab, msk


# --------------------------------------------------------------------------------------
# forward (P:98-133)
# --------------------------------------------------------------------------------------

def _w(sd, name, dt):
    return sd[f"{name}.weight"].reshape(sd[f"{name}.weight"].shape[0], -1).astype(dt)


def _bn_train(y, gamma, beta, eps=BN_EPS):
    """BatchNorm1d train mode over all rows of y [M,C] (pads included; P:106-127)."""
    mean = y.mean(axis=0)
    var = ((y - mean) ** 2).mean(axis=0)          # biased variance for normalisation
    rstd = 1.0 / np.sqrt(var + eps)
    xhat = (y - mean) * rstd
    return xhat * gamma + beta, (mean, var, rstd, xhat)


def _bn_eval(y, gamma, beta, rm, rv, eps=BN_EPS):
    return (y - rm) / np.sqrt(rv + eps) * gamma + beta


def forward(sd, x, train=True, masks=None, p=DROPOUT_P, dtype=np.float64):
    """PointNetSegmentation.forward (P:98-133) on x [B,N,input_dim].

    Returns (logits [B,N,C], cache).  In train mode ``masks`` = (keep1 [M,512],
    keep2 [M,256]) replays the two dropout draws (None => p treated as 0).
    ``cache['bn_stats'][bn] = (batch mean, biased var)`` for the running-stat update.
    """
    dt = dtype
    B, N, _ = x.shape
    M = B * N
    X0 = x.reshape(M, -1).astype(dt)                      # P:103 transpose -> points-major
    cache = {"B": B, "N": N, "x": X0, "train": train, "p": p, "bn": {}, "bn_stats": {}}

    def block(Xin, conv, bn):
        W = _w(sd, conv, dt)
        y = Xin @ W.T + sd[f"{conv}.bias"].astype(dt)
        g = sd[f"{bn}.weight"].astype(dt)
        b = sd[f"{bn}.bias"].astype(dt)
        if train:
            z, st = _bn_train(y, g, b)
            cache["bn"][bn] = st
            cache["bn_stats"][bn] = (st[0], st[1])
        else:
            z = _bn_eval(y, g, b, sd[f"{bn}.running_mean"].astype(dt),
                         sd[f"{bn}.running_var"].astype(dt))
        a = np.maximum(z, 0)
        cache[conv] = {"in": Xin, "y": y, "z": z, "a": a}
        return a

    a1 = block(X0, "conv1", "bn1")                          # P:106
    a2 = block(a1, "conv2", "bn2")                          # P:107 point_feat
    a3 = block(a2, "conv3", "bn3")                          # P:108
    a4 = block(a3, "conv4", "bn4")                          # P:109
    a5 = block(a4, "conv5", "bn5")                          # P:110
    ag = block(a5, "global_feat", "bn_global")              # P:113
    agb = ag.reshape(B, N, -1)
    idx = agb.argmax(axis=1)                                # first max, P:114
    g = np.take_along_axis(agb, idx[:, None, :], axis=1)[:, 0, :]   # [B,1024]
    cache["pool"] = {"idx": idx, "g": g}
    gexp = np.repeat(g, N, axis=0)                          # P:117 repeat (row b*N+n -> g[b])
    concat = np.concatenate([a2, gexp], axis=1)             # P:120, local first
    s1 = block(concat, "seg_conv1", "bn_seg1")              # P:123
    if train and masks is not None:
        k1 = masks[0].astype(dt) / (1.0 - p)
        k2 = masks[1].astype(dt) / (1.0 - p)
    else:
        k1 = k2 = None
    d1 = s1 * k1 if k1 is not None else s1                  # P:124
    s2 = block(d1, "seg_conv2", "bn_seg2")                  # P:125
    d2 = s2 * k2 if k2 is not None else s2                  # P:126
    s3 = block(d2, "seg_conv3", "bn_seg3")                  # P:127
    W4 = _w(sd, "seg_conv4", dt)
    logits = s3 @ W4.T + sd["seg_conv4.bias"].astype(dt)    # P:128
    cache["seg_conv4"] = {"in": s3}
    cache["drop"] = (k1, k2)
    return logits.reshape(B, N, -1), cache                  # P:131


def cross_entropy(logits, labels, weight, ignore_index=-1, denom=None):
    """nn.CrossEntropyLoss(weight=w, ignore_index=-1) mean reduction (P:216, P:251).

    loss = sum_{y!=-1} w[y] (logsumexp(z) - z[y]) / sum_{y!=-1} w[y]; returns (loss, dlogits).
    ``denom`` overrides the weight sum: under nn.DataParallel (P:208-211) the loss is taken
    once over the gathered outputs, so a replica's share uses the GLOBAL weight sum.
    """
    z = logits.reshape(-1, logits.shape[-1])
    y = labels.reshape(-1)
    valid = y != ignore_index
    ys = np.where(valid, y, 0)
    m = z.max(axis=1, keepdims=True)
    e = np.exp(z - m)
    se = e.sum(axis=1, keepdims=True)
    lse = (m + np.log(se))[:, 0]
    w = np.where(valid, np.asarray(weight, z.dtype)[ys], 0.0)
    nll = lse - z[np.arange(z.shape[0]), ys]
    if denom is None:
        denom = w.sum()
    loss = (w * nll).sum() / denom
    sm = e / se
    d = sm.copy()
    d[np.arange(z.shape[0]), ys] -= 1.0
    d *= (w / denom)[:, None]
    return loss, d.reshape(logits.shape)


# --------------------------------------------------------------------------------------
# backward (autograd of P:98-133, written out)
# --------------------------------------------------------------------------------------

def _bn_relu_bwd(da, c, st, gamma):
    """ReLU backward (grad where output>0) then BN train backward (biased var)."""
    dz = da * (c["z"] > 0)
    mean, var, rstd, xhat = st
    dgamma = (dz * xhat).sum(axis=0)
    dbeta = dz.sum(axis=0)
    dy = gamma * rstd * (dz - dz.mean(axis=0) - xhat * (dz * xhat).mean(axis=0))
    return dy, dgamma, dbeta


def backward(sd, cache, dlogits):
    """Gradients of every parameter (state-dict names) given dL/dlogits [B,N,C]."""
    dt = cache["x"].dtype
    B, N = cache["B"], cache["N"]
    grads = {}
    dL = dlogits.reshape(B * N, -1).astype(dt)

    def conv_bwd(conv, dy, need_dx=True):
        X = cache[conv]["in"]
        grads[f"{conv}.weight"] = (dy.T @ X)[:, :, None]
        grads[f"{conv}.bias"] = dy.sum(axis=0)
        return dy @ _w(sd, conv, dt) if need_dx else None

    def bn_bwd(conv, bn, da):
        g = sd[f"{bn}.weight"].astype(dt)
        dy, dg, db = _bn_relu_bwd(da, cache[conv], cache["bn"][bn], g)
        grads[f"{bn}.weight"] = dg
        grads[f"{bn}.bias"] = db
        return dy

    k1, k2 = cache["drop"]
    da_s3 = conv_bwd("seg_conv4", dL)
    dd2 = conv_bwd("seg_conv3", bn_bwd("seg_conv3", "bn_seg3", da_s3))
    da_s2 = dd2 * k2 if k2 is not None else dd2
    dd1 = conv_bwd("seg_conv2", bn_bwd("seg_conv2", "bn_seg2", da_s2))
    da_s1 = dd1 * k1 if k1 is not None else dd1
    dconcat = conv_bwd("seg_conv1", bn_bwd("seg_conv1", "bn_seg1", da_s1))
    da2_seg = dconcat[:, :64]
    dg = dconcat[:, 64:].reshape(B, N, -1).sum(axis=1)     # repeat backward: sum over N
    # max backward: scatter dg to the argmax rows (P:114)
    idx = cache["pool"]["idx"]
    dag = np.zeros((B, N, dg.shape[1]), dt)
    np.put_along_axis(dag, idx[:, None, :], dg[:, None, :], axis=1)
    da5 = conv_bwd("global_feat", bn_bwd("global_feat", "bn_global", dag.reshape(B * N, -1)))
    da4 = conv_bwd("conv5", bn_bwd("conv5", "bn5", da5))
    da3 = conv_bwd("conv4", bn_bwd("conv4", "bn4", da4))
    da2 = conv_bwd("conv3", bn_bwd("conv3", "bn3", da3)) + da2_seg
    da1 = conv_bwd("conv2", bn_bwd("conv2", "bn2", da2))
    conv_bwd("conv1", bn_bwd("conv1", "bn1", da1), need_dx=False)
    return grads


def update_running_stats(sd, cache, momentum=BN_MOMENTUM):
    """running = (1-m) running + m batch (unbiased var, n = B*N) ; num_batches_tracked += 1."""
    out = dict(sd)
    M = cache["B"] * cache["N"]
    for bn, (mean, var) in cache["bn_stats"].items():
        unb = var * M / max(M - 1, 1)
        out[f"{bn}.running_mean"] = ((1 - momentum) * sd[f"{bn}.running_mean"].astype(mean.dtype)
                                     + momentum * mean)
        out[f"{bn}.running_var"] = ((1 - momentum) * sd[f"{bn}.running_var"].astype(mean.dtype)
                                    + momentum * unb)
        out[f"{bn}.num_batches_tracked"] = np.array(int(sd[f"{bn}.num_batches_tracked"]) + 1,
                                                    np.int64)
    return out


# --------------------------------------------------------------------------------------
# optimizer (P:217-218, P:255, P:349)
# --------------------------------------------------------------------------------------

def adam_step(params, grads, state, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4):
    """torch.optim.Adam, L2 (coupled) weight decay, amsgrad=False (P:217, P:255).

    ``state[name] = {'step': t, 'exp_avg': m, 'exp_avg_sq': v}`` is updated in place;
    returns the new params dict.
    """
    b1, b2 = betas
    out = dict(params)
    for name, g in grads.items():
        p = params[name]
        st = state.setdefault(name, {"step": 0, "exp_avg": np.zeros_like(p, dtype=g.dtype),
                                     "exp_avg_sq": np.zeros_like(p, dtype=g.dtype)})
        st["step"] += 1
        t = st["step"]
        g = g.reshape(p.shape) + weight_decay * p
        st["exp_avg"] = b1 * st["exp_avg"] + (1 - b1) * g
        st["exp_avg_sq"] = b2 * st["exp_avg_sq"] + (1 - b2) * g * g
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = np.sqrt(st["exp_avg_sq"]) / np.sqrt(bc2) + eps
        out[name] = p - (lr / bc1) * st["exp_avg"] / denom
    return out


def step_lr(lr0, epoch, step_size=20, gamma=0.5):
    """StepLR(step_size=20, gamma=0.5) learning rate for a 0-based epoch (P:218, P:349)."""
    return lr0 * gamma ** (epoch // step_size)


# --------------------------------------------------------------------------------------
# metrics (P:261-266, P:341-346; mIoU is build-defined)
# --------------------------------------------------------------------------------------

def confusion(pred, labels, num_classes):
    valid = labels.reshape(-1) >= 0
    p = pred.reshape(-1)[valid]
    t = labels.reshape(-1)[valid]
    cm = np.zeros((num_classes, num_classes), np.int64)
    np.add.at(cm, (t, p), 1)
    return cm


def miou(cm):
    tp = np.diag(cm).astype(np.float64)
    denom = cm.sum(0) + cm.sum(1) - tp
    present = denom > 0
    return float((tp[present] / denom[present]).mean()) if present.any() else 0.0


def ce_weight_sum(labels, weight, ignore_index=-1):
    """sum_{y != ignore} w[y]: the CE denominator of P:216 for one shard."""
    y = np.asarray(labels).reshape(-1)
    y = y[y != ignore_index]
    return float(np.asarray(weight, np.float64)[y].sum())


def train_step(sd, x, labels, weight, masks=None, dtype=np.float64, denom=None):
    """One reference training step (P:241-255) without the optimizer: loss, grads, cache.

    With ``denom`` (the global CE weight sum) this is one DataParallel replica's share:
    its loss numerator / denom and the gradient of that, computed with the replica's own
    BatchNorm batch statistics (P:208-211; nn.DataParallel has no SyncBN).
    """
    logits, cache = forward(sd, x, train=True, masks=masks, dtype=dtype)
    loss, dl = cross_entropy(logits, labels, weight, denom=denom)
    grads = backward(sd, cache, dl)
    return loss, logits, grads, cache

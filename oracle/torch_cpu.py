"""CPU baseline: pure-PyTorch (ATen, fp32) restatement of the reference training step.

TEST / BASELINE INFRASTRUCTURE ONLY.  Only ``tests/`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module -- as the checker, or as the timed CPU baseline that
SURVEY.md §8(d) asks for ("the build's own pure-PyTorch CPU restatement ... fp32, train mode,
dropout on, timed on the GPU box's host cores").  The product path (``pcs_amd``) never
calls it.

It runs the same ATen CPU kernels the reference's ``PointNetSegmentation`` runs
(``/root/reference/point_cloud_segmentation.py``, cited ``P:<line>``), written as a
function over a state dict instead of a module:
  - 1x1 ``Conv1d`` on channels-first ``(B, C, N)`` (P:70-83, P:103-128) -> ``F.conv1d``;
  - ``BatchNorm1d`` in train mode, batch statistics over (B, N), pads included
    (P:86-94) -> ``F.batch_norm(training=True)`` (running buffers updated in place);
  - the global max over N with ``keepdim`` (P:114), ``repeat`` + ``cat`` (P:117-120);
  - ``Dropout(0.3)`` applied twice with independent draws (P:96, P:124, P:126), or replayed
    keep masks (parity tests);
  - ``CrossEntropyLoss(weight=w, ignore_index=-1)`` on the ``.contiguous().view(-1, C)``
    output (P:216, P:247-251), autograd backward (P:254).

Parity: ``tests/test_torch_cpu_baseline.py`` checks it against the goldens that
``tests/golden/make_golden.py`` recorded from the imported reference.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

DROPOUT_P = 0.3
BN_EPS = 1e-5
BN_MOMENTUM = 0.1

_CONV_BN = [("conv1", "bn1"), ("conv2", "bn2"), ("conv3", "bn3"), ("conv4", "bn4"),
            ("conv5", "bn5"), ("global_feat", "bn_global"), ("seg_conv1", "bn_seg1"),
            ("seg_conv2", "bn_seg2"), ("seg_conv3", "bn_seg3")]


def to_tensors(sd, requires_grad=True):
    """numpy state dict -> fp32 CPU tensors; conv / BN affine parameters require grad."""
    out = {}
    for k, v in sd.items():
        t = torch.from_numpy(np.array(v))
        if t.is_floating_point():
            t = t.float()
            if requires_grad and not ("running_" in k):
                t.requires_grad_(True)
        out[k] = t
    return out


def forward(T, x, train=True, masks=None, p=DROPOUT_P):
    """logits [B, N, C] for x [B, N, D] (P:98-133).  ``masks`` = (keep1 [B*N, 512],
    keep2 [B*N, 256]) replays the dropout draws; otherwise train mode draws them (ATen
    bernoulli, as the reference does)."""
    B, N, _ = x.shape

    def cbr(h, conv, bn):
        h = F.conv1d(h, T[f"{conv}.weight"], T[f"{conv}.bias"])
        h = F.batch_norm(h, T[f"{bn}.running_mean"], T[f"{bn}.running_var"], T[f"{bn}.weight"],
                         T[f"{bn}.bias"], training=train, momentum=BN_MOMENTUM, eps=BN_EPS)
        return F.relu(h)

    def drop(h, which):
        if not train:
            return h
        if masks is None:
            return F.dropout(h, p, training=True)
        keep = torch.from_numpy(np.ascontiguousarray(masks[which])).float()   # [B*N, C]
        keep = keep.reshape(B, N, -1).transpose(1, 2)
        return h * keep / (1.0 - p)

    h = x.transpose(1, 2)                                   # P:103
    h = cbr(h, "conv1", "bn1")                              # P:106
    point_feat = cbr(h, "conv2", "bn2")                     # P:107
    h = cbr(point_feat, "conv3", "bn3")
    h = cbr(h, "conv4", "bn4")
    h = cbr(h, "conv5", "bn5")                              # P:110
    h = cbr(h, "global_feat", "bn_global")                  # P:113
    g = torch.max(h, 2, keepdim=True)[0]                    # P:114
    h = torch.cat([point_feat, g.repeat(1, 1, N)], 1)       # P:117-120
    h = drop(cbr(h, "seg_conv1", "bn_seg1"), 0)             # P:123-124
    h = drop(cbr(h, "seg_conv2", "bn_seg2"), 1)             # P:125-126
    h = cbr(h, "seg_conv3", "bn_seg3")                      # P:127
    h = F.conv1d(h, T["seg_conv4.weight"], T["seg_conv4.bias"])   # P:128
    return h.transpose(1, 2)                                # P:131


def train_step(T, x, labels, weight, masks=None):
    """Forward + weighted CE (ignore -1) + backward (P:241-254; no optimizer step).
    Returns (loss, logits); gradients land in ``T[name].grad``."""
    for v in T.values():
        if v.grad is not None:
            v.grad = None
    out = forward(T, x, train=True, masks=masks)
    C = out.shape[-1]
    loss = F.cross_entropy(out.contiguous().view(-1, C), labels.view(-1), weight=weight,
                           ignore_index=-1)
    loss.backward()
    return loss, out

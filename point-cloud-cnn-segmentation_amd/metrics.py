"""Training / validation metrics on device (reference P:258-271, P:314-346).

The reference computes accuracy per step with host syncs (P:261-266) and F1 with sklearn
over host arrays (P:343).  Here a device confusion matrix (``pcs_confusion``) accumulates for
a whole epoch and the metrics come from that C x C matrix with one host read:

* accuracy = trace / total over non-padded points (P:263-266);
* ``f1_per_class`` follows ``sklearn.metrics.f1_score(y_true, y_pred, average=None)``: one
  entry per label present in y_true or y_pred, in sorted label order, 0 when undefined;
* ``f1_class2`` reproduces P:345-346 (positional index 2 of that list, 0.0 if absent);
* mIoU = mean over classes with any true or predicted point of TP / (TP + FP + FN).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


class ConfusionMeter:
    """Device-side confusion matrix; ``update`` enqueues one kernel and never syncs."""

    def __init__(self, num_classes: int, device=None):
        self.C = int(num_classes)
        self.cm = torch.zeros(self.C, self.C, dtype=torch.int64, device=device or "cuda")

    def reset(self):
        self.cm.zero_()

    def update(self, logits: torch.Tensor, labels: torch.Tensor):
        """logits [..., C] fp32 (HIP device), labels [...] int (-1 = padding)."""
        if not logits.is_cuda:
            raise RuntimeError("ConfusionMeter runs on a HIP device only")
        z = logits.reshape(-1, self.C)
        if z.dtype != torch.float32 or z.stride(1) != 1:
            z = z.float().contiguous()
        y = labels.reshape(-1)
        if y.dtype != torch.int64 or not y.is_contiguous():
            y = y.long().contiguous()
        if y.numel() != z.shape[0]:
            raise ValueError(f"{y.numel()} labels for {z.shape[0]} logit rows")
        L.call("pcs_confusion", L.ptr(z), z.stride(0), L.ptr(y), y.numel(), self.C, L.ptr(self.cm),
               L.stream_ptr())
        return self

    def compute(self) -> dict:
        return metrics_from_confusion(self.cm.cpu().numpy())


def accuracy(cm: np.ndarray) -> float:
    tot = cm.sum()
    return float(np.trace(cm) / tot) if tot else 0.0


def f1_per_class(cm: np.ndarray) -> np.ndarray:
    tp = np.diag(cm).astype(np.float64)
    fp = cm.sum(0) - tp
    fn = cm.sum(1) - tp
    present = (cm.sum(0) + cm.sum(1)) > 0          # labels in y_true U y_pred (sklearn)
    denom = 2 * tp + fp + fn
    f1 = np.divide(2 * tp, denom, out=np.zeros_like(tp), where=denom > 0)
    return f1[present]


def f1_class2(cm: np.ndarray) -> float:
    f1 = f1_per_class(cm)
    return float(f1[2]) if len(f1) > 2 else 0.0     # P:346


def miou(cm: np.ndarray) -> float:
    tp = np.diag(cm).astype(np.float64)
    denom = cm.sum(0) + cm.sum(1) - tp
    present = denom > 0
    return float((tp[present] / denom[present]).mean()) if present.any() else 0.0


def metrics_from_confusion(cm) -> dict:
    cm = np.asarray(cm, dtype=np.int64)
    return {"accuracy": accuracy(cm), "f1_per_class": f1_per_class(cm).tolist(),
            "f1_class2": f1_class2(cm), "miou": miou(cm), "points": int(cm.sum()),
            "confusion": cm.tolist()}

"""Checkpoint I/O and inference compatible with the reference.

* ``save_checkpoint`` writes the ``best_model.pth`` dictionary of P:373-382 (keys epoch,
  model_state_dict, optimizer_state_dict, train_loss, val_loss, f1_class2, f1_per_class,
  num_classes); ``data_parallel=True`` adds the ``module.`` prefix that an
  ``nn.DataParallel``-wrapped reference model would have saved.
* ``load_checkpoint`` reads such a file with ``torch.load(weights_only=True)`` (never
  unpickling code), strips a ``module.`` prefix like P:409-428, and returns a model (and
  optionally restores a FusedAdam).
* ``predict`` is the single-event inference of P:440-452: eval mode, forward, argmax over
  classes (``pcs_argmax``).
"""
from __future__ import annotations

import torch

from . import _lib as L
from .model import PointNetSegmentation, load_reference_checkpoint

CHECKPOINT_KEYS = ("epoch", "model_state_dict", "optimizer_state_dict", "train_loss", "val_loss",
                   "f1_class2", "f1_per_class", "num_classes")


def save_checkpoint(path, model, optimizer=None, *, epoch=0, train_loss=float("nan"),
                    val_loss=float("nan"), f1_class2=0.0, f1_per_class=(), data_parallel=False):
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    if data_parallel:
        sd = {f"module.{k}": v for k, v in sd.items()}
    osd = optimizer.state_dict() if optimizer is not None else {}
    osd = _to_cpu(osd)
    ckpt = {"epoch": int(epoch), "model_state_dict": sd, "optimizer_state_dict": osd,
            "train_loss": float(train_loss), "val_loss": float(val_loss), "f1_class2": float(f1_class2),
            "f1_per_class": [float(f) for f in f1_per_class], "num_classes": int(model.num_classes)}
    torch.save(ckpt, path)
    return ckpt


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def load_checkpoint(path, device="cuda", compute_dtype="fp32", optimizer=None):
    """-> (model on ``device`` in eval mode, checkpoint dict)."""
    sd, ckpt = load_reference_checkpoint(path)
    num_classes = int(ckpt.get("num_classes", sd["seg_conv4.weight"].shape[0]))
    input_dim = int(sd["conv1.weight"].shape[1])
    model = PointNetSegmentation(num_classes, input_dim, compute_dtype=compute_dtype)
    model.load_state_dict(sd)
    model = model.to(device).eval()
    if optimizer is not None and ckpt.get("optimizer_state_dict"):
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    return model, ckpt


@torch.no_grad()
def predict(model, points):
    """points [B, N, 4] (HIP device) -> int64 class predictions [B, N] (P:448-452)."""
    was_training = model.training
    model.eval()
    logits = model(points)
    if was_training:
        model.train()
    B, N, C = logits.shape
    out = torch.empty(B, N, dtype=torch.int64, device=logits.device)
    z = logits.reshape(B * N, C)
    L.call("pcs_argmax", L.ptr(z), z.stride(0), B * N, C, L.ptr(out), L.stream_ptr())
    return out

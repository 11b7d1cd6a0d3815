"""Fused Adam (L2 weight decay) over one flat fp32 parameter buffer.

Semantics of ``torch.optim.Adam(params, lr=1e-3, weight_decay=1e-4)`` as the reference
uses it (P:217, P:255): coupled weight decay (g += wd*p), betas (0.9, 0.999), eps 1e-8,
amsgrad off, bias-corrected step.  One HIP kernel (pcs_adam) updates every parameter;
``torch.optim.lr_scheduler.StepLR(opt, 20, 0.5)`` (P:218) works unchanged because this
is a regular ``torch.optim.Optimizer`` with ``param_groups``.
"""
from __future__ import annotations

import torch

from . import _lib as L


def flatten_parameters(module: torch.nn.Module):
    """Re-home every parameter of ``module`` as a view into one contiguous fp32 buffer
    (and give each a gradient view into one flat grad buffer).  Returns (pflat, gflat)."""
    params = list(module.parameters())
    dev = params[0].device
    n = sum(p.numel() for p in params)
    pflat = torch.empty(n, dtype=torch.float32, device=dev)
    gflat = torch.zeros(n, dtype=torch.float32, device=dev)
    off = 0
    for p in params:
        k = p.numel()
        pflat[off:off + k].copy_(p.data.reshape(-1))
        p.data = pflat[off:off + k].view_as(p)
        p.grad = gflat[off:off + k].view_as(p)
        off += k
    module._pcs_flat = (pflat, gflat)
    return pflat, gflat


def flat_buffers(module):
    """The (pflat, gflat) of a flattened module; re-flattens if the views were broken
    (e.g. by ``.to()`` or ``zero_grad(set_to_none=True)``)."""
    flat = getattr(module, "_pcs_flat", None)
    if flat is not None:
        pflat, gflat = flat
        off = 0
        ok = True
        for p in module.parameters():
            k = p.numel()
            if (p.data_ptr() != pflat[off:].data_ptr() or p.grad is None
                    or p.grad.data_ptr() != gflat[off:].data_ptr()):
                ok = False
                break
            off += k
        if ok:
            return pflat, gflat
    return flatten_parameters(module)


class FusedAdam(torch.optim.Optimizer):
    """Adam with L2 weight decay as one kernel over the flat buffers of ``module``."""

    def __init__(self, module: torch.nn.Module, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=1e-4):
        self.module = module
        pflat, gflat = flat_buffers(module)
        super().__init__(list(module.parameters()),
                         dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                              amsgrad=False, maximize=False, foreach=None, capturable=False,
                              differentiable=False, fused=None,
                              decoupled_weight_decay=False))
        self.exp_avg = torch.zeros_like(pflat)
        self.exp_avg_sq = torch.zeros_like(pflat)
        self.step_count = 0
        self.grad_scale = None   # optional device scalar multiplying every gradient

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        pflat, gflat = flat_buffers(self.module)
        self.step_count += 1
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        L.call("pcs_adam", L.ptr(pflat), L.ptr(gflat), L.ptr(self.exp_avg), L.ptr(self.exp_avg_sq),
               pflat.numel(), L.ptr(self.grad_scale), float(grp["lr"]), float(b1), float(b2),
               float(grp["eps"]), float(grp["weight_decay"]), self.step_count, L.stream_ptr())
        return loss

    def zero_grad(self, set_to_none: bool = False):
        # gradients are overwritten by every fused step; keep the flat views alive
        _, gflat = flat_buffers(self.module)
        gflat.zero_()

    def state_dict(self):
        """torch.optim.Adam-compatible layout (per-parameter step/exp_avg/exp_avg_sq)."""
        state = {}
        off = 0
        for i, p in enumerate(self.module.parameters()):
            k = p.numel()
            state[i] = {"step": torch.tensor(float(self.step_count)),
                        "exp_avg": self.exp_avg[off:off + k].view_as(p).clone(),
                        "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p).clone()}
            off += k
        groups = [dict(g, params=list(range(len(g["params"])))) for g in self.param_groups]
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        off = 0
        for i, p in enumerate(self.module.parameters()):
            k = p.numel()
            st = sd["state"].get(i) or sd["state"].get(str(i))
            if st is not None:
                self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                self.step_count = int(float(st["step"]))
            off += k
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for key in ("lr", "betas", "eps", "weight_decay"):
                if key in sg:
                    g[key] = sg[key]

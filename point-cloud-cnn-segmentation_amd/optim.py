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


def param_slices(module: torch.nn.Module):
    """[(param, offset, numel)] in registration order.  Offsets follow the module's flat
    layout when it defines one (PointNetSegmentation: gradient-bucket order, engine.flat_layout)
    and registration order otherwise."""
    named = list(module.named_parameters())
    offs = module._flat_offsets() if hasattr(module, "_flat_offsets") else None
    out, off = [], 0
    for name, p in named:
        k = p.numel()
        out.append((p, offs[name] if offs is not None else off, k))
        off += k
    return out


def flatten_parameters(module: torch.nn.Module):
    """Re-home every parameter of ``module`` as a view into one contiguous fp32 buffer
    (and give each a gradient view into one flat grad buffer, which carries the module's
    ``_flat_extra`` scalars after the parameters).  Returns (pflat, gflat)."""
    sl = param_slices(module)
    dev = sl[0][0].device
    n = sum(k for _, _, k in sl)
    pflat = torch.empty(n, dtype=torch.float32, device=dev)
    gflat = torch.zeros(n + getattr(module, "_flat_extra", 0), dtype=torch.float32, device=dev)
    for p, off, k in sl:
        pflat[off:off + k].copy_(p.data.reshape(-1))
        p.data = pflat[off:off + k].view_as(p)
        p.grad = gflat[off:off + k].view_as(p)
    module._pcs_flat = (pflat, gflat)
    return pflat, gflat


def flat_buffers(module):
    """The (pflat, gflat) of a flattened module; re-flattens if the views were broken
    (e.g. by ``.to()`` or ``zero_grad(set_to_none=True)``)."""
    flat = getattr(module, "_pcs_flat", None)
    if flat is not None:
        pflat, gflat = flat
        ok = True
        for p, off, k in param_slices(module):
            if (p.data_ptr() != pflat[off:].data_ptr() or p.grad is None
                    or p.grad.data_ptr() != gflat[off:].data_ptr()):
                ok = False
                break
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
        # optional device scalar multiplying every gradient; the kernel writes the scaled
        # gradient back, so p.grad holds it after the step (data-parallel normalisation)
        self.grad_scale = None

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
        for i, (p, off, k) in enumerate(param_slices(self.module)):
            state[i] = {"step": torch.tensor(float(self.step_count)),
                        "exp_avg": self.exp_avg[off:off + k].view_as(p).clone(),
                        "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p).clone()}
        groups = [dict(g, params=list(range(len(g["params"])))) for g in self.param_groups]
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        for i, (p, off, k) in enumerate(param_slices(self.module)):
            st = sd["state"].get(i) or sd["state"].get(str(i))
            if st is not None:
                self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                self.step_count = int(float(st["step"]))
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for key in ("lr", "betas", "eps", "weight_decay"):
                if key in sg:
                    g[key] = sg[key]

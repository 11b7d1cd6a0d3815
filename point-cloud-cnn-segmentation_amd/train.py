"""Fused training step: the reference inner loop P:241-255 as one stream of HIP kernels.

    optimizer.zero_grad(); out = model(points); loss = criterion(out.view(-1,C), labels)
    loss.backward(); optimizer.step()

becomes ``loss = step(points, labels)``: forward, weighted CE (P:216, P:251) fused into the
head kernel, backward into one flat gradient buffer, the data-parallel all-reduce, and the
fused Adam update.  Nothing synchronises with the host; ``loss`` is a device scalar (read it
once per epoch, not per step as P:258-269 does).

Data parallelism (replaces nn.DataParallel, P:208-211) is one process per GPU, each rank
running its own scenes with its own BatchNorm statistics (DataParallel has no SyncBN).
DataParallel takes ONE loss over the gathered outputs (P:251), i.e. every replica's share
is divided by the GLOBAL CE weight sum.  Here each rank's head computes the un-normalised
gradient (the loss is linear in 1/sum_w), the local loss numerator and weight sum ride in
the gradient buffer's tail, and the buffer is summed by RCCL in three buckets
(engine.bucket_ranges), each issued the moment the backward has enqueued its last writer,
so the collectives overlap the rest of the backward (§8 e).  Adam then scales the summed
gradient by 1 / global sum_w (and writes the scaled gradient back into p.grad).  One
collective pass per step, no blocking denominator exchange before the forward.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib as L
from .engine import BNS
from .optim import FusedAdam, flat_buffers


def _all_reduce(t, group=None, async_op=False):
    """SUM all-reduce in place.  RCCL ("nccl") reduces device tensors directly, enqueued
    behind the work already on the current stream; a gloo group (CPU rendezvous, e.g. several
    ranks sharing one device in tests) is staged through host memory synchronously."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
        return None
    return dist.all_reduce(t, group=group, async_op=async_op)


class GradientBuckets:
    """Bucketed all-reduce of a flat gradient buffer: ``issue(name)`` starts the collective
    of one [lo, hi) range as soon as its gradients are enqueued; ``wait()`` makes the current
    stream wait for all of them (before the optimizer reads the buffer)."""

    def __init__(self, flat, ranges, group=None):
        self.flat, self.ranges, self.group = flat, ranges, group
        self.works = []
        self.issued = []

    def issue(self, name):
        lo, hi = self.ranges[name]
        w = _all_reduce(self.flat[lo:hi], self.group, async_op=True)
        self.issued.append(name)
        if w is not None:
            self.works.append(w)

    def wait(self):
        if sorted(self.issued) != sorted(self.ranges):
            raise RuntimeError(f"gradient buckets issued {self.issued}, expected {sorted(self.ranges)}")
        for w in self.works:
            w.wait()
        self.works = []


class FusedTrainStep:
    def __init__(self, model, optimizer: FusedAdam | None = None, class_weight=None,
                 process_group=None, lr=1e-3, weight_decay=1e-4):
        """``process_group``: data-parallel group; None = the default group when one is
        initialised with more than one rank.  An explicit group always takes the collective
        path (also at world size 1)."""
        self.model = model
        self.opt = optimizer or FusedAdam(model, lr=lr, weight_decay=weight_decay)
        dev = next(model.parameters()).device
        C = model.num_classes
        w = torch.ones(C) if class_weight is None else torch.as_tensor(class_weight, dtype=torch.float32)
        self.class_weight = w.to(dev, torch.float32).contiguous()
        self.pg = process_group
        self.wsum = torch.empty(3, dtype=torch.float32, device=dev)
        self.counts = torch.empty(max(16, C), dtype=torch.int64, device=dev)
        self.inv_wsum = torch.empty(1, dtype=torch.float32, device=dev)
        self.timing = None   # optional dict tag -> list of (start, end) events
        self.timing_tags = None   # optional set: only these tags are bracketed (None = all)

    def _distributed(self):
        if not (dist.is_available() and dist.is_initialized()):
            return False
        return self.pg is not None or dist.get_world_size() > 1

    def __call__(self, points, labels, masks=None, seed=None):
        model = self.model
        eng = model._engine()
        eng.timing = self.timing
        eng.timing_tags = self.timing_tags
        model.train()
        P = model._param_dict()
        bufs = model._buffer_dict()
        pflat, gflat = flat_buffers(model)
        ext = gflat[eng.total_params:]   # [loss numerator, CE weight sum, valid count, pad]
        labels = labels.reshape(-1)
        if labels.dtype != torch.int64:
            labels = labels.long()
        s = L.stream_ptr()
        L.call("pcs_ce_weight_sum", L.ptr(labels), labels.numel(), L.ptr(self.class_weight),
               model.num_classes, L.ptr(self.counts), L.ptr(self.wsum), s)
        ddp = self._distributed()
        if seed is None:
            seed = model._next_seed()
        # single process: the head normalises by the local weight sum; data-parallel: the
        # gradient stays un-normalised until the global sum is known (after the all-reduce)
        sv = eng.forward(P, bufs, points, train=True, masks=masks, seed=seed,
                         head_mode=L.HEAD_CE, labels=labels, class_weight=self.class_weight,
                         wsum=None if ddp else self.wsum, want_logits=False)
        for bn, _ in BNS:
            getattr(model, bn).num_batches_tracked.add_(1)
        hb = sv.head
        L.call("pcs_reduce_partials", L.ptr(hb["loss_partial"]), hb["nch"], 1, 1.0, L.ptr(ext), 1, 1, s)
        if ddp:
            ext[1:3].copy_(self.wsum[:2])
            buckets = GradientBuckets(gflat, eng.buckets, self.pg)
            eng.backward(P, sv, gflat, on_bucket=buckets.issue)
            buckets.wait()
            torch.reciprocal(ext[1:2], out=self.inv_wsum)
            self.opt.grad_scale = self.inv_wsum
            loss = ext[0] / ext[1]
        else:
            eng.backward(P, sv, gflat)
            self.opt.grad_scale = None
            loss = ext[0] / self.wsum[0]
        del sv, hb
        self.opt.step()
        return loss

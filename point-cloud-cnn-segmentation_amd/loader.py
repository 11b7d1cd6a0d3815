"""Device side of the data path: CSR batches -> the padded batch the model
consumes, built on the GPU.

The reference pads on the host in ``collate_fn`` (P:44-63) and copies the padded
[B, N, 4] / [B, N] tensors to the device every step (P:242-243).  Here the DataLoader
yields a ``RaggedBatch`` (CSR, no padding, pinned by ``pin_memory=True``), the flat
arrays are copied host->device asynchronously on a side stream, and ``pcs_pad_scatter``
writes the padded points / labels / masks in HBM -- byte-identical to collate_fn's output.
``DevicePrefetcher`` runs batch i+1's copy and scatter while batch i trains.

Data parallelism: the reference pads the GLOBAL batch to its max length before
DataParallel scatters it (P:50), so pads -- which enter every BatchNorm's
statistics and the max-pool -- are counted against the global max.  ``global_max_points``
all-reduces (MAX) the local max over the process group so each rank pads identically.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib as L
from .data import RaggedBatch


def global_max_points(n_local: int, group=None, device=None) -> int:
    """MAX of the per-rank padded lengths (DataParallel pads the whole batch, P:50)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return n_local
    if dist.get_backend(group) == "gloo":
        t = torch.tensor([n_local], dtype=torch.int64)
    else:
        t = torch.tensor([n_local], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def pad_on_device(rb: RaggedBatch, device=None, scene_rows: int | None = None, stream=None):
    """(points f32 [B,N,4], labels i64 [B,N], masks bool [B,N]) on ``device`` from a CSR
    batch, equal byte for byte to collate_fn (P:44-63): pads are (0,0,0,0) / -1 / False.

    ``rb`` may live on the host (copied with non_blocking, so pin it for an async copy) or
    already on the device.  ``scene_rows`` defaults to the batch max (collate_fn's N); a
    larger value pads further (the DP global max)."""
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if device.type != "cuda":
        raise RuntimeError("pad_on_device runs on a HIP device only (no CPU fallback)")
    B = rb.num_scenes
    n_max = rb.max_points
    N = n_max if scene_rows is None else int(scene_rows)
    if N < n_max:
        raise ValueError(f"scene_rows={N} is shorter than the longest scene ({n_max})")
    lab = rb.labels
    if lab.dtype not in (torch.int32, torch.int64):
        lab = lab.long()
    if rb.points.ndim != 2 or rb.points.shape[1] != 4 or lab.numel() != rb.points.shape[0] \
            or int(rb.offsets[-1]) != rb.points.shape[0]:
        raise ValueError("inconsistent RaggedBatch (points [T,4], labels [T], offsets[-1] == T)")
    with torch.cuda.device(device), torch.cuda.stream(stream or torch.cuda.current_stream(device)):
        pts_d = rb.points.to(device, torch.float32, non_blocking=True).contiguous()
        lab_d = lab.to(device, non_blocking=True).contiguous()
        off_d = rb.offsets.to(device, torch.int64, non_blocking=True).contiguous()
        points = torch.empty(B, N, 4, dtype=torch.float32, device=device)
        labels = torch.empty(B, N, dtype=torch.int64, device=device)
        masks = torch.empty(B, N, dtype=torch.bool, device=device)
        L.call("pcs_pad_scatter", L.ptr(pts_d), L.ptr(lab_d), lab_d.element_size(), L.ptr(off_d), B, N,
               L.ptr(points), L.ptr(labels), L.ptr(masks), L.stream_ptr(device))
    return points, labels, masks


class DevicePrefetcher:
    """Iterate a DataLoader of RaggedBatch (``collate_fn=ragged_collate``, ideally
    ``pin_memory=True``) and yield padded device batches, staging batch i+1 (H2D copy +
    pcs_pad_scatter) on a side stream while the caller computes on batch i.

    With a process group, each rank pads to the global max length (``global_max_points``)
    so the model sees exactly the padding DataParallel would have produced."""

    def __init__(self, loader, device=None, process_group=None):
        self.loader = loader
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.pg = process_group
        self.stream = torch.cuda.Stream(self.device)

    def _stage(self, rb):
        n = global_max_points(rb.max_points, self.pg, self.device)
        batch = pad_on_device(rb, self.device, scene_rows=n, stream=self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return batch, ev

    def __iter__(self):
        it = iter(self.loader)
        nxt = None
        try:
            nxt = self._stage(next(it))
        except StopIteration:
            return
        while nxt is not None:
            batch, ev = nxt
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for t in batch:   # allocated on the side stream, consumed on the compute stream
                t.record_stream(cur)
            try:
                nxt = self._stage(next(it))
            except StopIteration:
                nxt = None
            yield batch

    def __len__(self):
        return len(self.loader)

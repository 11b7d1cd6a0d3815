"""Point -> voxel path on the device (north-star voxel vocabulary).

The reference segments raw points (P:98-133); it has no voxel grid.  This module adds the
north star's "point->voxel scatter" and "hash-indexed gather" around the unchanged model:

    vb = voxelize(rb, grid=256, lo=(-1,-1,-1), hi=(1,1,1), num_classes=C)   # pcs_voxelize
    points, labels, masks = pad_on_device(vb.batch)                         # voxel batch
    logits = model(points)                                                   # [B, Nv, C]
    point_logits = to_points(logits, vb)                                     # pcs_gather_rows

A voxel is one occupied cell of a G^3 lattice per scene: (mean x, mean y, mean z, summed e)
of its points, the most frequent label, and its point count.  Integer outputs (voxel ids,
voxel order, inverse map, counts, labels) are bit-exact with oracle/voxel_oracle.py; its
semantics are build-defined ("not reference parity").
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib as L
from .data import RaggedBatch


@dataclass
class VoxelBatch:
    batch: RaggedBatch            # voxels as a CSR batch: points [V,4], labels [V], offsets [B+1]
    counts: torch.Tensor          # int64 [V] points per voxel
    voxel_of_point: torch.Tensor  # int64 [T] global voxel index of every input point
    grid: int


def _box(lo, hi):
    lo = [float(v) for v in lo]
    hi = [float(v) for v in hi]
    if len(lo) != 3 or len(hi) != 3 or any(h <= l for l, h in zip(lo, hi)):
        raise ValueError("lo / hi must be 3 bounds with hi > lo")
    return lo + hi


def voxel_ids(points: torch.Tensor, grid: int, lo=(-1.0, -1.0, -1.0), hi=(1.0, 1.0, 1.0)):
    """int64 voxel id of each point (points: fp32 [T, 4] on the device)."""
    if not points.is_cuda:
        raise RuntimeError("voxel_ids runs on a HIP device only (no CPU fallback)")
    pts = points.contiguous().float()
    out = torch.empty(pts.shape[0], dtype=torch.int64, device=pts.device)
    L.call("pcs_voxel_ids", L.ptr(pts), pts.shape[0], int(grid), *_box(lo, hi), L.ptr(out), L.stream_ptr())
    return out


def voxelize(rb: RaggedBatch, grid: int, lo=(-1.0, -1.0, -1.0), hi=(1.0, 1.0, 1.0), num_classes: int = 2,
             device=None) -> VoxelBatch:
    """Occupied-voxel scatter of a CSR batch (pcs_voxelize).  One host read (the voxel count)
    sizes the outputs."""
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if device.type != "cuda":
        raise RuntimeError("voxelize runs on a HIP device only (no CPU fallback)")
    pts = rb.points.to(device, torch.float32).contiguous()
    lab = rb.labels.to(device, torch.int64).contiguous() if rb.labels is not None else None
    off = rb.offsets.to(device, torch.int64).contiguous()
    B, T = off.numel() - 1, pts.shape[0]
    if T == 0:
        raise ValueError("voxelize needs at least one point")
    ws = torch.empty(int(L.load().pcs_voxelize_workspace(T)), dtype=torch.uint8, device=device)
    vop = torch.empty(T, dtype=torch.int64, device=device)
    vpts = torch.empty(T, 4, dtype=torch.float32, device=device)
    vlab = torch.empty(T, dtype=torch.int64, device=device)
    vcnt = torch.empty(T, dtype=torch.int64, device=device)
    voff = torch.empty(B + 1, dtype=torch.int64, device=device)
    nv = torch.empty(1, dtype=torch.int64, device=device)
    L.call("pcs_voxelize", L.ptr(pts), L.ptr(lab), L.ptr(off), B, T, int(grid), *_box(lo, hi), int(num_classes),
           L.ptr(ws), ws.numel(), L.ptr(vop), L.ptr(vpts), L.ptr(vlab), L.ptr(vcnt), L.ptr(voff), L.ptr(nv),
           L.stream_ptr(device))
    V = int(nv.item())
    return VoxelBatch(RaggedBatch(vpts[:V], vlab[:V], voff), vcnt[:V], vop, int(grid))


def to_points(voxel_logits: torch.Tensor, vb: VoxelBatch) -> torch.Tensor:
    """Per-point outputs [T, C] from per-voxel outputs: padded [B, Nv, C] (the model's output
    on pad_on_device(vb.batch)) or flat [V, C] (pcs_voxel_padded_index + pcs_gather_rows)."""
    out_dev = voxel_logits.device
    x = voxel_logits.contiguous().float()
    T = vb.voxel_of_point.numel()
    C = x.shape[-1]
    if x.dim() == 3:
        B, Nv = x.shape[0], x.shape[1]
        idx = torch.empty(T, dtype=torch.int64, device=out_dev)
        L.call("pcs_voxel_padded_index", L.ptr(vb.voxel_of_point), T, L.ptr(vb.batch.offsets), B, Nv, L.ptr(idx),
               L.stream_ptr(out_dev))
        src = x.view(B * Nv, C)
    else:
        idx, src = vb.voxel_of_point, x
    out = torch.empty(T, C, dtype=torch.float32, device=out_dev)
    L.call("pcs_gather_rows", L.ptr(src), src.stride(0), L.ptr(idx), T, C, L.ptr(out), L.stream_ptr(out_dev))
    return out

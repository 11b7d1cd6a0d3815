"""Host-side data path: reference-compatible collate, class weights, synthetic clouds.

Pure numpy/torch host code (no HIP).  Mirrors the reference's data contract:

* ``collate_fn`` — P:44-63: pad a ragged batch to the batch max; pads are (0,0,0,0)
  points, label -1, mask False, and the model sees them.
* ``class_weights`` — P:146-183: inverse-frequency weights, class 2 doubled, normalised
  so the weights sum to ``num_classes``.
* ``synthetic_batch`` — the seeded synthetic clouds of SURVEY.md §8(d) (the reference's
  HDF5 data is not available): voxel-centre xyz on a G^3 lattice, energy e, labels from
  a random sphere and a random line "track".
* ``shard_batch`` — the ``tensor.chunk`` rule nn.DataParallel uses to split a padded
  batch over ranks (torch/nn/parallel/scatter_gather.py).
"""
from __future__ import annotations

from collections import Counter

import numpy as np


def collate_fn(batch):
    """Reference collate (P:44-63) on a list of (points[N_i,4], labels[N_i]) torch tensors."""
    import torch
    points_list, labels_list = zip(*batch)
    B = len(points_list)
    N = max(p.shape[0] for p in points_list)
    pts = torch.zeros(B, N, 4)
    lab = torch.full((B, N), -1, dtype=torch.long)
    msk = torch.zeros(B, N, dtype=torch.bool)
    for i, (p, l) in enumerate(zip(points_list, labels_list)):
        n = p.shape[0]
        pts[i, :n] = p
        lab[i, :n] = l
        msk[i, :n] = True
    return pts, lab, msk


def class_weights(labels_iterable, num_classes=None):
    """Inverse-frequency class weights exactly as P:148-183 computes them.

    ``labels_iterable`` yields per-event label arrays (the reference scans the first 1000
    events, P:149).  ``num_classes`` defaults to ``len(set(labels))`` like P:153 (which
    assumes the labels are 0..C-1).
    """
    all_labels = []
    for lab in labels_iterable:
        all_labels.extend(np.asarray(lab).reshape(-1).tolist())
    counts = Counter(all_labels)
    if num_classes is None:
        num_classes = len(set(all_labels))
    max_count = max(counts.values())
    w = []
    for c in range(num_classes):
        if c in counts:
            v = max_count / counts[c]
            if c == 2:
                v *= 2.0
            w.append(v)
        else:
            w.append(1.0)
    s = sum(w)
    return [v * num_classes / s for v in w]


def _scene(rng, grid, n_points, num_classes, dense):
    G = grid
    if dense:
        idx = np.arange(G ** 3, dtype=np.int64)
    else:
        idx = rng.choice(G ** 3, size=n_points, replace=False)
    i = idx // (G * G)
    j = (idx // G) % G
    k = idx % G
    xyz = (np.stack([i, j, k], axis=1).astype(np.float32) + 0.5) * (2.0 / G) - 1.0
    e = (rng.uniform(size=idx.shape[0]) if dense else rng.exponential(size=idx.shape[0]))
    pts = np.concatenate([xyz, e.astype(np.float32)[:, None]], axis=1)
    # labels: 1 inside a random sphere, 2 (or 1 when C==2) along a random track
    c = rng.uniform(-0.5, 0.5, size=3).astype(np.float32)
    r = np.float32(rng.uniform(0.3, 0.7))
    o = rng.uniform(-0.5, 0.5, size=3).astype(np.float32)
    d = rng.normal(size=3).astype(np.float32)
    d /= np.linalg.norm(d)
    lab = np.zeros(idx.shape[0], np.int64)
    if num_classes >= 2:
        lab[((xyz - c) ** 2).sum(1) < r * r] = 1
    rel = xyz - o
    perp = rel - (rel @ d)[:, None] * d[None, :]
    track = (perp ** 2).sum(1) < np.float32(0.08) ** 2
    lab[track] = 2 if num_classes >= 3 else min(1, num_classes - 1)
    return pts.astype(np.float32), lab


def synthetic_clouds(seed, n_points, num_classes=2, grid=32, dense=False):
    """List of (points[N_i,4] f32, labels[N_i] i64) numpy clouds, numpy PCG64 seeded.

    ``n_points`` is a list of per-scene point counts (ignored when ``dense``: every voxel
    of the G^3 grid is a point).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    return [_scene(rng, grid, n, num_classes, dense) for n in n_points]


def synthetic_batch(seed, n_points, num_classes=2, grid=32, dense=False):
    """Padded numpy batch (points[B,N,4], labels[B,N], mask[B,N]) of synthetic clouds."""
    clouds = synthetic_clouds(seed, n_points, num_classes, grid, dense)
    B = len(clouds)
    N = max(p.shape[0] for p, _ in clouds)
    pts = np.zeros((B, N, 4), np.float32)
    lab = np.full((B, N), -1, np.int64)
    msk = np.zeros((B, N), bool)
    for b, (p, l) in enumerate(clouds):
        pts[b, :p.shape[0]] = p
        lab[b, :p.shape[0]] = l
        msk[b, :p.shape[0]] = True
    return pts, lab, msk


def shard_bounds(batch_size, rank, world_size):
    """[lo, hi) scene range of ``rank`` under tensor.chunk(world_size, dim=0)."""
    chunk = -(-batch_size // world_size)
    lo = min(rank * chunk, batch_size)
    return lo, min(lo + chunk, batch_size)


def shard_batch(tensors, rank, world_size):
    """Slice each [B,...] tensor to this rank's scenes (DataParallel's scatter rule)."""
    lo, hi = shard_bounds(tensors[0].shape[0], rank, world_size)
    return tuple(t[lo:hi] for t in tensors)

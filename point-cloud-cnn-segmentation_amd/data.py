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
* ``PointCloudDataset`` — P:20-42, the HDF5 vlen event reader (needs h5py, absent in this
  image: it raises ImportError with a pointer to the CSR store instead).
* ``CSRPointCloudDataset`` / ``write_csr_store`` — the same per-event contract over a
  memory-mapped CSR store (flat points f32 [T,4], labels [T], offsets [E+1] as .npy files),
  the vlen layout of the reference's HDF5 files without the h5py dependency.
* ``RaggedBatch`` / ``ragged_collate`` — CSR batching for the DataLoader: no host padding;
  ``pcs_amd.loader`` pads on the device (pcs_pad_scatter) after a pinned async copy.
"""
from __future__ import annotations

import os
from collections import Counter
from typing import NamedTuple

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
    return class_weights_from_counts(counts, num_classes)


def class_weights_from_counts(counts, num_classes):
    """The P:168-183 formula from per-label counts (a mapping label -> count, or a sequence
    indexed by label; labels with a zero count are absent, as in the reference's Counter)."""
    if not hasattr(counts, "items"):
        counts = {c: int(v) for c, v in enumerate(counts) if int(v) > 0}
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


def label_counts(labels_iterable, num_classes):
    """Per-class counts (int64 [num_classes]) of the labels 0..num_classes-1 (pads, -1, skipped)."""
    out = np.zeros(num_classes, dtype=np.int64)
    for lab in labels_iterable:
        a = np.asarray(lab).reshape(-1)
        a = a[(a >= 0) & (a < num_classes)]
        out += np.bincount(a.astype(np.int64), minlength=num_classes)[:num_classes]
    return out


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


# ----------------------------------------------------------------------------- event stores
class PointCloudDataset:
    """The reference's HDF5 event reader (P:20-42): ``data`` holds one flat float32 vlen
    array (x,y,z,e per point) per event, ``labels`` one int array per event.  Returns
    (points f32 [N,4], labels i64 [N]) torch tensors like P:31-36."""

    def __init__(self, data_path, label_path):
        try:
            import h5py
        except ImportError as e:   # h5py is not part of this image
            raise ImportError(
                "PointCloudDataset needs h5py to read the reference's HDF5 files; convert them "
                "with convert_hdf5_to_csr() on a machine that has it, then use "
                "CSRPointCloudDataset") from e
        self.data_file = h5py.File(data_path, "r")
        self.label_file = h5py.File(label_path, "r")
        self.num_events = len(self.data_file["data"])

    def __len__(self):
        return self.num_events

    def __getitem__(self, idx):
        import torch
        points = torch.tensor(np.asarray(self.data_file["data"][idx]).reshape(-1, 4), dtype=torch.float32)
        labels = torch.tensor(np.asarray(self.label_file["labels"][idx]), dtype=torch.long)
        return points, labels

    def __del__(self):
        for f in ("data_file", "label_file"):
            if hasattr(self, f):
                getattr(self, f).close()


CSR_FILES = ("points.npy", "labels.npy", "offsets.npy")


def write_csr_store(path, clouds, label_dtype=np.int32):
    """Write [(points[N_i,4], labels[N_i])] as a CSR store directory (three .npy files)."""
    os.makedirs(path, exist_ok=True)
    lens = np.array([len(p) for p, _ in clouds], np.int64)
    offsets = np.zeros(len(clouds) + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    pts = np.concatenate([np.asarray(p, np.float32).reshape(-1, 4) for p, _ in clouds]) if clouds \
        else np.zeros((0, 4), np.float32)
    lab = np.concatenate([np.asarray(l).reshape(-1) for _, l in clouds]).astype(label_dtype) if clouds \
        else np.zeros(0, label_dtype)
    for name, arr in zip(CSR_FILES, (pts, lab, offsets)):
        np.save(os.path.join(path, name), arr)
    return path


def convert_hdf5_to_csr(data_path, label_path, out_dir, label_dtype=np.int32):
    """Stream the reference's HDF5 vlen files (P:20-36) into a CSR store (needs h5py)."""
    ds = PointCloudDataset(data_path, label_path)
    clouds = [(p.numpy(), l.numpy()) for p, l in (ds[i] for i in range(len(ds)))]
    return write_csr_store(out_dir, clouds, label_dtype)


class CSRPointCloudDataset:
    """Per-event (points f32 [N,4], labels i64 [N]) over a memory-mapped CSR store: the
    __getitem__ contract of PointCloudDataset (P:30-36) without h5py.  ``__getitem__``
    returns torch tensors; ``cloud(idx)`` returns the numpy views (no copy)."""

    def __init__(self, path):
        self.points, self.labels, self.offsets = (
            np.load(os.path.join(path, n), mmap_mode="r") for n in CSR_FILES)
        if self.points.ndim != 2 or self.points.shape[1] != 4 or self.offsets[-1] != len(self.points) \
                or len(self.labels) != len(self.points) or np.any(np.diff(self.offsets) < 0):
            raise ValueError(f"{path}: inconsistent CSR store")
        self.num_events = len(self.offsets) - 1

    def __len__(self):
        return self.num_events

    def cloud(self, idx):
        lo, hi = int(self.offsets[idx]), int(self.offsets[idx + 1])
        return self.points[lo:hi], self.labels[lo:hi]

    def __getitem__(self, idx):
        import torch
        p, l = self.cloud(idx)
        return torch.from_numpy(np.array(p, np.float32)), torch.from_numpy(np.array(l, np.int64))


# ----------------------------------------------------------------------------- CSR batching
class RaggedBatch(NamedTuple):
    """A batch in CSR form: scene b owns rows offsets[b]:offsets[b+1] of points / labels.
    A NamedTuple of tensors, so DataLoader(pin_memory=True) pins every field."""
    points: "torch.Tensor"    # f32 [T, 4]
    labels: "torch.Tensor"    # i32 or i64 [T]
    offsets: "torch.Tensor"   # i64 [B + 1]

    @property
    def num_scenes(self):
        return self.offsets.numel() - 1

    @property
    def max_points(self):
        """The padded length collate_fn would use (P:50)."""
        if self.num_scenes == 0:
            return 0
        return int((self.offsets[1:] - self.offsets[:-1]).max())


def ragged_collate(batch, label_dtype=None):
    """DataLoader collate building a RaggedBatch (no padding) from (points, labels) pairs;
    the padded view collate_fn (P:44-63) returns is produced on the device by
    pcs_amd.loader.pad_on_device."""
    import torch
    points_list, labels_list = zip(*batch)
    lens = torch.tensor([p.shape[0] for p in points_list], dtype=torch.int64)
    offsets = torch.zeros(len(points_list) + 1, dtype=torch.int64)
    torch.cumsum(lens, 0, out=offsets[1:])
    pts = torch.cat([p.reshape(-1, 4).float() for p in points_list])
    lab = torch.cat([l.reshape(-1) for l in labels_list])
    if label_dtype is not None:
        lab = lab.to(label_dtype)
    return RaggedBatch(pts.contiguous(), lab.contiguous(), offsets)


def occupied_clouds(seed, num_scenes, grid=256, occupancy=0.02, jitter=0.1, num_classes=2):
    """Occupied-only sparse clouds of SURVEY §8(d) cfg3: each scene keeps a ragged
    ~``occupancy`` fraction of the grid^3 lattice voxels (count drawn per scene within
    +-``jitter``), xyz = voxel centres, e ~ Exp(1), labels as synthetic_clouds."""
    rng = np.random.Generator(np.random.PCG64(seed))
    base = occupancy * grid ** 3
    n = [int(base * rng.uniform(1 - jitter, 1 + jitter)) for _ in range(num_scenes)]
    return [_scene(rng, grid, k, num_classes, dense=False) for k in n]


def jittered_clouds(seed, num_scenes, grid=256, occupancy=0.01, per_voxel=4, num_classes=2, noise=0.2):
    """Raw-hit clouds for the voxel path (pcs_amd.voxel): occupied_clouds' lattice cells, each
    repeated 1..per_voxel times with the points jittered inside their cell, fresh e ~ Exp(1),
    and a fraction ``noise`` of labels redrawn from {-1, 0, .., C-1} (so voxels mix labels)."""
    rng = np.random.Generator(np.random.PCG64(seed + 7919))
    out = []
    for p, l in occupied_clouds(seed, num_scenes, grid=grid, occupancy=occupancy, num_classes=num_classes):
        reps = rng.integers(1, per_voxel + 1, size=len(p))
        q = np.repeat(p, reps, axis=0)
        q[:, :3] += rng.uniform(-0.49, 0.49, size=(len(q), 3)).astype(np.float32) * (2.0 / grid)
        q[:, 3] = rng.exponential(size=len(q)).astype(np.float32)
        lab = np.repeat(l, reps)
        flip = rng.random(len(lab)) < noise
        lab[flip] = rng.integers(-1, num_classes, size=int(flip.sum()))
        out.append((q.astype(np.float32), lab.astype(np.int64)))
    return out

"""Host side of the data path (reference P:20-63) on CPU.

* CSR store round trip and the per-event contract of PointCloudDataset.__getitem__
  (points f32 [N,4], labels i64 [N], P:30-36).
* ragged_collate (CSR batching) holds exactly what collate_fn (P:44-63) would pad: the
  oracle's collate restatement applied to the CSR rows equals the reference-semantics
  collate_fn on the original clouds.
* PointCloudDataset needs h5py (absent here) and says so.
* global_max_points over a world-2 gloo group (DataParallel pads to the global max, P:50).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pointnet_oracle as orc
from pcs_amd.data import (CSRPointCloudDataset, PointCloudDataset, RaggedBatch, collate_fn,
                          occupied_clouds, ragged_collate, synthetic_clouds, write_csr_store)


def _clouds():
    cl = synthetic_clouds(11, [300, 0, 1, 257, 128], num_classes=3, grid=32)
    return [(torch.from_numpy(p), torch.from_numpy(l)) for p, l in cl]


def test_csr_store_round_trip(tmp_path):
    cl = _clouds()
    write_csr_store(str(tmp_path), [(p.numpy(), l.numpy()) for p, l in cl])
    ds = CSRPointCloudDataset(str(tmp_path))
    assert len(ds) == len(cl)
    for i, (p, l) in enumerate(cl):
        q, m = ds[i]
        assert q.dtype == torch.float32 and q.shape == (p.shape[0], 4)
        assert m.dtype == torch.int64
        assert torch.equal(q, p) and torch.equal(m, l)


def test_csr_store_rejects_inconsistent_offsets(tmp_path):
    write_csr_store(str(tmp_path), [(p.numpy(), l.numpy()) for p, l in _clouds()])
    off = np.load(tmp_path / "offsets.npy")
    off[-1] += 1
    np.save(tmp_path / "offsets.npy", off)
    with pytest.raises(ValueError):
        CSRPointCloudDataset(str(tmp_path))


def test_ragged_collate_matches_collate_fn():
    cl = _clouds()
    rb = ragged_collate(cl)
    assert isinstance(rb, RaggedBatch)
    assert rb.offsets.tolist() == [0, 300, 300, 301, 558, 686]
    assert rb.max_points == 300 and rb.num_scenes == 5
    # re-pad the CSR rows with the oracle's collate restatement -> collate_fn's tensors
    o = rb.offsets
    pl = [rb.points[o[i]:o[i + 1]].numpy() for i in range(rb.num_scenes)]
    ll = [rb.labels[o[i]:o[i + 1]].numpy() for i in range(rb.num_scenes)]
    pts, lab, msk = orc.collate(pl, ll)
    rp, rl, rm = collate_fn(cl)
    assert np.array_equal(pts, rp.numpy()) and np.array_equal(lab, rl.numpy())
    assert np.array_equal(msk, rm.numpy())


def test_ragged_collate_label_dtype_and_dataloader(tmp_path):
    cl = _clouds()
    write_csr_store(str(tmp_path), [(p.numpy(), l.numpy()) for p, l in cl])
    ds = CSRPointCloudDataset(str(tmp_path))
    dl = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False,
                                     collate_fn=lambda b: ragged_collate(b, torch.int32))
    batches = list(dl)
    assert len(batches) == 3
    assert batches[0].labels.dtype == torch.int32
    assert batches[0].offsets.tolist() == [0, 300, 300]
    assert batches[2].max_points == 128


def test_hdf5_reader_needs_h5py():
    try:
        import h5py  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError, match="CSRPointCloudDataset"):
            PointCloudDataset("data.h5", "labels.h5")
    else:
        pytest.skip("h5py present: the reader is exercised by real data")


def test_occupied_clouds_are_ragged_lattice_points():
    cl = occupied_clouds(3, 4, grid=256, occupancy=2e-4, jitter=0.1)
    n = [len(p) for p, _ in cl]
    assert len(set(n)) == 4 and all(0.9 * 3355 <= k <= 1.1 * 3356 for k in n)
    for p, l in cl:
        idx = np.round((p[:, :3] + 1.0) * 128 - 0.5).astype(np.int64)
        assert idx.min() >= 0 and idx.max() < 256
        flat = (idx[:, 0] * 256 + idx[:, 1]) * 256 + idx[:, 2]
        assert len(np.unique(flat)) == len(p)          # occupied-only: one point per voxel
        assert set(np.unique(l)) <= {0, 1}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _max_worker(rank, world, port, out):
    from pcs_amd.loader import global_max_points
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out[rank] = global_max_points([300, 4097][rank])
    finally:
        dist.destroy_process_group()


def test_global_max_points_gloo_world2():
    out = mp.Manager().dict()
    mp.spawn(_max_worker, args=(2, _port(), out), nprocs=2, join=True)
    assert dict(out) == {0: 4097, 1: 4097}

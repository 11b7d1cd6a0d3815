"""Device-side collate and the occupied-only (cfg3-shaped) path on MI355X.

* pcs_pad_scatter (through pad_on_device) is byte-identical to collate_fn (P:44-63) on
  ragged batches with empty / single-point scenes, int32 and int64 labels, and a padded
  length beyond the batch max (the DP global max).
* DevicePrefetcher over a pinned DataLoader yields the same batches.
* Sparse occupied-only clouds on a 256^3 lattice (ragged, N not a multiple of any tile):
  padded on the device, the fp32 model matches the numpy oracle on the same padded batch
  (logits 1e-4, gradients 2e-3 as in test_gpu_parity); the bf16 fused step runs and tracks
  the fp32 loss.
"""
import numpy as np
import pytest
import torch

import pointnet_oracle as orc
from golden_util import rel_err
from pcs_amd.data import collate_fn, occupied_clouds, ragged_collate, synthetic_clouds

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _clouds(lens, seed=5, C=3):
    return [(torch.from_numpy(p), torch.from_numpy(l))
            for p, l in synthetic_clouds(seed, lens, num_classes=C, grid=32)]


@pytest.mark.parametrize("lens", [[300, 0, 1, 257, 128], [1], [4096, 3000, 4096, 2500], [0, 0]])
@pytest.mark.parametrize("label_dtype", [torch.int64, torch.int32])
def test_pad_on_device_is_collate_fn(lens, label_dtype):
    from pcs_amd.loader import pad_on_device
    cl = _clouds(lens)
    rb = ragged_collate(cl, label_dtype)
    p, l, m = pad_on_device(rb, DEV)
    rp, rl, rm = collate_fn(cl)
    torch.cuda.synchronize()
    assert p.dtype == torch.float32 and l.dtype == torch.int64 and m.dtype == torch.bool
    assert torch.equal(p.cpu(), rp) and torch.equal(l.cpu(), rl) and torch.equal(m.cpu(), rm)


def test_pad_on_device_longer_rows_and_device_input():
    from pcs_amd.loader import pad_on_device
    cl = _clouds([100, 37])
    rb = ragged_collate(cl)
    rbd = type(rb)(*(t.to(DEV) for t in rb))
    p, l, m = pad_on_device(rbd, DEV, scene_rows=200)
    rp, rl, rm = collate_fn(cl + [(torch.zeros(200, 4), torch.zeros(200, dtype=torch.long))])
    assert torch.equal(p.cpu(), rp[:2]) and torch.equal(l.cpu(), rl[:2]) and torch.equal(m.cpu(), rm[:2])
    with pytest.raises(ValueError):
        pad_on_device(rb, DEV, scene_rows=50)


def test_device_prefetcher_matches_collate_fn():
    from pcs_amd.loader import DevicePrefetcher
    cl = _clouds([300, 17, 900, 1, 64, 513, 2], seed=9)
    dl = torch.utils.data.DataLoader(cl, batch_size=3, shuffle=False, collate_fn=ragged_collate,
                                     pin_memory=True)
    got = [tuple(t.cpu() for t in b) for b in DevicePrefetcher(dl, DEV)]
    ref = [collate_fn(cl[i:i + 3]) for i in range(0, len(cl), 3)]
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert all(torch.equal(a, b) for a, b in zip(g, r))


def _model(sd, C, dtype="fp32"):
    from pcs_amd.model import PointNetSegmentation
    m = PointNetSegmentation(C, compute_dtype=dtype).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
    return m


def test_occupied_only_ragged_fp32_parity():
    """cfg3 geometry at test size: 256^3 lattice, ragged occupied-only scenes (~3.3k points,
    no length a multiple of a tile), padded on the device, train step vs the oracle."""
    from pcs_amd.loader import pad_on_device
    cl = occupied_clouds(21, 3, grid=256, occupancy=2e-4)
    rb = ragged_collate([(torch.from_numpy(p), torch.from_numpy(l)) for p, l in cl])
    pts, lab, _ = pad_on_device(rb, DEV)
    B, N = lab.shape
    assert N % 64 != 0
    sd = orc.init_params(2, 31, bn_affine_random=True)
    masks = orc.dropout_masks(4, B * N)
    w = np.array([0.7, 1.3], np.float32)
    m = _model(sd, 2)
    m.train()
    m.set_dropout_masks(*(torch.from_numpy(np.packbits(k, axis=1, bitorder="little")).to(DEV) for k in masks))
    out = m(pts)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    loss = crit(out.contiguous().view(-1, 2), lab.view(-1))
    loss.backward()
    rloss, rlogits, grads, _ = orc.train_step(sd, pts.cpu().numpy(), lab.cpu().numpy(), w, masks=masks)
    assert rel_err(out.detach().cpu().numpy(), rlogits) < 1e-4
    assert abs(loss.item() - rloss) < 1e-4 * max(1.0, abs(rloss))
    gmax = max(np.linalg.norm(v) for v in grads.values())
    for n, p in m.named_parameters():
        if n.endswith(".bias") and not n.startswith(("bn", "seg_conv4")):
            continue   # BN-cancelled conv biases: analytically 0 (see test_gpu_parity)
        rv = grads[n].reshape(-1)
        e = np.linalg.norm(p.grad.detach().cpu().numpy().reshape(-1) - rv) / max(np.linalg.norm(rv), 1e-3 * gmax)
        assert e < 2e-3, (n, e)


def test_occupied_only_bf16_fused_step_tracks_fp32():
    """Larger ragged occupied-only batch through the bf16 fused step (256x256 kernels with
    a ragged tail in every scene): finite and within bf16 tolerance of the fp32 loss."""
    from pcs_amd.loader import pad_on_device
    from pcs_amd.train import FusedTrainStep
    cl = occupied_clouds(8, 4, grid=256, occupancy=2e-3)
    rb = ragged_collate([(torch.from_numpy(p), torch.from_numpy(l)) for p, l in cl])
    pts, lab, _ = pad_on_device(rb, DEV)
    assert lab.shape[1] % 256 != 0
    sd = orc.init_params(2, 3)
    losses = {}
    for dt in ("fp32", "bf16"):
        m = _model(sd, 2, dt)
        m.train()
        step = FusedTrainStep(m, class_weight=[0.6, 1.4])
        losses[dt] = float(step(pts, lab, seed=77))
    assert np.isfinite(losses["bf16"])
    assert abs(losses["bf16"] - losses["fp32"]) < 2e-2 * max(1.0, abs(losses["fp32"])), losses

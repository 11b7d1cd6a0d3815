"""Point -> voxel path on MI355X (csrc/voxel.hip) against oracle/voxel_oracle.py (not
reference parity: the reference has no voxelisation).  Integer outputs
bit-exact (ids, voxel order, inverse map, counts, labels, CSR offsets); features within
fp32 summation tolerance; the voxel batch then trains through the model and per-voxel
logits gather back to points."""
import numpy as np
import pytest
import torch

import voxel_oracle as vo
from pcs_amd.data import RaggedBatch, occupied_clouds, ragged_collate

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
BOX = ((-1.0, -1.0, -1.0), (1.0, 1.0, 1.0))


def _jittered(seed, n_scenes, grid, per_voxel):
    """Clouds with several points per voxel (pcs_amd.data.jittered_clouds, 1 % of a G^3 lattice)."""
    from pcs_amd.data import jittered_clouds
    return jittered_clouds(seed, n_scenes, grid=grid, occupancy=0.01, per_voxel=per_voxel)


@pytest.mark.parametrize("grid", [4, 32, 256])
def test_voxel_ids_bit_exact(grid):
    from pcs_amd.voxel import voxel_ids
    rng = np.random.Generator(np.random.PCG64(grid))
    pts = rng.uniform(-1.2, 1.2, size=(100000, 4)).astype(np.float32)
    pts[:7, :3] = np.array([[-1, -1, -1], [1, 1, 1], [0, 0, 0], [-1.5, 2, 0.5], [0.99999994, 0.5, -0.5],
                            [-0.9999999, 0.0, 1e-8], [0.5, -0.25, 0.125]], np.float32)
    got = voxel_ids(torch.from_numpy(pts).to(DEV), grid, *BOX).cpu().numpy()
    assert np.array_equal(got, vo.voxel_ids(pts, grid, *BOX))


@pytest.mark.parametrize("grid,per_voxel", [(64, 3), (256, 1), (16, 6)])
def test_voxelize_matches_oracle(grid, per_voxel):
    from pcs_amd.voxel import voxelize
    clouds = _jittered(7 + grid, 3, grid=64, per_voxel=per_voxel)
    clouds.insert(1, (np.zeros((0, 4), np.float32), np.zeros(0, np.int64)))   # empty scene
    rb = ragged_collate([(torch.from_numpy(p), torch.from_numpy(l)) for p, l in clouds])
    vb = voxelize(rb, grid, *BOX, num_classes=2, device=DEV)
    vop, vp, vl, vc, voff = vo.voxelize(rb.points.numpy(), rb.labels.numpy(), rb.offsets.numpy(), grid, *BOX, 2)
    assert np.array_equal(vb.voxel_of_point.cpu().numpy(), vop)
    assert np.array_equal(vb.counts.cpu().numpy(), vc)
    assert np.array_equal(vb.batch.labels.cpu().numpy(), vl)
    assert np.array_equal(vb.batch.offsets.cpu().numpy(), voff)
    np.testing.assert_allclose(vb.batch.points.cpu().numpy(), vp, rtol=2e-6, atol=1e-6)


def test_voxel_batch_trains_and_gathers_back():
    from pcs_amd.loader import pad_on_device
    from pcs_amd.model import PointNetSegmentation
    from pcs_amd.train import FusedTrainStep
    from pcs_amd.voxel import to_points, voxelize
    clouds = _jittered(3, 4, grid=128, per_voxel=4)
    rb = ragged_collate([(torch.from_numpy(p), torch.from_numpy(l)) for p, l in clouds])
    vb = voxelize(rb, 128, *BOX, num_classes=2, device=DEV)
    x, y, _ = pad_on_device(vb.batch, DEV)
    m = PointNetSegmentation(2, compute_dtype="bf16").to(DEV)
    loss = float(FusedTrainStep(m, class_weight=[0.5, 1.5])(x, y, seed=5))
    assert np.isfinite(loss)
    m.eval()
    with torch.no_grad():
        logits = m(x)                                   # [B, Nv, 2]
    pl = to_points(logits, vb)                          # [T, 2]
    # reference gather: point p -> its voxel's row in the padded batch
    off = vb.batch.offsets.cpu().numpy()
    vop = vb.voxel_of_point.cpu().numpy()
    scene = np.searchsorted(off, vop, side="right") - 1
    rows = scene * x.shape[1] + (vop - off[scene])
    assert torch.equal(pl.cpu(), logits.reshape(-1, 2).cpu()[torch.from_numpy(rows)])

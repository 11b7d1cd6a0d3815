"""Throughput of the point -> voxel scatter (pcs_voxelize) at the cfg3 geometry: 4 scenes of
jittered points, ~2 % of a 256^3 lattice occupied, 1-4 points per voxel (~0.85 M points per
scene).  Prints M points/s (device-resident CSR input; includes the voxel-count read)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from pcs_amd.data import jittered_clouds, ragged_collate  # noqa: E402
from pcs_amd.voxel import voxelize  # noqa: E402

DEV = torch.device("cuda")
clouds = jittered_clouds(11, 4, grid=256, occupancy=0.02, per_voxel=4)
rb = ragged_collate([(torch.from_numpy(p), torch.from_numpy(l)) for p, l in clouds])
rbd = type(rb)(*(t.to(DEV) for t in rb))
T = rb.points.shape[0]
for _ in range(2):
    vb = voxelize(rbd, 256, num_classes=2, device=DEV)
torch.cuda.synchronize()
reps = 10
t0 = time.perf_counter()
for _ in range(reps):
    vb = voxelize(rbd, 256, num_classes=2, device=DEV)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print(f"voxelize: {T} points -> {vb.counts.numel()} voxels in {dt * 1e3:.3f} ms = {T / dt / 1e6:.1f} M points/s")

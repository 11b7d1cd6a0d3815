"""The sparse-voxel oracle (oracle/sparse_oracle.py) against brute force on small cases (CPU), and
the submanifold convolution restatement against torch's dense conv3d on the occupied sites."""
import numpy as np
import torch
import torch.nn.functional as F

import sparse_oracle as so


def _keys(seed, G, B, frac):
    rng = np.random.default_rng(seed)
    n = int(frac * B * G ** 3)
    return np.unique(rng.integers(0, B * G ** 3, size=n)).astype(np.int64)


def test_neighbors_bruteforce():
    G, B = 6, 2
    keys = _keys(1, G, B, 0.3)
    nbr = so.neighbors(keys, G)
    s, ix, iy, iz = so.decode(keys, G)
    for v in range(0, len(keys), 7):
        for t in range(27):
            a, b, c = t // 9 - 1, (t // 3) % 3 - 1, t % 3 - 1
            hit = np.nonzero((s == s[v]) & (ix == ix[v] + a) & (iy == iy[v] + b) & (iz == iz[v] + c))[0]
            assert nbr[v, t] == (hit[0] if len(hit) else -1)


def test_submanifold_conv_equals_dense_on_occupied_sites():
    G, B = 7, 2
    keys = _keys(2, G, B, 0.25)
    rng = np.random.default_rng(3)
    x = rng.standard_normal((len(keys), 5))
    w = rng.standard_normal((6, 5, 3, 3, 3))
    b = rng.standard_normal(6)
    y = so.submanifold_conv(x, w, b, so.neighbors(keys, G))
    s, ix, iy, iz = so.decode(keys, G)
    d = torch.zeros(B, 5, G, G, G, dtype=torch.float64)
    d[s, :, ix, iy, iz] = torch.from_numpy(x)
    ref = F.conv3d(d, torch.from_numpy(w), torch.from_numpy(b), padding=1)[s, :, ix, iy, iz].numpy()
    assert np.abs(y - ref).max() < 1e-10

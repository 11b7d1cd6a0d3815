"""The voxel oracle (oracle/voxel_oracle.py) pinned against its dictionary restatement, and
its float32 id arithmetic against hand-computed cases (CPU).  Build-defined semantics: the
reference has no voxelisation, so this is not reference parity."""
import numpy as np

import voxel_oracle as vo


def _cloud(seed, n, spread=1.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    p = rng.uniform(-spread, spread, size=(n, 4)).astype(np.float32)
    p[:, 3] = rng.exponential(size=n).astype(np.float32)
    return p


def test_voxel_ids_hand_cases():
    pts = np.array([[-1, -1, -1, 0], [1, 1, 1, 0], [0, 0, 0, 0], [-2, 0.5, 3, 0],
                    [0.99999994, -0.5, 0.25, 0]], np.float32)
    ids = vo.voxel_ids(pts, 4, (-1, -1, -1), (1, 1, 1))
    # (-1,-1,-1) -> cell 0; upper bound -> last cell; 0 -> cell 2; outside -> clamped
    assert ids.tolist() == [0, 63, (2 * 4 + 2) * 4 + 2, (0 * 4 + 3) * 4 + 3, (3 * 4 + 1) * 4 + 2]


def test_voxelize_matches_bruteforce():
    pts = np.concatenate([_cloud(1, 500), _cloud(2, 300, 0.2), _cloud(3, 1)])
    lab = np.random.Generator(np.random.PCG64(4)).integers(-1, 3, size=len(pts))
    off = np.array([0, 500, 500, 800, 801])   # includes an empty scene
    vop, vp, vl, vc, voff = vo.voxelize(pts, lab, off, 8, (-1, -1, -1), (1, 1, 1), 3)
    ref = vo.voxelize_bruteforce(pts, lab, off, 8, (-1, -1, -1), (1, 1, 1), 3)
    assert len(ref) == len(vp) == len(vl) == len(vc)
    for v, ((b, vid), ps, best) in enumerate(ref):
        assert vc[v] == len(ps) and vl[v] == best and all(vop[p] == v for p in ps)
        np.testing.assert_allclose(vp[v, :3], pts[ps, :3].mean(0), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(vp[v, 3], pts[ps, 3].sum(), rtol=1e-5)
    scenes = [b for (b, _), _, _ in ref]
    assert voff.tolist() == [int(np.searchsorted(scenes, b)) for b in range(5)]

"""CPU restatement of the occupied-voxel (sparse) indexing (TEST INFRASTRUCTURE: imported only by
tests/ as the checker of csrc/sparse.hip; the product path never calls it).

Build-defined, NOT reference parity: the reference segments raw points and has no voxel grid
(SURVEY §0.3, §8 f4).  Its voxel key is the one of oracle/voxel_oracle.py (scene * G^3 +
(ix * G + iy) * G + iz).  The neighbour map is the 27-tap submanifold map: nbr[v][t] = row of
the voxel at (ix + a - 1, iy + b - 1, iz + c - 1) of the same scene, t = (a * 3 + b) * 3 + c, or
-1 -- the tap order of a torch Conv3d weight [Cout, Cin, 3, 3, 3] on a dense grid indexed
[scene, ix, iy, iz].  Plain dict lookups (no hashing scheme is restated: the device table's
slot layout is unobservable, only its lookups are, and those must equal this dict's)."""
import numpy as np


def decode(keys, G):
    k = np.asarray(keys, dtype=np.uint64).astype(np.int64)
    G3 = G * G * G
    scene, loc = k // G3, k % G3
    return scene, loc // (G * G), (loc // G) % G, loc % G


def neighbors(keys, G):
    """int32 [n, 27] neighbour rows of the voxels with these keys."""
    keys = np.asarray(keys, dtype=np.uint64)
    row = {int(k): i for i, k in enumerate(keys)}
    scene, ix, iy, iz = decode(keys, G)
    G3 = G * G * G
    out = np.full((len(keys), 27), -1, dtype=np.int32)
    for t in range(27):
        a, b, c = t // 9 - 1, (t // 3) % 3 - 1, t % 3 - 1
        jx, jy, jz = ix + a, iy + b, iz + c
        ok = (jx >= 0) & (jx < G) & (jy >= 0) & (jy < G) & (jz >= 0) & (jz < G)
        for v in np.nonzero(ok)[0]:
            out[v, t] = row.get(int(scene[v] * G3 + (jx[v] * G + jy[v]) * G + jz[v]), -1)
    return out


def submanifold_conv(x, w, b, nbr):
    """Y[m] = b + sum_t W[:, :, t] X[nbr[m, t]] in fp64; x [n, Cin], w [Cout, Cin, 3, 3, 3]."""
    x = np.asarray(x, np.float64)
    wt = np.asarray(w, np.float64).reshape(w.shape[0], w.shape[1], 27)
    y = np.zeros((nbr.shape[0], w.shape[0]), np.float64) + (0 if b is None else np.asarray(b, np.float64))
    for t in range(27):
        rows = nbr[:, t]
        ok = rows >= 0
        y[ok] += x[rows[ok]] @ wt[:, :, t].T
    return y

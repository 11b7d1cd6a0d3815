"""CPU restatement (numpy) of the point -> voxel path of csrc/voxel.hip.

TEST INFRASTRUCTURE ONLY: imported by tests/ (the checker), never by the product path.

The reference has no voxelisation (its PointNet consumes raw points, point_cloud_segmentation.py
P:98-133); this path comes from the north star's voxel vocabulary (SURVEY.md §0 decision 3,
§8 f4), so this oracle defines the semantics and parity here is "not reference parity":
  * voxel id: ix = clamp(floor(float32((x - lo) / (hi - lo)) * G), 0, G-1) in float32, in this
    operation order; id = (ix * G + iy) * G + iz;
  * one voxel per distinct (scene, id), ordered scene-major then by id;
  * features: mean x, y, z and summed e of the voxel's points (float32 sums in point order);
    label: most frequent label >= 0 (ties -> smaller label; -1 if none); counts;
  * voxel_of_point: each point's voxel index.
`voxelize_bruteforce` restates the same definition with Python dicts, to pin `voxelize`.
"""
import numpy as np


def voxel_ids(points, grid, lo, hi):
    p = np.asarray(points, np.float32)[:, :3]
    lo = np.asarray(lo, np.float32)
    hi = np.asarray(hi, np.float32)
    t = (p - lo) / (hi - lo)                      # float32 division (IEEE, as the kernel)
    i = np.floor(t * np.float32(grid)).astype(np.int64)
    i = np.clip(i, 0, grid - 1)
    return (i[:, 0] * grid + i[:, 1]) * grid + i[:, 2]


def voxelize(points, labels, offsets, grid, lo, hi, num_classes):
    points = np.asarray(points, np.float32)
    T = len(points)
    offsets = np.asarray(offsets, np.int64)
    B = len(offsets) - 1
    scene = np.searchsorted(offsets, np.arange(T), side="right") - 1
    keys = scene.astype(np.uint64) * np.uint64(grid) ** 3 + voxel_ids(points, grid, lo, hi).astype(np.uint64)
    order = np.argsort(keys, kind="stable")
    skeys = keys[order]
    head = np.ones(T, bool)
    head[1:] = skeys[1:] != skeys[:-1]
    starts = np.nonzero(head)[0]
    V = len(starts)
    ends = np.append(starts[1:], T)
    vox_of_point = np.empty(T, np.int64)
    vp = np.zeros((V, 4), np.float32)
    vl = np.full(V, -1, np.int64)
    vc = (ends - starts).astype(np.int64)
    for v, (s, e) in enumerate(zip(starts, ends)):
        idx = order[s:e]
        vox_of_point[idx] = v
        acc = np.zeros(4, np.float32)
        for q in idx:                              # float32 sums in point order
            acc += points[q]
        n = np.float32(e - s)
        vp[v] = [acc[0] / n, acc[1] / n, acc[2] / n, acc[3]]
        if labels is not None:
            lab = np.asarray(labels)[idx]
            lab = lab[(lab >= 0) & (lab < num_classes)]
            if len(lab):
                cnt = np.bincount(lab, minlength=num_classes)
                vl[v] = int(np.argmax(cnt))        # first maximum = smaller label on ties
    vscene = (skeys[starts] // np.uint64(grid) ** 3).astype(np.int64)
    voff = np.searchsorted(vscene, np.arange(B + 1), side="left").astype(np.int64)
    return vox_of_point, vp, vl, vc, voff


def voxelize_bruteforce(points, labels, offsets, grid, lo, hi, num_classes):
    """Dictionary restatement of the same definition (pins `voxelize`)."""
    ids = voxel_ids(points, grid, lo, hi)
    buckets = {}
    for b in range(len(offsets) - 1):
        for p in range(int(offsets[b]), int(offsets[b + 1])):
            buckets.setdefault((b, int(ids[p])), []).append(p)
    keys = sorted(buckets)
    out = []
    for k in keys:
        ps = buckets[k]
        labs = [int(labels[p]) for p in ps if labels is not None and 0 <= labels[p] < num_classes]
        best = -1
        if labs:
            cnt = [labs.count(c) for c in range(num_classes)]
            best = cnt.index(max(cnt))
        out.append((k, ps, best))
    return out

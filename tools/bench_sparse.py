"""Occupied-voxel path at BASELINE configs[2]'s scale: a 256^3 effective grid, jittered clouds
occupying ~2 % of it (pcs_amd.data.jittered_clouds), 4 scenes.  Times the sparse index (voxel keys,
hash table, 27-neighbour map) and one 64 -> 64 submanifold 3x3x3 convolution forward, input
gradient and weight gradient, in the tile-gather form and through per-tap pair lists; prints
voxels/s and the useful TF/s (taps with a neighbour only).
    python tools/bench_sparse.py [reps] [occupancy]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402
from pcs_amd.data import jittered_clouds, ragged_collate  # noqa: E402
from pcs_amd.sparse import TAPS, sparse_voxels  # noqa: E402
from pcs_amd.voxel import voxelize  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    occ = float(sys.argv[2]) if len(sys.argv) > 2 else 0.02
    G, B, C = 256, 4, 64
    dev = torch.device("cuda")
    clouds = jittered_clouds(5, B, grid=G, occupancy=occ, per_voxel=2)
    rb = ragged_collate([(torch.from_numpy(p), torch.from_numpy(l)) for p, l in clouds])
    vb = voxelize(rb, G)
    sv = sparse_voxels(rb, vb)
    V = sv.num_voxels
    pairs = int((sv.nbr >= 0).sum())
    ms_idx = timeit(lambda: sparse_voxels(rb, vb), reps)
    x = torch.randn(V, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(C, TAPS * C, device=dev) * 0.05).to(torch.bfloat16)
    wt = torch.empty_like(w)
    L.call("pcs_conv3d_weight_t", L.ptr(w), C, TAPS, C, L.ptr(wt), L.stream_ptr())
    y = torch.empty(V, C, device=dev, dtype=torch.bfloat16)
    st = L.stream_ptr()
    fwd = lambda: L.call("pcs_sparse_conv", L.ptr(sv.nbr), V, TAPS, L.ptr(x), C, L.ptr(w), C, None, L.ptr(y), L.BF16, 0, st)  # noqa: E731
    dgr = lambda: L.call("pcs_sparse_conv", L.ptr(sv.nbr), V, TAPS, L.ptr(y), C, L.ptr(wt), C, None, L.ptr(x), L.BF16, 1, st)  # noqa: E731
    nb = int(L.load().pcs_sparse_conv_wgrad_workspace(V, TAPS, C, C))
    ws = torch.empty(nb // 4, device=dev)
    dw = torch.empty(C, TAPS * C, device=dev)
    db = torch.empty(C, device=dev)
    wgr = lambda: L.call("pcs_sparse_conv_wgrad", L.ptr(sv.nbr), V, TAPS, L.ptr(x), C, L.ptr(y), C, L.ptr(ws), nb, L.ptr(dw), L.ptr(db), st)  # noqa: E731
    useful = 2.0 * pairs * C * C / 1e12
    print(f"grid {G}^3 x {B} scenes, occupancy {occ}: {V} voxels ({V / B / G ** 3:.4f} of the grid), "
          f"{pairs / V:.2f} occupied taps per voxel", flush=True)
    print(f"sparse index (keys + hash + neighbours): {ms_idx:.3f} ms = {V / ms_idx / 1e3:.1f} M voxels/s", flush=True)
    tot = 0.0
    for name, fn in [("forward", fwd), ("input gradient", dgr), ("weight gradient", wgr)]:
        ms = timeit(fn, reps)
        tot += ms
        print(f"submanifold 3x3x3 {C}->{C} {name}: {ms:.3f} ms = {V / ms / 1e3:.1f} M voxels/s, "
              f"{useful / ms * 1e3:.1f} useful TF/s", flush=True)
    print(f"fwd + bwd: {tot:.3f} ms = {V / tot / 1e3:.1f} M voxels/s", flush=True)
    # the per-tap pair-list form of the same three convolutions (pairs built once per map)
    import ctypes as ct
    ms_pairs = timeit(lambda: (setattr(sv, "_pairs", None), sv.pairs()), 1)
    pin, pout, ppos, tap_off, P = sv.pairs()
    z = torch.empty(max(P, 1), C, device=dev)
    ta = ct.addressof(tap_off)
    pfwd = lambda: L.call("pcs_sparse_conv_pairs", L.ptr(pin), L.ptr(ppos), ta, TAPS, V, L.ptr(x), C, L.ptr(w), C, None, L.ptr(z), L.ptr(y), L.BF16, 0, st)  # noqa: E731
    pdgr = lambda: L.call("pcs_sparse_conv_pairs", L.ptr(pin), L.ptr(ppos), ta, TAPS, V, L.ptr(y), C, L.ptr(wt), C, None, L.ptr(z), L.ptr(x), L.BF16, 1, st)  # noqa: E731
    nbp = int(L.load().pcs_sparse_conv_wgrad_pairs_workspace(ta, TAPS, V, C, C))
    wsp = torch.empty(nbp // 4, device=dev)
    pwgr = lambda: L.call("pcs_sparse_conv_wgrad_pairs", L.ptr(pin), L.ptr(pout), ta, TAPS, V, L.ptr(x), C, L.ptr(y), C, L.ptr(wsp), nbp, L.ptr(dw), L.ptr(db), st)  # noqa: E731
    print(f"pair lists (build, once per neighbour map): {ms_pairs:.3f} ms", flush=True)
    tot = 0.0
    for name, fn in [("forward", pfwd), ("input gradient", pdgr), ("weight gradient", pwgr)]:
        ms = timeit(fn, reps)
        tot += ms
        print(f"pairs: submanifold 3x3x3 {C}->{C} {name}: {ms:.3f} ms = {V / ms / 1e3:.1f} M voxels/s, "
              f"{useful / ms * 1e3:.1f} useful TF/s", flush=True)
    print(f"pairs: fwd + bwd: {tot:.3f} ms = {V / tot / 1e3:.1f} M voxels/s", flush=True)


if __name__ == "__main__":
    main()

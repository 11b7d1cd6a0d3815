"""Occupied-voxel (sparse) path: the north star's "hash-indexed gather" (BASELINE configs[2],
SURVEY §8 f4).  Build-defined, like the rest of the voxel vocabulary: the reference has no voxel
grid, so parity is against oracle/sparse_oracle.py and against torch's dense conv3d evaluated on
the occupied sites ("not reference parity").

    vb = voxelize(rb, grid=256)                          # pcs_voxelize (voxel.py)
    sv = sparse_voxels(rb, vb)                           # keys, hash table, 27-neighbour map
    conv = SubMConv3d(64, 64)                            # torch Conv3d parameter layout
    y = conv(x, sv)                                      # x: bf16 [V, 64] per-voxel features

A submanifold 3x3x3 convolution: outputs exist only at occupied voxels and read only occupied
neighbours (nbr[v][t], -1 = empty), so an occupied-only network never densifies.  The neighbour
map is built once per voxelisation (pcs_voxel_hash_build + pcs_sparse_neighbors) and shared by
every layer at that resolution, forward and backward (the input gradient is the same gather with
the transposed, tap-flipped weight).
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass, field

import torch

from . import _lib as L
from .data import RaggedBatch
from .voxel import CH_ALIGN, VoxelBatch, _box, _bf16_2d, _ceil, _pad_channels

TAPS = 27
# forward / input gradient through the pair lists (gather-GEMM-reduce) when the map has at most
# this many occupied taps per voxel; above it the tile-gather kernel, whose zero rows are then few
# and which keeps no per-pair products in memory.  The weight gradient takes the pair lists at
# every occupancy (PAIR_WGRAD) for layers of at most PAIR_WGRAD_MAX_CH2 = Cin x Cout channel
# pairs (64 -> 64, the shape profiles/bench_sparse_pairs_r05.txt measured); wider layers keep
# the tile-gather weight gradient until the pair form is measured there
PAIR_TAPS_MAX = 3.0
PAIR_WGRAD = True
PAIR_WGRAD_MAX_CH2 = 64 * 64


@dataclass
class SparseVoxels:
    keys: torch.Tensor         # int64 [V] (u64 keys: scene * G^3 + (ix * G + iy) * G + iz), ascending
    table_keys: torch.Tensor   # int64 [cap] (u64, all ones = empty)
    table_vals: torch.Tensor   # int32 [cap]
    nbr: torch.Tensor          # int32 [V, 27]
    grid: int
    _pairs: tuple = field(default=None, repr=False)   # (pair_in, pair_out, pair_pos, tap_off host array, P)

    @property
    def num_voxels(self) -> int:
        return self.keys.numel()

    def pairs(self):
        """Per-tap pair lists of the neighbour map, built once (pcs_sparse_pairs_*; one host read of
        the 27 tap counts): (pair_in, pair_out, pair_pos, tap_off, P) with tap_off a host int64
        array of 28 entries."""
        if self._pairs is None:
            V, dev = self.num_voxels, self.nbr.device
            st = L.stream_ptr(dev)
            nb = int(L.load().pcs_sparse_pairs_workspace(V, TAPS))
            if nb < 0:
                raise L.PcsError(L.load().pcs_last_error().decode())
            ws = torch.empty(max(nb // 4, 1), dtype=torch.int32, device=dev)
            counts = torch.empty(TAPS, dtype=torch.int64, device=dev)
            L.call("pcs_sparse_pairs_count", L.ptr(self.nbr), V, TAPS, L.ptr(ws), L.ptr(counts), st)
            tap_off = (ct.c_int64 * (TAPS + 1))(0, *torch.cumsum(counts, 0).tolist())
            P = int(tap_off[TAPS])
            pin = torch.empty(max(P, 1), dtype=torch.int32, device=dev)
            pout = torch.empty(max(P, 1), dtype=torch.int32, device=dev)
            ppos = torch.empty(V, TAPS, dtype=torch.int32, device=dev)
            L.call("pcs_sparse_pairs_build", L.ptr(self.nbr), V, TAPS, L.ptr(ws), L.ptr(counts), L.ptr(pin), L.ptr(pout),
                   L.ptr(ppos), st)
            self._pairs = (pin, pout, ppos, tap_off, P)
        return self._pairs

    def use_pairs(self) -> bool:
        """The forward / input gradient form for this map (the pair lists or the tile gather)."""
        return self.num_voxels > 0 and self.pairs()[4] <= PAIR_TAPS_MAX * self.num_voxels

    def find(self, keys: torch.Tensor) -> torch.Tensor:
        """int32 rows of the voxels with these keys (-1: unoccupied), one device lookup each."""
        q = keys.reshape(-1).to(torch.int64).contiguous()
        out = torch.empty(q.numel(), dtype=torch.int32, device=q.device)
        L.call("pcs_voxel_hash_find", L.ptr(self.table_keys), L.ptr(self.table_vals), self.table_keys.numel(),
               L.ptr(q), q.numel(), L.ptr(out), L.stream_ptr(q.device))
        return out


def sparse_from_keys(keys: torch.Tensor, grid: int) -> SparseVoxels:
    """Hash table and neighbour map of the occupied voxels with these keys (int64 [V] on a HIP
    device; unique)."""
    if not keys.is_cuda:
        raise RuntimeError("pcs_amd sparse voxels run on a HIP device only (no CPU fallback)")
    keys = keys.to(torch.int64).contiguous()
    n, dev = keys.numel(), keys.device
    # the open-addressing table keeps one row per key: duplicates (or negative keys, which as
    # uint64 could equal the EMPTY sentinel) would silently alias rows
    if n and (int(keys.min()) < 0 or torch.unique(keys).numel() != n):
        raise ValueError("sparse_from_keys: keys must be unique and non-negative")
    cap = int(L.load().pcs_voxel_hash_capacity(n))
    if cap < 0:
        raise L.PcsError(L.load().pcs_last_error().decode())
    tk = torch.empty(cap, dtype=torch.int64, device=dev)
    tv = torch.empty(cap, dtype=torch.int32, device=dev)
    st = L.stream_ptr(dev)
    L.call("pcs_voxel_hash_build", L.ptr(keys), n, L.ptr(tk), L.ptr(tv), cap, st)
    nbr = torch.empty(n, TAPS, dtype=torch.int32, device=dev)
    L.call("pcs_sparse_neighbors", L.ptr(tk), L.ptr(tv), cap, L.ptr(keys), n, int(grid), L.ptr(nbr), st)
    return SparseVoxels(keys, tk, tv, nbr, int(grid))


def sparse_voxels(rb: RaggedBatch, vb: VoxelBatch, lo=(-1.0, -1.0, -1.0), hi=(1.0, 1.0, 1.0)) -> SparseVoxels:
    """The sparse index of a voxelisation (the same points, box and grid as voxelize())."""
    dev = vb.voxel_of_point.device
    pts = rb.points.to(dev, torch.float32).contiguous()
    off = rb.offsets.to(dev, torch.int64).contiguous()
    V = vb.batch.points.shape[0]
    keys = torch.empty(V, dtype=torch.int64, device=dev)
    L.call("pcs_voxel_keys", L.ptr(pts), L.ptr(off), off.numel() - 1, pts.shape[0], int(vb.grid), *_box(lo, hi),
           L.ptr(vb.voxel_of_point), L.ptr(keys), L.stream_ptr(dev))
    return sparse_from_keys(keys, vb.grid)


def _conv_pairs(sv, x, cin, w, cout, bias, y, ydt, flip):
    """y = the submanifold convolution of x through the pair lists (Z = per-pair products, fp32)."""
    pin, _, ppos, tap_off, P = sv.pairs()
    z = torch.empty(max(P, 1), cout, dtype=torch.float32, device=x.device)
    L.call("pcs_sparse_conv_pairs", L.ptr(pin), L.ptr(ppos), ct.addressof(tap_off), TAPS, sv.num_voxels, L.ptr(x), cin,
           L.ptr(w), cout, L.ptr(bias) if bias is not None else None, L.ptr(z), L.ptr(y), ydt, flip,
           L.stream_ptr(x.device))


class _SubMConvFn(torch.autograd.Function):
    """y = b + sum_t W_t x[nbr[:, t]] with w in kernel layout [Cout, 27 * Cin] (fp32 master);
    channel counts off the 64 multiple run zero-padded (exact, as voxel._Conv3dFn)."""

    @staticmethod
    def forward(ctx, x, wk, bias, sv, out_dtype):
        nbr = sv.nbr
        if not x.is_cuda:
            raise RuntimeError("pcs_amd sparse conv runs on a HIP device only (no CPU fallback)")
        if x.dtype != torch.bfloat16 or x.dim() != 2 or nbr.shape != (x.shape[0], TAPS):
            raise ValueError("x must be bf16 [V, C] with a [V, 27] neighbour map")
        V, cin = x.shape
        cout = wk.shape[0]
        if wk.shape[1] != TAPS * cin:
            raise ValueError(f"weight has {wk.shape[1] // TAPS} input channels, x has {cin}")
        cin_k, cout_k = _ceil(cin), _ceil(cout)
        xk = _pad_channels(x, cin_k)
        if (cin_k, cout_k) != (cin, cout):
            wp = wk.new_zeros(cout_k, TAPS, cin_k)
            wp[:cout, :, :cin] = wk.reshape(cout, TAPS, cin)
            wk = wp.reshape(cout_k, TAPS * cin_k)
        wb = _bf16_2d(wk, cout_k, TAPS * cin_k)
        bk = None
        if bias is not None:
            bk = bias.float().contiguous() if cout_k == cout else _pad_channels(bias.float(), cout_k)
        y = torch.empty(V, cout_k, dtype=out_dtype, device=x.device)
        ydt = L.BF16 if out_dtype == torch.bfloat16 else L.F32
        pairs = sv.use_pairs()
        if pairs:
            _conv_pairs(sv, xk, cin_k, wb, cout_k, bk, y, ydt, 0)
        else:
            L.call("pcs_sparse_conv", L.ptr(nbr), V, TAPS, L.ptr(xk), cin_k, L.ptr(wb), cout_k,
                   L.ptr(bk) if bk is not None else None, L.ptr(y), ydt, 0, L.stream_ptr(x.device))
        ctx.save_for_backward(xk, wb, nbr)
        ctx.sv, ctx.pairs = sv, pairs
        ctx.wpairs = PAIR_WGRAD and V > 0 and cin_k * cout_k <= PAIR_WGRAD_MAX_CH2
        ctx.cfg = (bias is not None, cin, cout)
        return y if cout_k == cout else y[:, :cout].contiguous()

    @staticmethod
    def backward(ctx, dy):
        xk, wb, nbr = ctx.saved_tensors
        has_bias, cin, cout = ctx.cfg
        V, cin_k = xk.shape
        cout_k = wb.shape[0]
        dev, st = xk.device, L.stream_ptr(xk.device)
        dyb = _bf16_2d(_pad_channels(dy, cout_k), V, cout_k)
        dx = dwk = db = None
        if ctx.needs_input_grad[0]:
            wt = torch.empty(cin_k, TAPS * cout_k, dtype=torch.bfloat16, device=dev)
            L.call("pcs_conv3d_weight_t", L.ptr(wb), cout_k, TAPS, cin_k, L.ptr(wt), st)
            dx = torch.empty(V, cin_k, dtype=torch.bfloat16, device=dev)
            if ctx.pairs:
                _conv_pairs(ctx.sv, dyb, cout_k, wt, cin_k, None, dx, L.BF16, 1)
            else:
                L.call("pcs_sparse_conv", L.ptr(nbr), V, TAPS, L.ptr(dyb), cout_k, L.ptr(wt), cin_k, None, L.ptr(dx),
                       L.BF16, 1, st)
            if cin_k != cin:
                dx = dx[:, :cin].contiguous()
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            if ctx.wpairs:
                pin, pout, _, tap_off, _ = ctx.sv.pairs()
                nbytes = int(L.load().pcs_sparse_conv_wgrad_pairs_workspace(ct.addressof(tap_off), TAPS, V, cin_k,
                                                                            cout_k))
            else:
                nbytes = int(L.load().pcs_sparse_conv_wgrad_workspace(V, TAPS, cin_k, cout_k))
            if nbytes < 0:
                raise L.PcsError(L.load().pcs_last_error().decode())
            ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=dev)
            dwk = torch.empty(cout_k, TAPS * cin_k, dtype=torch.float32, device=dev)
            db = torch.empty(cout_k, dtype=torch.float32, device=dev) if has_bias else None
            if ctx.wpairs:
                L.call("pcs_sparse_conv_wgrad_pairs", L.ptr(pin), L.ptr(pout), ct.addressof(tap_off), TAPS, V, L.ptr(xk),
                       cin_k, L.ptr(dyb), cout_k, L.ptr(ws), nbytes, L.ptr(dwk), L.ptr(db), st)
            else:
                L.call("pcs_sparse_conv_wgrad", L.ptr(nbr), V, TAPS, L.ptr(xk), cin_k, L.ptr(dyb), cout_k, L.ptr(ws),
                       nbytes, L.ptr(dwk), L.ptr(db), st)
            if (cin_k, cout_k) != (cin, cout):
                dwk = dwk.reshape(cout_k, TAPS, cin_k)[:cout, :, :cin].reshape(cout, TAPS * cin)
                db = db[:cout] if db is not None else None
        return dx, dwk, db, None, None


def submanifold_conv3d(x, weight, sv: SparseVoxels, bias=None, out_dtype=torch.bfloat16):
    """3x3x3 submanifold convolution of per-voxel features x (bf16 [V, Cin]); weight [Cout, Cin,
    3, 3, 3] (torch Conv3d layout, fp32), bias [Cout] or None."""
    cout, cin, k = weight.shape[0], weight.shape[1], weight.shape[2]
    if k != 3 or tuple(weight.shape[2:]) != (3, 3, 3):
        raise ValueError("submanifold_conv3d is the 3x3x3 form")
    wk = weight.permute(0, 2, 3, 4, 1).reshape(cout, TAPS * cin)
    return _SubMConvFn.apply(x, wk, bias, sv, out_dtype)


class SubMConv3d(torch.nn.Module):
    """Submanifold 3x3x3 convolution on occupied voxels with nn.Conv3d(cin, cout, 3, padding=1)'s
    parameter layout and init: on a dense grid that is zero off the occupied voxels, its output at
    the occupied voxels equals that Conv3d's."""

    def __init__(self, cin, cout, bias=True):
        super().__init__()
        ref = torch.nn.Conv3d(cin, cout, 3, 1, 1, bias=bias)
        self.weight, self.bias = ref.weight, ref.bias

    def forward(self, x, sv: SparseVoxels, out_dtype=torch.bfloat16):
        return submanifold_conv3d(x, self.weight, sv, self.bias, out_dtype)


__all__ = ["CH_ALIGN", "SparseVoxels", "SubMConv3d", "sparse_from_keys", "sparse_voxels", "submanifold_conv3d"]

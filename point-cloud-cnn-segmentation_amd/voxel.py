"""Point -> voxel path on the device (north-star voxel vocabulary).

The reference segments raw points (P:98-133); it has no voxel grid.  This module adds the
north star's "point->voxel scatter" and "hash-indexed gather" around the unchanged model:

    vb = voxelize(rb, grid=256, lo=(-1,-1,-1), hi=(1,1,1), num_classes=C)   # pcs_voxelize
    points, labels, masks = pad_on_device(vb.batch)                         # voxel batch
    logits = model(points)                                                   # [B, Nv, C]
    point_logits = to_points(logits, vb)                                     # pcs_gather_rows

A voxel is one occupied cell of a G^3 lattice per scene: (mean x, mean y, mean z, summed e)
of its points, the most frequent label, and its point count.  Integer outputs (voxel ids,
voxel order, inverse map, counts, labels) are bit-exact with oracle/voxel_oracle.py; its
semantics are build-defined ("not reference parity").
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass

import torch

from . import _lib as L
from .data import RaggedBatch


@dataclass
class VoxelBatch:
    batch: RaggedBatch            # voxels as a CSR batch: points [V,4], labels [V], offsets [B+1]
    counts: torch.Tensor          # int64 [V] points per voxel
    voxel_of_point: torch.Tensor  # int64 [T] global voxel index of every input point
    grid: int


def _box(lo, hi):
    lo = [float(v) for v in lo]
    hi = [float(v) for v in hi]
    if len(lo) != 3 or len(hi) != 3 or any(h <= l for l, h in zip(lo, hi)):
        raise ValueError("lo / hi must be 3 bounds with hi > lo")
    return lo + hi


def voxel_ids(points: torch.Tensor, grid: int, lo=(-1.0, -1.0, -1.0), hi=(1.0, 1.0, 1.0)):
    """int64 voxel id of each point (points: fp32 [T, 4] on the device)."""
    if not points.is_cuda:
        raise RuntimeError("voxel_ids runs on a HIP device only (no CPU fallback)")
    pts = points.contiguous().float()
    out = torch.empty(pts.shape[0], dtype=torch.int64, device=pts.device)
    L.call("pcs_voxel_ids", L.ptr(pts), pts.shape[0], int(grid), *_box(lo, hi), L.ptr(out), L.stream_ptr())
    return out


def voxelize(rb: RaggedBatch, grid: int, lo=(-1.0, -1.0, -1.0), hi=(1.0, 1.0, 1.0), num_classes: int = 2,
             device=None) -> VoxelBatch:
    """Occupied-voxel scatter of a CSR batch (pcs_voxelize).  One host read (the voxel count)
    sizes the outputs."""
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if device.type != "cuda":
        raise RuntimeError("voxelize runs on a HIP device only (no CPU fallback)")
    pts = rb.points.to(device, torch.float32).contiguous()
    lab = rb.labels.to(device, torch.int64).contiguous() if rb.labels is not None else None
    off = rb.offsets.to(device, torch.int64).contiguous()
    B, T = off.numel() - 1, pts.shape[0]
    if T == 0:
        raise ValueError("voxelize needs at least one point")
    ws = torch.empty(int(L.load().pcs_voxelize_workspace(T)), dtype=torch.uint8, device=device)
    vop = torch.empty(T, dtype=torch.int64, device=device)
    vpts = torch.empty(T, 4, dtype=torch.float32, device=device)
    vlab = torch.empty(T, dtype=torch.int64, device=device)
    vcnt = torch.empty(T, dtype=torch.int64, device=device)
    voff = torch.empty(B + 1, dtype=torch.int64, device=device)
    nv = torch.empty(1, dtype=torch.int64, device=device)
    L.call("pcs_voxelize", L.ptr(pts), L.ptr(lab), L.ptr(off), B, T, int(grid), *_box(lo, hi), int(num_classes),
           L.ptr(ws), ws.numel(), L.ptr(vop), L.ptr(vpts), L.ptr(vlab), L.ptr(vcnt), L.ptr(voff), L.ptr(nv),
           L.stream_ptr(device))
    V = int(nv.item())
    return VoxelBatch(RaggedBatch(vpts[:V], vlab[:V], voff), vcnt[:V], vop, int(grid))


def to_points(voxel_logits: torch.Tensor, vb: VoxelBatch) -> torch.Tensor:
    """Per-point outputs [T, C] from per-voxel outputs: padded [B, Nv, C] (the model's output
    on pad_on_device(vb.batch)) or flat [V, C] (pcs_voxel_padded_index + pcs_gather_rows)."""
    out_dev = voxel_logits.device
    x = voxel_logits.contiguous().float()
    T = vb.voxel_of_point.numel()
    C = x.shape[-1]
    if x.dim() == 3:
        B, Nv = x.shape[0], x.shape[1]
        idx = torch.empty(T, dtype=torch.int64, device=out_dev)
        L.call("pcs_voxel_padded_index", L.ptr(vb.voxel_of_point), T, L.ptr(vb.batch.offsets), B, Nv, L.ptr(idx),
               L.stream_ptr(out_dev))
        src = x.view(B * Nv, C)
    else:
        idx, src = vb.voxel_of_point, x
    out = torch.empty(T, C, dtype=torch.float32, device=out_dev)
    L.call("pcs_gather_rows", L.ptr(src), src.stride(0), L.ptr(idx), T, C, L.ptr(out), L.stream_ptr(out_dev))
    return out


# ---------------------------------------------------------------------------------------------
# Dense 3-D convolutions on channels-last voxel grids (pcs_conv3d*, csrc/conv3d.hip): the north
# star's U-Net building blocks -- the 3x3x3 stencil (k=3, s=1, p=1), the 2x2x2 stride-2
# downsampling and its transposed upsampling.  Build-defined like the rest of this module: the
# reference has no voxel grid, parity is against torch's conv3d / conv_transpose3d (fp64).
# Activations are [B, D, H, W, C] bf16 (channels innermost); parameters keep torch's layouts
# (Conv3d [Cout, Cin, k, k, k], ConvTranspose3d [Cin, Cout, k, k, k]) in fp32, cast to bf16 per
# call by pcs_cast_weight.
# ---------------------------------------------------------------------------------------------

def _out_size(d, k, s, p, transposed, op=0):
    return (d - 1) * s - 2 * p + k + op if transposed else (d + 2 * p - k) // s + 1


def _geom(B, grid_in, cin, cout, k, s, p, transposed, op=(0, 0, 0)):
    """Conv3dGeom of one call.  op = torch's output_padding (transposed form only, 0 <= op < s per
    dimension): the trailing output planes a strided convolution's floor division skips, which the
    input gradient of that convolution needs to cover its whole input grid."""
    op = (op,) * 3 if isinstance(op, int) else tuple(op)
    if any(o < 0 or o >= max(s, 1) for o in op) or (any(op) and not transposed):
        raise ValueError(f"output_padding {op} must satisfy 0 <= op < stride = {s} (transposed form only)")
    out = [_out_size(d, k, s, p, transposed, o) for d, o in zip(grid_in, op)]
    if min(out) <= 0:
        raise ValueError(f"empty output grid {out} for input {list(grid_in)}, k={k}, s={s}, p={p}")
    return L.Conv3dGeom(B=B, Di=grid_in[0], Hi=grid_in[1], Wi=grid_in[2], Do=out[0], Ho=out[1], Wo=out[2],
                        Cin=cin, Cout=cout, k=k, s=s, p=p, transposed=int(transposed))


def _bf16_2d(t, rows, cols):
    """bf16 copy of a [rows, cols] tensor on the device (pcs_cast_weight for fp32 input)."""
    t = t.contiguous()
    if t.dtype == torch.bfloat16:
        return t
    out = torch.empty(rows, cols, dtype=torch.bfloat16, device=t.device)
    L.call("pcs_cast_weight", L.ptr(t.float()), rows, cols, cols, L.BF16, L.ptr(out), None, L.stream_ptr(t.device))
    return out


CH_ALIGN = 64   # channel multiple of the sparse conv kernels' 64-wide tiles (sparse.py)
DENSE_CH_ALIGN = 32   # the dense conv3d kernels' tiles: 64 channels, or 32 for a 32-channel level


def _ceil(c, m=CH_ALIGN):
    return (c + m - 1) // m * m


def _pad_channels(t, c_to):
    """[..., C] -> [..., c_to] with zero channels appended (a device copy; no-op when C == c_to)."""
    if t.shape[-1] == c_to:
        return t.contiguous()
    out = t.new_zeros(*t.shape[:-1], c_to)
    out[..., : t.shape[-1]] = t
    return out


class _Conv3dFn(torch.autograd.Function):
    """y = conv(x, w) + b with w in kernel layout [Cout, taps * Cin] (fp32 master).

    Multiples of 32 run natively (a 32-channel U-Net level on 32-channel tiles); other channel
    counts (a first layer on raw point features) run on zero-padded channels: x and W^T get zero
    input channels, W and b zero output channels, and the padded output / gradient channels are
    sliced off.  Zero channels contribute exact zeros, so results equal the unpadded
    convolution's."""

    @staticmethod
    def forward(ctx, x, wk, bias, k, s, p, transposed, out_dtype, op):
        if not x.is_cuda:
            raise RuntimeError("pcs_amd conv3d runs on a HIP device only (no CPU fallback)")
        if x.dtype != torch.bfloat16 or x.dim() != 5:
            raise ValueError("x must be a bf16 [B, D, H, W, C] channels-last voxel grid")
        B, D, H, W, cin = x.shape
        cout, taps = wk.shape[0], k ** 3
        if wk.shape[1] != taps * cin:
            raise ValueError(f"weight has {wk.shape[1] // taps} input channels, x has {cin}")
        cin_k, cout_k = _ceil(cin, DENSE_CH_ALIGN), _ceil(cout, DENSE_CH_ALIGN)
        g = _geom(B, (D, H, W), cin_k, cout_k, k, s, p, transposed, op)
        xk = _pad_channels(x, cin_k)
        if (cin_k, cout_k) != (cin, cout):
            wp = wk.new_zeros(cout_k, taps, cin_k)
            wp[:cout, :, :cin] = wk.reshape(cout, taps, cin)
            wk = wp.reshape(cout_k, taps * cin_k)
        wb = _bf16_2d(wk, cout_k, taps * cin_k)
        bk = None
        if bias is not None:
            bk = bias.float().contiguous() if cout_k == cout else _pad_channels(bias.float(), cout_k)
        y = torch.empty(B, g.Do, g.Ho, g.Wo, cout_k, dtype=out_dtype, device=x.device)
        L.call("pcs_conv3d", ct.byref(g), L.ptr(xk), L.ptr(wb), L.ptr(bk) if bk is not None else None, L.ptr(y),
               L.BF16 if out_dtype == torch.bfloat16 else L.F32, L.stream_ptr(x.device))
        ctx.save_for_backward(xk, wb)
        ctx.cfg = (k, s, p, transposed, bias is not None, op, cin, cout)
        return y if cout_k == cout else y[..., :cout].contiguous()

    @staticmethod
    def backward(ctx, dy):
        xk, wb = ctx.saved_tensors
        k, s, p, transposed, has_bias, op, cin, cout = ctx.cfg
        B, D, H, W, cin_k = xk.shape
        cout_k = wb.shape[0]
        taps = k ** 3
        g = _geom(B, (D, H, W), cin_k, cout_k, k, s, p, transposed, op)
        M = B * g.Do * g.Ho * g.Wo
        dyb = _bf16_2d(_pad_channels(dy, cout_k).reshape(M, cout_k), M, cout_k)
        dev, st = xk.device, L.stream_ptr(xk.device)
        dx = dwk = db = None
        if ctx.needs_input_grad[0]:
            # the input gradient of a convolution is the transposed convolution of dy with W_t^T
            # (and vice versa): same k, s, p, grids swapped.  A strided convolution whose floor
            # division skipped trailing input planes gets them back as the transposed form's
            # output_padding; a transposed one's own output_padding planes are read as rows of dy.
            wt = torch.empty(cin_k, taps * cout_k, dtype=torch.bfloat16, device=dev)
            L.call("pcs_conv3d_weight_t", L.ptr(wb), cout_k, taps, cin_k, L.ptr(wt), st)
            back_op = (0, 0, 0)
            if not transposed:
                back_op = tuple(d - _out_size(o, k, s, p, True) for d, o in zip((D, H, W), (g.Do, g.Ho, g.Wo)))
            gb = _geom(B, (g.Do, g.Ho, g.Wo), cout_k, cin_k, k, s, p, not transposed, back_op)
            if (gb.Do, gb.Ho, gb.Wo) != (D, H, W):
                raise ValueError("input gradient: the strided output grid does not map back onto the input grid")
            dx = torch.empty_like(xk)
            L.call("pcs_conv3d", ct.byref(gb), L.ptr(dyb), L.ptr(wt), None, L.ptr(dx), L.BF16, st)
            if cin_k != cin:
                dx = dx[..., :cin].contiguous()
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            nbytes = L.load().pcs_conv3d_wgrad_workspace(ct.byref(g))
            if nbytes < 0:
                raise L.PcsError(L.load().pcs_last_error().decode())
            ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
            dwk = torch.empty(cout_k, taps * cin_k, dtype=torch.float32, device=dev)
            db = torch.empty(cout_k, dtype=torch.float32, device=dev) if has_bias else None
            L.call("pcs_conv3d_wgrad", ct.byref(g), L.ptr(xk), L.ptr(dyb), L.ptr(ws), nbytes, L.ptr(dwk), L.ptr(db), st)
            if (cin_k, cout_k) != (cin, cout):
                dwk = dwk.reshape(cout_k, taps, cin_k)[:cout, :, :cin].reshape(cout, taps * cin)
                db = db[:cout] if db is not None else None
        return dx, dwk, db, None, None, None, None, None, None


def conv3d(x, weight, bias=None, stride=1, padding=0, out_dtype=torch.bfloat16):
    """torch.nn.functional.conv3d on a channels-last bf16 grid x [B, D, H, W, Cin];
    weight [Cout, Cin, k, k, k] (torch layout, fp32), bias [Cout] or None."""
    cout, cin, k = weight.shape[0], weight.shape[1], weight.shape[2]
    wk = weight.permute(0, 2, 3, 4, 1).reshape(cout, k ** 3 * cin)
    return _Conv3dFn.apply(x, wk, bias, k, int(stride), int(padding), False, out_dtype, 0)


def conv_transpose3d(x, weight, bias=None, stride=2, padding=0, out_dtype=torch.bfloat16, output_padding=0):
    """torch.nn.functional.conv_transpose3d on a channels-last bf16 grid x [B, D, H, W, Cin];
    weight [Cin, Cout, k, k, k] (torch layout, fp32), bias [Cout] or None; output_padding as
    torch's (an int or 3 ints, each < stride)."""
    cin, cout, k = weight.shape[0], weight.shape[1], weight.shape[2]
    wk = weight.permute(1, 2, 3, 4, 0).reshape(cout, k ** 3 * cin)
    op = (int(output_padding),) * 3 if isinstance(output_padding, int) else tuple(int(o) for o in output_padding)
    return _Conv3dFn.apply(x, wk, bias, k, int(stride), int(padding), True, out_dtype, op)


class Conv3d(torch.nn.Module):
    """nn.Conv3d(cin, cout, k, stride, padding) with torch's parameter layout and init, on
    channels-last bf16 voxel grids (pcs_conv3d)."""

    def __init__(self, cin, cout, kernel_size=3, stride=1, padding=1, bias=True):
        super().__init__()
        ref = torch.nn.Conv3d(cin, cout, kernel_size, stride, padding, bias=bias)
        self.weight, self.bias = ref.weight, ref.bias
        self.stride, self.padding = stride, padding

    def forward(self, x, out_dtype=torch.bfloat16):
        return conv3d(x, self.weight, self.bias, self.stride, self.padding, out_dtype)


class ConvTranspose3d(torch.nn.Module):
    """nn.ConvTranspose3d(cin, cout, k, stride, padding) with torch's parameter layout and init,
    on channels-last bf16 voxel grids (pcs_conv3d, transposed form)."""

    def __init__(self, cin, cout, kernel_size=2, stride=2, padding=0, output_padding=0, bias=True):
        super().__init__()
        ref = torch.nn.ConvTranspose3d(cin, cout, kernel_size, stride, padding, output_padding, bias=bias)
        self.weight, self.bias = ref.weight, ref.bias
        self.stride, self.padding, self.output_padding = stride, padding, output_padding

    def forward(self, x, out_dtype=torch.bfloat16):
        return conv_transpose3d(x, self.weight, self.bias, self.stride, self.padding, out_dtype, self.output_padding)

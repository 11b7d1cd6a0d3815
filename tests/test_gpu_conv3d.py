"""Dense 3-D convolutions on channels-last voxel grids (csrc/conv3d.hip) against
torch's conv3d / conv_transpose3d in fp64 on the same bf16-rounded operands, through the C ABI.

Build-defined: the reference has no voxel grid, so this is not reference parity.  Products of
bf16 operands are exact in fp32, so the forward and the fp32 weight gradients match fp64 to fp32
summation error; the input gradient is stored in bf16.  Grids are ragged (odd, unequal sides)
so the stencil's borders, the stride lattice and the partial last tiles are all exercised."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ncdhw(x):            # [B, D, H, W, C] -> [B, C, D, H, W] fp64 on the host
    return x.permute(0, 4, 1, 2, 3).double().cpu()


def _rel(a, b):
    return float((a.double().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-30))


CASES = [
    # (k, s, p, transposed, grid, cin, cout)
    (3, 1, 1, False, (5, 6, 7), 64, 64),      # the U-Net stencil
    (3, 1, 1, False, (4, 3, 9), 32, 128),     # Cin = one k-step
    (2, 2, 0, False, (6, 4, 8), 64, 64),      # 2x2x2 stride-2 downsampling
    (3, 2, 1, False, (7, 5, 7), 64, 64),      # strided stencil, odd grid
    (2, 2, 0, True, (3, 2, 4), 64, 64),       # 2x2x2 stride-2 upsampling
    (3, 1, 1, True, (4, 5, 3), 64, 64),       # transposed stencil (= flipped convolution)
    (3, 2, 1, True, (3, 4, 2), 64, 128),      # strided transposed stencil
    (3, 2, 1, True, (1, 4, 2), 64, 64),       # output depth 1: two parity classes are empty
    (3, 2, 1, False, (6, 6, 8), 64, 64),      # strided stencil, even grid (input grad needs op = 1)
    (2, 2, 0, False, (7, 5, 7), 64, 128),     # 2x2x2 down on an odd grid (skipped last plane)
    (3, 2, 1, True, (3, 4, 2), 64, 64, 1),    # transposed with output_padding 1
    (2, 2, 0, True, (3, 2, 4), 64, 64, (1, 0, 1)),   # 2x2x2 up with per-dimension output_padding
    (3, 1, 1, False, (4, 3, 5), 32, 64),      # the U-Net's 32 -> 64 step (32-channel halo slices)
    (3, 1, 1, False, (5, 4, 3), 4, 32),       # raw point features in (padded to 32), 32 channels out
    (2, 2, 0, True, (2, 3, 2), 64, 32),       # transposed up to a 32-channel level
    (3, 1, 1, False, (5, 6, 7), 32, 32),      # the 32-channel level's own stencil (32 x 32 tiles)
    (3, 1, 1, True, (4, 5, 3), 64, 32),       # transposed stencil, 64-channel slices into 32-channel tiles
    (2, 2, 0, False, (6, 4, 7), 32, 64),      # 2x2x2 down from the 32-channel level (gather, 32-deep k-steps)
    (3, 2, 1, False, (7, 5, 7), 32, 32),      # strided gather on 32-channel tiles both ways
    (1, 1, 0, False, (3, 5, 4), 96, 32),      # 1x1x1 channel mix, three 32-channel slices in
    (3, 1, 1, False, (3, 4, 5), 96, 96),      # odd multiples of 32 both ways (three tiles each)
]


def _case(c):
    return c if len(c) == 8 else c + (0,)


def _operands(k, transposed, grid, cin, cout, B=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, *grid, cin, generator=g).to(torch.bfloat16)
    shape = (cin, cout, k, k, k) if transposed else (cout, cin, k, k, k)
    w = (torch.randn(*shape, generator=g) * 0.05).to(torch.bfloat16).float()   # bf16-exact fp32 master
    b = torch.randn(cout, generator=g) * 0.1
    return x, w, b


def _ref_fn(transposed, op):
    if transposed:
        return lambda *a, **kw: F.conv_transpose3d(*a, output_padding=op, **kw)
    return F.conv3d


def _fn(V, transposed, op):
    if transposed:
        return lambda *a, **kw: V.conv_transpose3d(*a, output_padding=op, **kw)
    return V.conv3d


def _ref(x, w, b, s, p, transposed, op=0):
    return _ref_fn(transposed, op)(_ncdhw(x), w.double(), b.double(), stride=s, padding=p).permute(0, 2, 3, 4, 1)


@pytest.mark.parametrize("k,s,p,transposed,grid,cin,cout,op", [_case(c) for c in CASES])
def test_forward_matches_torch(k, s, p, transposed, grid, cin, cout, op):
    import pcs_amd.voxel as V
    x, w, b = _operands(k, transposed, grid, cin, cout)
    ref = _ref(x, w, b, s, p, transposed, op)
    f = _fn(V, transposed, op)
    y = f(x.to(DEV), w.to(DEV), b.to(DEV), s, p, out_dtype=torch.float32)
    yb = f(x.to(DEV), w.to(DEV), b.to(DEV), s, p, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert tuple(y.shape) == tuple(ref.shape)
    assert _rel(y, ref) < 1e-5
    assert _rel(yb.float(), ref) < 8e-3           # one bf16 rounding of the stored output


@pytest.mark.parametrize("k,s,p,transposed,grid,cin,cout", [(3, 1, 1, False, (41, 40, 40), 64, 128),
                                                            (2, 2, 0, True, (32, 32, 32), 64, 128)])
def test_forward_large_tiles(k, s, p, transposed, grid, cin, cout):
    """Grids large enough for the 128-voxel tiles (pcs_conv3d switches at 2048 tiles), against
    torch fp32 on the host (its own rounding is ~1e-6 of the output scale)."""
    import pcs_amd.voxel as V
    x, w, b = _operands(k, transposed, grid, cin, cout, seed=3)
    f_ref = F.conv_transpose3d if transposed else F.conv3d
    ref = f_ref(x.permute(0, 4, 1, 2, 3).float(), w, b, stride=s, padding=p).permute(0, 2, 3, 4, 1).double()
    f = V.conv_transpose3d if transposed else V.conv3d
    y = f(x.to(DEV), w.to(DEV), b.to(DEV), s, p, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert _rel(y, ref) < 2e-5


@pytest.mark.parametrize("k,s,p,transposed,grid,cin,cout,op", [_case(c) for c in CASES])
def test_backward_matches_torch(k, s, p, transposed, grid, cin, cout, op):
    """Every case, including even grids under a stride (the input gradient's output_padding),
    odd grids under the 2x2x2 down layer, odd multiples of 32 (32-channel tiles) and counts off
    the 32 multiple (padded)."""
    import pcs_amd.voxel as V
    x, w, b = _operands(k, transposed, grid, cin, cout, seed=1)
    xr = _ncdhw(x).requires_grad_()
    wr, br = w.double().requires_grad_(), b.double().requires_grad_()
    yr = _ref_fn(transposed, op)(xr, wr, br, stride=s, padding=p)
    g = torch.Generator().manual_seed(2)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64).to(torch.bfloat16).double()   # bf16-exact
    yr.backward(dy)
    xd = x.to(DEV).requires_grad_()
    wd, bd = w.to(DEV).requires_grad_(), b.to(DEV).requires_grad_()
    f = _fn(V, transposed, op)
    y = f(xd, wd, bd, s, p, out_dtype=torch.float32)
    assert tuple(y.shape) == (yr.shape[0],) + tuple(yr.shape[2:]) + (yr.shape[1],)
    y.backward(dy.permute(0, 2, 3, 4, 1).float().to(DEV))
    torch.cuda.synchronize()
    assert _rel(wd.grad, wr.grad) < 1e-5
    assert _rel(bd.grad, br.grad) < 1e-5
    assert _rel(xd.grad.float().permute(0, 4, 1, 2, 3), xr.grad) < 8e-3      # dx stored in bf16


def test_wgrad_deterministic_and_validated():
    import ctypes as ct
    import pcs_amd._lib as L
    import pcs_amd.voxel as V
    x, w, _ = _operands(3, False, (9, 8, 7), 64, 64, B=3, seed=5)
    g = V._geom(3, (9, 8, 7), 64, 64, 3, 1, 1, False)
    dy = torch.randn(3, 9, 8, 7, 64).to(torch.bfloat16).to(DEV)
    xd = x.to(DEV)
    nb = L.load().pcs_conv3d_wgrad_workspace(ct.byref(g))
    outs = []
    for _ in range(2):
        ws = torch.full((nb // 4,), float("nan"), device=DEV)
        dw = torch.empty(64, 27 * 64, device=DEV)
        db = torch.empty(64, device=DEV)
        L.call("pcs_conv3d_wgrad", ct.byref(g), L.ptr(xd), L.ptr(dy), L.ptr(ws), nb, L.ptr(dw), L.ptr(db),
               L.stream_ptr())
        outs.append((dw, db))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = dy.double().reshape(-1, 64).sum(0).cpu()
    assert _rel(outs[0][1], ref) < 1e-5
    bad = V._geom(3, (9, 8, 7), 48, 64, 3, 1, 1, False)
    with pytest.raises(L.PcsError):
        L.call("pcs_conv3d_wgrad", ct.byref(bad), L.ptr(xd), L.ptr(dy), L.ptr(ws), nb, L.ptr(dw), None, L.stream_ptr())


def test_unet_block_trains():
    """A two-level channels-last U-Net block (stencil, 2x2x2 down, stencil, transposed up, skip
    add, stencil) built from the modules: finite gradients and a falling loss over a few SGD steps."""
    import pcs_amd.voxel as V
    torch.manual_seed(0)
    enc = V.Conv3d(64, 64).to(DEV)
    down = V.Conv3d(64, 128, 2, 2, 0).to(DEV)
    mid = V.Conv3d(128, 128).to(DEV)
    up = V.ConvTranspose3d(128, 64, 2, 2, 0).to(DEV)
    head = V.Conv3d(64, 64).to(DEV)
    params = [p for m in (enc, down, mid, up, head) for p in m.parameters()]
    opt = torch.optim.SGD(params, lr=0.05)
    x = torch.randn(2, 8, 8, 8, 64, device=DEV).to(torch.bfloat16)
    target = torch.randn(2, 8, 8, 8, 64, device=DEV) * 0.1
    losses = []
    for _ in range(8):
        e = enc(x)
        u = up(mid(down(e)))
        y = head((e.float() + u.float()).to(torch.bfloat16), out_dtype=torch.float32)
        loss = ((y - target) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        assert all(torch.isfinite(p.grad).all() for p in params)
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0]

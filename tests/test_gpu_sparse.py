"""Occupied-voxel (sparse) path on MI355X (csrc/sparse.hip, the sparse kernels of csrc/conv3d.hip):
the hash table, the voxel keys and the 27-neighbour map bit-exact against oracle/sparse_oracle.py;
the submanifold 3x3x3 convolution, forward and backward, against torch's dense conv3d in fp64 on a
grid that is zero off the occupied voxels, read back at the occupied voxels.  Build-defined: the
reference has no voxel grid, so none of this is reference parity."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import sparse_oracle as so
import voxel_oracle as vo

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
BOX = ((-1.0, -1.0, -1.0), (1.0, 1.0, 1.0))


def _batch(seed, n_scenes, grid, occupancy, per_voxel=2):
    from pcs_amd.data import jittered_clouds, ragged_collate
    clouds = jittered_clouds(seed, n_scenes, grid=grid, occupancy=occupancy, per_voxel=per_voxel)
    return ragged_collate([(torch.from_numpy(p), torch.from_numpy(l)) for p, l in clouds])


def _sparse(rb, grid):
    from pcs_amd.sparse import sparse_voxels
    from pcs_amd.voxel import voxelize
    vb = voxelize(rb, grid, *BOX)
    return vb, sparse_voxels(rb, vb, *BOX)


def _oracle_keys(rb, grid):
    pts, off = rb.points.numpy(), rb.offsets.numpy()
    ids = vo.voxel_ids(pts, grid, *BOX).astype(np.int64)
    scene = np.searchsorted(off, np.arange(len(pts)), side="right") - 1
    return np.unique(scene * grid ** 3 + ids)


def test_hash_table_lookups():
    from pcs_amd.sparse import sparse_from_keys
    rng = np.random.default_rng(3)
    keys = np.unique(rng.integers(0, 1 << 40, size=20000))
    sv = sparse_from_keys(torch.from_numpy(keys).to(DEV), grid=1 << 13)
    got = sv.find(torch.from_numpy(keys).to(DEV)).cpu().numpy()
    assert np.array_equal(got, np.arange(len(keys), dtype=np.int32))
    absent = np.setdiff1d(rng.integers(0, 1 << 40, size=5000), keys)
    assert (sv.find(torch.from_numpy(absent).to(DEV)).cpu().numpy() == -1).all()
    # the table holds every key exactly once, the rest of the slots empty
    tk = sv.table_keys.cpu().numpy()
    assert np.array_equal(np.sort(tk[tk != -1]), keys) and sv.table_keys.numel() >= 2 * len(keys)


@pytest.mark.parametrize("grid,occupancy", [(16, 0.3), (32, 0.05), (64, 0.01)])
def test_keys_and_neighbours_bit_exact(grid, occupancy):
    rb = _batch(11 + grid, 3, grid, occupancy)
    vb, sv = _sparse(rb, grid)
    keys = sv.keys.cpu().numpy()
    assert np.array_equal(keys, _oracle_keys(rb, grid))           # one key per voxel, voxel order
    nbr = sv.nbr.cpu().numpy()
    assert np.array_equal(nbr, so.neighbors(keys, grid))
    assert (nbr[:, 13] == np.arange(len(keys))).all()              # the centre tap is the voxel itself


def _dense(x, keys, grid, B):
    """[V, C] features -> fp64 dense [B, C, G, G, G] (zeros off the occupied voxels)."""
    s, ix, iy, iz = so.decode(keys, grid)
    d = torch.zeros(B, x.shape[1], grid, grid, grid, dtype=torch.float64)
    d[s, :, ix, iy, iz] = x.double().cpu()
    return d, (s, ix, iy, iz)


@pytest.fixture(params=["gather", "pairs", "default"])
def conv_path(request, monkeypatch):
    """Both forms of the submanifold convolution: the tile-gather kernel and the per-tap pair lists
    (sparse.PAIR_TAPS_MAX picks between them by occupied taps per voxel), and the module's own mix
    (the weight gradient always on the pair lists)."""
    import pcs_amd.sparse as S
    if request.param != "default":
        monkeypatch.setattr(S, "PAIR_TAPS_MAX", 0.0 if request.param == "gather" else 27.0)
        monkeypatch.setattr(S, "PAIR_WGRAD", request.param == "pairs")
    return request.param


@pytest.mark.parametrize("grid,occupancy,cin,cout", [(16, 0.3, 64, 64), (32, 0.05, 64, 128),
                                                    (16, 0.2, 4, 32), (24, 0.1, 32, 64)])
def test_submanifold_conv_matches_dense_conv3d(grid, occupancy, cin, cout, conv_path):
    from pcs_amd.sparse import submanifold_conv3d
    rb = _batch(5 + cin + grid, 2, grid, occupancy)
    _, sv = _sparse(rb, grid)
    V = sv.num_voxels
    keys = sv.keys.cpu().numpy()
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn(V, cin, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, 3, generator=g) * 0.05).to(torch.bfloat16).float()   # bf16-exact
    b = torch.randn(cout, generator=g) * 0.1
    dy = torch.randn(V, cout, generator=g).to(torch.bfloat16)
    # dense reference in fp64 (outputs read at the occupied voxels; dy scattered the same way)
    xd, idx = _dense(x, keys, grid, 2)
    xd.requires_grad_()
    wr, br = w.double().requires_grad_(), b.double().requires_grad_()
    yd = F.conv3d(xd, wr, br, padding=1)
    ref = yd[idx[0], :, idx[1], idx[2], idx[3]]
    ref.backward(dy.double())
    # device
    xs = x.to(DEV).requires_grad_()
    ws, bs = w.to(DEV).requires_grad_(), b.to(DEV).requires_grad_()
    y = submanifold_conv3d(xs, ws, sv, bs, out_dtype=torch.float32)
    y.backward(dy.float().to(DEV))
    torch.cuda.synchronize()
    rel = lambda a, r: float((a.double().cpu() - r).abs().max() / r.abs().max().clamp_min(1e-30))  # noqa: E731
    assert rel(y, ref.detach()) < 1e-5
    assert rel(ws.grad, wr.grad) < 1e-5
    assert rel(bs.grad, br.grad) < 1e-5
    assert rel(xs.grad.float(), xd.grad[idx[0], :, idx[1], idx[2], idx[3]]) < 8e-3   # dx stored in bf16
    # and the numpy restatement on the neighbour map
    assert rel(y, torch.from_numpy(so.submanifold_conv(x.double().numpy(), w.numpy(), b.numpy(),
                                                       sv.nbr.cpu().numpy()))) < 1e-5
    if conv_path != "default":
        assert sv.use_pairs() == (conv_path == "pairs")


def test_pair_lists_match_the_neighbour_map():
    """Per-tap pair lists: tap t's pairs are exactly the rows m with nbr[m][t] >= 0, ascending,
    pair_in = nbr[pair_out][t], and pair_pos indexes them back (-1 elsewhere); the same lists on a
    rebuild (deterministic)."""
    from pcs_amd.sparse import TAPS, sparse_from_keys
    rb = _batch(3, 3, 20, 0.07)
    _, sv = _sparse(rb, 20)
    pin, pout, ppos, tap_off, P = sv.pairs()
    nbr = sv.nbr.cpu().numpy()
    pin, pout, ppos = pin.cpu().numpy()[:P], pout.cpu().numpy()[:P], ppos.cpu().numpy()
    assert P == int((nbr >= 0).sum())
    for t in range(TAPS):
        rows = np.nonzero(nbr[:, t] >= 0)[0]
        a, b = tap_off[t], tap_off[t + 1]
        assert np.array_equal(pout[a:b], rows)
        assert np.array_equal(pin[a:b], nbr[rows, t])
        assert np.array_equal(ppos[rows, t], np.arange(a, b))
    assert (ppos[nbr < 0] == -1).all()
    sv2 = sparse_from_keys(sv.keys, 20)
    assert all(torch.equal(u[:P].cpu(), v[:P].cpu()) for u, v in zip(sv.pairs()[:3], sv2.pairs()[:3]))


def test_isolated_voxels_run_only_the_centre_tap(conv_path):
    """Voxels with no occupied neighbour: every tile's tap mask is the centre tap alone, and the
    output is the 1x1 channel mix of the centre weight."""
    from pcs_amd.sparse import sparse_from_keys, submanifold_conv3d
    G = 64
    c = np.arange(0, G, 3)
    ix, iy, iz = np.meshgrid(c, c, c, indexing="ij")
    keys = np.sort(((ix * G + iy) * G + iz).reshape(-1)).astype(np.int64)
    sv = sparse_from_keys(torch.from_numpy(keys).to(DEV), G)
    assert (sv.nbr[:, 13].cpu().numpy() == np.arange(len(keys))).all()
    assert int((sv.nbr >= 0).sum()) == len(keys)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(len(keys), 64, generator=g).to(torch.bfloat16)
    w = (torch.randn(64, 64, 3, 3, 3, generator=g) * 0.05).to(torch.bfloat16).float()
    y = submanifold_conv3d(x.to(DEV), w.to(DEV), sv, None, out_dtype=torch.float32).cpu().double()
    ref = x.double() @ w[:, :, 1, 1, 1].double().T
    assert float((y - ref).abs().max() / ref.abs().max()) < 1e-5


def test_sparse_block_trains():
    """Two submanifold layers (module API) with a ReLU between: finite gradients, falling loss."""
    from pcs_amd.sparse import SubMConv3d
    torch.manual_seed(0)
    rb = _batch(21, 2, 24, 0.15)
    _, sv = _sparse(rb, 24)
    l1, l2 = SubMConv3d(4, 64).to(DEV), SubMConv3d(64, 32).to(DEV)
    params = list(l1.parameters()) + list(l2.parameters())
    opt = torch.optim.SGD(params, lr=0.05)
    x = torch.randn(sv.num_voxels, 4, device=DEV).to(torch.bfloat16)
    target = torch.randn(sv.num_voxels, 32, device=DEV) * 0.1
    losses = []
    for _ in range(8):
        h = torch.relu(l1(x, sv, out_dtype=torch.float32)).to(torch.bfloat16)
        y = l2(h, sv, out_dtype=torch.float32)
        loss = ((y - target) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        assert all(torch.isfinite(p.grad).all() for p in params)
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]

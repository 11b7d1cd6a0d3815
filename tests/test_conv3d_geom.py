"""Host-side geometry of the channels-last conv3d layer (pcs_amd.voxel): output
grids, torch's output_padding rule, the input gradient's grid (which must map back onto the
forward's input grid for every stride / parity combination), and early rejection.  CPU only:
no kernel runs here (tests/test_gpu_conv3d.py runs them against torch fp64)."""
import itertools

import pytest
import torch


def _torch_out(d, k, s, p, transposed, op=0):
    """Output side of torch's own module on a 1 x 1 x d x 1 x 1 probe (the authority)."""
    if transposed:
        m = torch.nn.ConvTranspose3d(1, 1, k, s, p, output_padding=op, bias=False)
    else:
        m = torch.nn.Conv3d(1, 1, k, s, p, bias=False)
    with torch.no_grad():
        return m(torch.zeros(1, 1, d, 1 + 2 * p + k, 1 + 2 * p + k)).shape[2]


@pytest.mark.parametrize("k,s,p", [(3, 1, 1), (3, 2, 1), (2, 2, 0), (1, 1, 0), (3, 2, 0)])
def test_output_grid_matches_torch(k, s, p):
    import pcs_amd.voxel as V
    for d in range(max(1, k - 2 * p), 12):
        g = V._geom(1, (d, d, d), 64, 64, k, s, p, False)
        assert g.Do == _torch_out(d, k, s, p, False)
        for op in range(s):
            gt = V._geom(1, (d, d, d), 64, 64, k, s, p, True, op)
            assert gt.Do == _torch_out(d, k, s, p, True, op)


@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (2, 2, 0), (3, 1, 1), (3, 2, 0)])
def test_input_gradient_grid_covers_the_input(k, s, p):
    """The backward's transposed pass gets output_padding = D - (Do - 1) s + 2p - k, always in
    [0, s): even grids under (3, 2, 1) and odd grids under (2, 2, 0) included."""
    import pcs_amd.voxel as V
    for dims in itertools.product(range(max(1, k - 2 * p), 10), repeat=1):
        d = dims[0]
        g = V._geom(2, (d, d + 1, d + 2), 64, 64, k, s, p, False)
        back = tuple(D - V._out_size(o, k, s, p, True) for D, o in zip((d, d + 1, d + 2), (g.Do, g.Ho, g.Wo)))
        assert all(0 <= b < s for b in back), (d, back)
        gb = V._geom(2, (g.Do, g.Ho, g.Wo), 64, 64, k, s, p, True, back)
        assert (gb.Do, gb.Ho, gb.Wo) == (d, d + 1, d + 2)


def test_bad_output_padding_is_rejected_up_front():
    import pcs_amd.voxel as V
    with pytest.raises(ValueError):
        V._geom(1, (4, 4, 4), 64, 64, 2, 2, 0, True, 2)        # op >= stride
    with pytest.raises(ValueError):
        V._geom(1, (4, 4, 4), 64, 64, 3, 1, 1, True, 1)        # stride 1: op must be 0
    with pytest.raises(ValueError):
        V._geom(1, (4, 4, 4), 64, 64, 3, 2, 1, False, 1)       # only the transposed form takes op
    with pytest.raises(ValueError):
        V._geom(1, (1, 4, 4), 64, 64, 3, 1, 0, False)          # empty output grid


def test_channel_padding_rule():
    import pcs_amd.voxel as V
    assert [V._ceil(c) for c in (1, 4, 32, 63, 64, 65, 128)] == [64, 64, 64, 64, 64, 128, 128]
    t = torch.arange(6, dtype=torch.float32).reshape(1, 2, 3)
    pt = V._pad_channels(t, 64)
    assert pt.shape == (1, 2, 64) and torch.equal(pt[..., :3], t) and not pt[..., 3:].any()
    assert V._pad_channels(t, 3).data_ptr() == t.data_ptr()

"""The bf16-storage emulation (oracle/bf16_emulation.py) used to judge the bf16 path: with no
rounding it must be the reference step itself (vs the fp64 oracle), and its bf16 rounding
must be round-to-nearest-even."""
import numpy as np

import bf16_emulation as emu
import pointnet_oracle as orc
from golden_util import inputs, load


def test_round_bf16_nearest_even():
    x = np.array([1.0, 1.00390625, 1.01171875, -3.0e-3, 65504.0, 0.0], np.float32)
    r = emu.round_bf16(x)
    # 1 + 2^-8 is a tie between 1 and 1 + 2^-7: even mantissa -> 1; 1 + 3*2^-8 -> 1 + 2^-6
    assert r[0] == 1.0 and r[1] == 1.0 and r[2] == np.float32(1.015625)
    u = r.view(np.uint32)
    assert np.all(u & 0xFFFF == 0)
    assert np.abs(r - x).max() <= np.abs(x).max() * 2.0 ** -9


def test_fp32_mode_is_the_reference_step():
    g = load("train_c3_ragged_bnrand")
    sd, pts, lab, msk, masks = inputs(g)
    l64, _, g64, _ = orc.train_step(sd, pts, lab, g["weight"], masks=masks)
    l32, g32 = emu.train_step(sd, pts, lab, g["weight"], masks, store="fp32")
    assert abs(l32 - l64) < 1e-5 * abs(l64)
    gmax = max(np.linalg.norm(v) for v in g64.values())
    for n, v in g64.items():
        if n.endswith(".bias") and not n.startswith(("bn", "seg_conv4")):
            continue   # BN-cancelled conv biases: the emulation returns their analytic 0
        if n == "bn_global.bias":
            continue
        err = np.linalg.norm(g32[n].ravel() - v.ravel()) / max(np.linalg.norm(v), 1e-3 * gmax)
        assert err < 5e-3, (n, err)


def test_e4m3_rounding_matches_torch():
    """round_e4m3 / quant_rows_e4m3 (the fp8 storage emulation) against torch's
    float8_e4m3fn cast, bit for bit, over normal and subnormal binades."""
    import torch
    from bf16_emulation import quant_rows_e4m3, round_e4m3
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(100000) * np.exp2(rng.integers(-14, 9, 100000))).astype(np.float32)
    x = np.clip(x, -448, 448)
    ref = torch.from_numpy(x).to(torch.float8_e4m3fn).float().numpy()
    assert np.array_equal(round_e4m3(x), ref)
    W = (rng.standard_normal((32, 100)) * 0.02).astype(np.float32)
    mx = np.abs(W).max(1)
    e = np.ceil(np.log2(mx / 448.0))
    ref = torch.from_numpy(W * np.exp2(-e)[:, None].astype(np.float32)).to(torch.float8_e4m3fn).double().numpy()
    assert np.array_equal(quant_rows_e4m3(W), (ref * np.exp2(e)[:, None]).astype(np.float32))


def test_eval_logits_without_rounding_is_the_reference_eval():
    """eval_logits with no rounding site is the reference's eval forward (P:98-133 under
    model.eval()): the reference-written eval fixture's logits and the fp64 oracle."""
    g = load("eval_c2_bnrand")
    sd, pts, _, _, _ = inputs(g)
    l64, _ = orc.forward(sd, pts, train=False)
    l32 = emu.eval_logits(sd, pts, frozenset())
    scale = np.abs(l64).max()
    assert np.abs(l32 - l64).max() <= 1e-4 * scale
    assert np.abs(l32 - np.asarray(g["logits"])).max() <= 1e-4 * scale
    # the site sets: the fp32 trunk drops exactly conv1..conv4's sites, bf16 storage is lossy
    b, f = emu.eval_sites("bf16"), emu.eval_sites("fp32")
    assert b - f == {f"{k}conv{i}" for k in "YA" for i in (1, 2, 3, 4)} | {"Wconv2", "Wconv3", "Wconv4"}
    assert f - b == {"Asplit4"}   # conv5 fed pcs_bnrelu_bf16's [hi | lo] of a4
    a = np.random.default_rng(0).standard_normal(4096).astype(np.float32)
    hi = emu.round_bf16(a)
    lo = emu.round_bf16(a - hi)
    assert np.all(np.abs(a - (hi + lo)) <= np.abs(a) * 2.0 ** -16) and np.any(hi + lo != a)
    lb = emu.eval_logits(sd, pts, b)
    assert 0 < np.abs(lb - l64).max() <= 0.1 * scale

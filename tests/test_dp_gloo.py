"""Data-parallel path (SURVEY §8 e) on CPU: world_size-2 ``gloo`` process groups.

The reference trains with ``nn.DataParallel`` (P:208-211): the padded batch is chunked over
replicas, each replica normalises with its own BatchNorm batch statistics, ONE loss is
taken over the gathered outputs (P:251), replica gradients are summed into the base module,
and replica 0 shares the base module's running buffers.  ``tests/golden/train_c3_dp2.npz``
records exactly that, computed by the reference module itself (make_golden.make_dp_case).

``pcs_amd.FusedTrainStep`` implements it as one process per GPU: each rank runs its own
scenes and computes its un-normalised gradient; the flat gradient buffer (engine.flat_layout
order, with the loss numerator and CE weight sum in its tail) is summed in the three
``engine.bucket_ranges`` buckets by ``train.GradientBuckets``, then scaled by 1 / the global
weight sum.  Here the per-rank compute is the oracle (fp64) and the buckets / collectives are
the product's own over gloo.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pointnet_oracle as orc
from golden_util import assert_train_matches, inputs, load, rel_err
from pcs_amd.data import shard_batch, shard_bounds

CASE = "train_c3_dp2"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_share(g, rank, world, denom=None):
    """Oracle compute of one replica: its scenes, its dropout rows, optional global denom."""
    sd, pts, lab, msk, masks = inputs(g)
    B, N = pts.shape[:2]
    lo, hi = shard_bounds(B, rank, world)
    rows = slice(lo * N, hi * N)
    w = g["weight"]
    if denom is None:
        return orc.ce_weight_sum(lab[lo:hi], w)
    return orc.train_step(sd, pts[lo:hi], lab[lo:hi], w, masks=(masks[0][rows], masks[1][rows]),
                          denom=denom)


def _dp_worker(rank, world, port, out):
    from pcs_amd.engine import bucket_ranges, flat_layout
    from pcs_amd.train import GradientBuckets
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        g = load(CASE)
        C = int(g["C"])
        wloc = _rank_share(g, rank, world)
        # un-normalised share (denominator 1): the loss is linear in 1 / sum_w
        loss, logits, grads, cache = _rank_share(g, rank, world, denom=1.0)
        names = [n for n, _ in flat_layout(C)]
        gflat = torch.from_numpy(np.concatenate([grads[n].reshape(-1) for n in names]
                                                + [np.array([loss, wloc, 0.0, 0.0])]))
        b = GradientBuckets(gflat, bucket_ranges(C))
        for name in ("seg", "global", "tail"):   # the order the backward finishes them
            b.issue(name)
        b.wait()
        nparam = gflat.numel() - 4
        wsum = float(gflat[nparam + 1])
        grads_flat = gflat[:nparam] / wsum
        sd = inputs(g)[0]
        run = orc.update_running_stats(sd, cache)
        np.savez(os.path.join(out, f"rank{rank}.npz"), gflat=grads_flat.numpy(),
                 loss=float(gflat[nparam] / wsum), logits=logits,
                 **{f"buf/{k}": np.asarray(v) for k, v in run.items()
                    if "running" in k or "num_batches" in k})
    finally:
        dist.destroy_process_group()


def _unflatten(g, flat):
    from pcs_amd.engine import flat_layout
    sd = inputs(g)[0]
    out, o = {}, 0
    for n, _ in flat_layout(int(g["C"])):
        k = sd[n].size
        out[n] = flat[o:o + k].reshape(sd[n].shape)
        o += k
    assert o == flat.size
    return out


def test_bucket_ranges_cover_the_flat_buffer():
    from pcs_amd.engine import FLAT_EXTRA, bucket_ranges, flat_offsets, param_layout
    for C, D in ((2, 4), (3, 4), (20, 3)):
        offs, total = flat_offsets(C, D)
        assert sorted(offs) == sorted(n for n, _ in param_layout(C, D))
        r = sorted(bucket_ranges(C, D).values())
        assert r[0][0] == 0 and r[-1][1] == total + FLAT_EXTRA
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        # seg_conv4's weight and bias are adjacent (the head writes them as one block)
        assert offs["seg_conv4.bias"] == offs["seg_conv4.weight"] + C * 128


@pytest.mark.parametrize("B", [1, 2, 3, 4, 5, 7, 8])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_bounds_follow_tensor_chunk(B, world):
    t = torch.arange(B)
    chunks = list(t.chunk(world))
    for r in range(world):
        (mine,) = shard_batch([t], r, world)
        ref = chunks[r] if r < len(chunks) else t[:0]
        assert torch.equal(mine, ref)


def test_oracle_dataparallel_matches_reference():
    """Single process: summing the oracle's replica shares reproduces the reference's
    DataParallel step (loss, grads, replica-0 running stats, Adam)."""
    g = load(CASE)
    world = int(g["world"])
    denom = sum(_rank_share(g, r, world) for r in range(world))
    shares = [_rank_share(g, r, world, denom=denom) for r in range(world)]
    loss = sum(s[0] for s in shares)
    names = [str(n) for n in g["param_names"]]
    grads = {n: sum(s[2][n] for s in shares) for n in names}
    assert rel_err(np.concatenate([s[1] for s in shares], 0), g["logits"]) < 2e-5
    sd = inputs(g)[0]
    assert_train_matches(g, sd, loss, grads, orc.update_running_stats(sd, shares[0][3]))
    # and it is NOT the single-replica (full-batch BN) step: DP semantics matter here
    _, _, full, _ = orc.train_step(sd, *inputs(g)[1:3], g["weight"], masks=inputs(g)[4])
    n = "conv1.weight"
    assert np.abs(full[n] - grads[n]).max() > 1e-3 * np.abs(grads[n]).max()


def test_gloo_world2_dataparallel_step():
    """Two gloo ranks, the product's collective helpers: every rank ends with the
    reference's DataParallel gradient; rank 0 holds replica 0's running stats."""
    g = load(CASE)
    world = int(g["world"])
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_dp_worker, args=(world, _free_port(), out), nprocs=world,
                           join=True, start_method="spawn")
        res = [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(world)]
    np.testing.assert_array_equal(res[0]["gflat"], res[1]["gflat"])
    assert res[0]["loss"] == res[1]["loss"]
    sd = inputs(g)[0]
    run = {k[4:]: v for k, v in res[0].items() if k.startswith("buf/")}
    assert_train_matches(g, sd, float(res[0]["loss"]), _unflatten(g, res[0]["gflat"]), run)
    B, N = inputs(g)[1].shape[:2]
    lo, hi = shard_bounds(B, 1, world)
    assert rel_err(res[1]["logits"], g["logits"][lo:hi]) < 2e-5

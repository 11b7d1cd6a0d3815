"""Data-parallel training step on the device: two ranks of ``pcs_amd.FusedTrainStep`` (gloo
process group, both ranks on cuda:0 — a 1-GPU box cannot run two RCCL ranks) against the
reference's nn.DataParallel step (tests/golden/train_c3_dp2.npz, P:208-211) and the
oracle's replica shares.  Tolerances are those of test_gpu_parity's fp32 fused step."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pointnet_oracle as orc
from golden_util import inputs, load
from pcs_amd.data import shard_bounds

pytestmark = pytest.mark.gpu
CASE = "train_c3_dp2"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    from pcs_amd.model import PointNetSegmentation
    from pcs_amd.optim import FusedAdam
    from pcs_amd.train import FusedTrainStep
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        g = load(CASE)
        sd, pts, lab, msk, masks = inputs(g)
        B, N = pts.shape[:2]
        lo, hi = shard_bounds(B, rank, world)
        rows = slice(lo * N, hi * N)
        m = PointNetSegmentation(int(g["C"])).to(dev)
        m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
        step = FusedTrainStep(m, FusedAdam(m, lr=1e-3, weight_decay=1e-4),
                              class_weight=g["weight"])
        bits = tuple(torch.from_numpy(np.packbits(mk[rows], axis=1, bitorder="little")).to(dev)
                     for mk in masks)
        loss = step(torch.from_numpy(pts[lo:hi]).to(dev), torch.from_numpy(lab[lo:hi]).to(dev),
                    masks=bits)
        torch.cuda.synchronize()
        res = {"loss": float(loss.item())}
        for n, p in m.named_parameters():
            res[f"g/{n}"] = p.grad.detach().cpu().numpy()
            res[f"p/{n}"] = p.detach().cpu().numpy()
        for k, v in m.state_dict().items():
            if "running" in k:
                res[f"buf/{k}"] = v.cpu().numpy()
        np.savez(os.path.join(out, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


def test_fused_train_step_dp2_matches_dataparallel():
    g = load(CASE)
    world = int(g["world"])
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                           start_method="spawn")
        res = [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(world)]
    names = [str(n) for n in g["param_names"]]
    # every rank holds the same gradient, loss and updated weights
    for n in names:
        np.testing.assert_array_equal(res[0][f"g/{n}"], res[1][f"g/{n}"], err_msg=n)
        np.testing.assert_array_equal(res[0][f"p/{n}"], res[1][f"p/{n}"], err_msg=n)
    assert abs(res[0]["loss"] - float(g["loss"])) < 1e-5 * max(1.0, abs(float(g["loss"])))
    # gradient == sum of the oracle's replica shares (global CE denominator, per-replica BN)
    sd, pts, lab, msk, masks = inputs(g)
    B, N = pts.shape[:2]
    denom = sum(orc.ce_weight_sum(lab[slice(*shard_bounds(B, r, world))], g["weight"])
                for r in range(world))
    grads = {n: 0.0 for n in names}
    for r in range(world):
        lo, hi = shard_bounds(B, r, world)
        rows = slice(lo * N, hi * N)
        _, _, gr, _ = orc.train_step(sd, pts[lo:hi], lab[lo:hi], g["weight"],
                                     masks=(masks[0][rows], masks[1][rows]), denom=denom)
        for n in names:
            grads[n] = grads[n] + gr[n]
    gmax = max(np.linalg.norm(v) for v in grads.values())
    for n in names:
        gv = res[0][f"g/{n}"].astype(np.float64).reshape(-1)
        rv = grads[n].reshape(-1)
        noisy = n.endswith(".bias") and not n.startswith(("bn", "seg_conv4"))
        scale = 1e-3 * gmax if noisy else max(np.linalg.norm(rv), 1e-3 * gmax)
        assert np.linalg.norm(gv - rv) / scale <= 2e-3, n
        # and against the reference's own DataParallel gradient samples
        idx = g[f"gidx/{n}"]
        assert np.abs(gv[idx] - g[f"gval/{n}"]).max() <= 2e-3 * scale, n
    # rank 0's running statistics == replica 0's (DataParallel shares device[0]'s buffers)
    for k in g.keys():
        if k.startswith("buf/") and "running" in k:
            np.testing.assert_allclose(res[0][k], g[k], rtol=2e-5, atol=1e-6, err_msg=k)

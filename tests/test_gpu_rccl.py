"""The data-parallel collective path over RCCL on the device (SURVEY §8 e): one rank of
``init_process_group("nccl")`` on cuda:0 with an explicit process group, so
``FusedTrainStep`` takes its bucketed all-reduce path (un-normalised gradients, loss
numerator and CE weight sum in the buffer tail, three async RCCL buckets issued from inside
the backward, Adam scaling by 1 / the global weight sum).  At world size 1 the result must
equal the single-process step (where the head normalises) up to fp32 rounding, and the
reference's golden step (tests/golden/train_c2.npz)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from golden_util import inputs, load

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, out):
    from pcs_amd.model import PointNetSegmentation
    from pcs_amd.optim import FusedAdam
    from pcs_amd.train import FusedTrainStep
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    try:
        g = load("train_c2")
        sd, pts, lab, msk, masks = inputs(g)
        bits = tuple(torch.from_numpy(np.packbits(mk, axis=1, bitorder="little")).to(dev) for mk in masks)
        res = {}
        for tag, pg in (("rccl", dist.group.WORLD), ("local", None)):
            m = PointNetSegmentation(int(g["C"])).to(dev)
            m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
            step = FusedTrainStep(m, FusedAdam(m, lr=1e-3, weight_decay=1e-4), class_weight=g["weight"],
                                  process_group=pg)
            assert step._distributed() == (pg is not None)
            loss = step(torch.from_numpy(pts).to(dev), torch.from_numpy(lab).to(dev), masks=bits)
            torch.cuda.synchronize()
            res[f"{tag}/loss"] = float(loss.item())
            for n, p in m.named_parameters():
                res[f"{tag}/g/{n}"] = p.grad.detach().cpu().numpy()
                res[f"{tag}/p/{n}"] = p.detach().cpu().numpy()
        np.savez(os.path.join(out, "res.npz"), **res)
    finally:
        dist.destroy_process_group()


def test_fused_step_rccl_world1_matches_local_step():
    g = load("train_c2")
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(_free_port(), out), nprocs=1, join=True, start_method="spawn")
        r = dict(np.load(os.path.join(out, "res.npz")))
    assert abs(r["rccl/loss"] - r["local/loss"]) <= 1e-6 * abs(r["local/loss"])
    assert abs(r["rccl/loss"] - float(g["loss"])) < 1e-5 * max(1.0, abs(float(g["loss"])))
    names = [k[len("local/g/"):] for k in r if k.startswith("local/g/")]
    gmax = max(np.linalg.norm(r[f"local/g/{n}"]) for n in names)
    for n in names:
        a, b = r[f"rccl/g/{n}"].astype(np.float64), r[f"local/g/{n}"].astype(np.float64)
        # the same kernels; only where the 1/sum_w normalisation is applied differs
        assert np.linalg.norm(a - b) <= 1e-5 * max(np.linalg.norm(b), 1e-3 * gmax), n
        # Adam's first step moves each weight by ~lr * sign(g) (lr = 1e-3): entries whose
        # |g| ~ eps (1e-8) can differ by up to lr; all others agree to 1e-5
        if np.linalg.norm(b) < 1e-4 * gmax:   # analytically ~0 (BN-cancelled biases, bn_global.bias):
            continue                          # Adam steps by lr * sign(rounding noise)
        d = np.abs(r[f"rccl/p/{n}"].astype(np.float64) - r[f"local/p/{n}"])
        assert (d > 1e-5).mean() < 1e-4 and d.max() <= 2e-3, (n, float(d.max()))

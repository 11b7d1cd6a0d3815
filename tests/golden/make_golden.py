"""Generate golden vectors by running the REFERENCE model itself (not our oracle).

Run in the build container, where /root/reference exists:

    python tests/golden/make_golden.py

It imports /root/reference/point_cloud_segmentation.py with an ``h5py`` stub (h5py is
not installed; only PointCloudDataset touches it), loads seeded weights
(oracle.init_params) into the reference ``PointNetSegmentation``, replays seeded dropout
masks into its ``nn.Dropout`` module, and records what the reference computes with
torch CPU fp32 autograd: logits, the weighted CE loss of P:216/P:251, per-parameter
gradient norms plus seeded samples, BN running stats after the step, and Adam-updated
parameter samples (P:217, P:255).  Only data is written (tests/golden/*.npz); the
reference source never leaves /root/reference.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import torch  # noqa: E402

import pointnet_oracle as orc  # noqa: E402
import pcs_amd.data as pdata  # noqa: E402

REF = "/root/reference/point_cloud_segmentation.py"
OUT = os.path.dirname(os.path.abspath(__file__))
N_SAMPLES = 512


def load_reference():
    sys.modules.setdefault("h5py", types.ModuleType("h5py"))
    spec = importlib.util.spec_from_file_location("pcs_reference", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class ReplayDropout(torch.nn.Module):
    """Stands in for the reference's nn.Dropout(0.3): applies pre-drawn keep masks in call order."""

    def __init__(self, masks, p=0.3):
        super().__init__()
        self.masks = [torch.from_numpy(m.astype(np.float32)) for m in masks]
        self.p = p
        self.calls = 0

    def forward(self, x):  # x is (B, C, N) in the reference layout
        if not self.training:
            return x
        m = self.masks[self.calls % len(self.masks)]
        self.calls += 1
        B, C, N = x.shape
        m = m.reshape(B, N, C).permute(0, 2, 1)
        return x * m / (1.0 - self.p)


def sample_idx(seed, n):
    rng = np.random.Generator(np.random.PCG64(seed))
    return np.sort(rng.choice(n, size=min(N_SAMPLES, n), replace=False))


def make_case(ref, name, *, C, n_points, seed, train, bn_rand, dropout, grid=32):
    sd = orc.init_params(C, seed, bn_affine_random=bn_rand)
    pts, lab, msk = pdata.synthetic_batch(seed + 1, n_points, C, grid=grid)
    B, N, _ = pts.shape
    M = B * N
    model = ref.PointNetSegmentation(num_classes=C)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
    masks = orc.dropout_masks(seed + 2, M) if dropout else (np.ones((M, 512), np.uint8),
                                                           np.ones((M, 256), np.uint8))
    model.dropout = ReplayDropout(masks)
    weight = pdata.class_weights([lab[b][msk[b]] for b in range(B)], num_classes=C)
    out = {"C": C, "seed": seed, "n_points": np.array(n_points), "train": int(train),
           "bn_rand": int(bn_rand), "dropout": int(dropout), "grid": grid,
           "weight": np.array(weight, np.float32)}
    x = torch.from_numpy(pts)
    if not train:
        model.eval()
        with torch.no_grad():
            logits = model(x)
        out["logits"] = logits.contiguous().numpy()
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
        return
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)   # P:217
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(weight))  # P:216
    opt.zero_grad()
    logits = model(x)
    loss = crit(logits.contiguous().view(-1, C), torch.from_numpy(lab).view(-1))   # P:247-251
    loss.backward()
    out["logits"] = logits.detach().contiguous().numpy()
    out["loss"] = np.float64(loss.item())
    names = [n for n, _ in model.named_parameters()]
    out["param_names"] = np.array(names)
    for i, (n, p) in enumerate(model.named_parameters()):
        g = p.grad.detach().numpy().reshape(-1)
        idx = sample_idx(1000 + i, g.size)
        out[f"gnorm/{n}"] = np.float64(np.linalg.norm(g.astype(np.float64)))
        out[f"gidx/{n}"] = idx
        out[f"gval/{n}"] = g[idx]
    opt.step()                                                                # P:255
    for i, (n, p) in enumerate(model.named_parameters()):
        idx = out[f"gidx/{n}"]
        out[f"pval/{n}"] = p.detach().numpy().reshape(-1)[idx]
    for k, v in model.state_dict().items():
        if "running" in k or "num_batches" in k:
            out[f"buf/{k}"] = v.numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)


def make_dp_case(ref, name, *, C, n_points, seed, world, bn_rand=False):
    """nn.DataParallel semantics (P:208-211), emulated on CPU with the reference module:
    the padded batch is chunked over ``world`` replicas (scatter = tensor.chunk), each
    replica runs forward on its scenes with its own BatchNorm batch statistics, outputs are
    gathered and ONE loss is taken over all of them (P:251), replica gradients are
    reduce-added into the base module, and Adam steps the base.  Replica 0 shares the base
    module's buffers (DataParallel's guarantee), so the running stats are replica 0's."""
    import copy
    sd = orc.init_params(C, seed, bn_affine_random=bn_rand)
    pts, lab, msk = pdata.synthetic_batch(seed + 1, n_points, C, grid=32)
    B, N, _ = pts.shape
    masks = orc.dropout_masks(seed + 2, B * N)
    base = ref.PointNetSegmentation(num_classes=C)
    base.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
    base.train()
    replicas = [base] + [copy.deepcopy(base) for _ in range(world - 1)]
    weight = pdata.class_weights([lab[b][msk[b]] for b in range(B)], num_classes=C)
    outs = []
    for r, mod in enumerate(replicas):
        lo, hi = pdata.shard_bounds(B, r, world)
        rows = slice(lo * N, hi * N)
        mod.dropout = ReplayDropout((masks[0][rows], masks[1][rows]))
        outs.append(mod(torch.from_numpy(pts[lo:hi])))
    logits = torch.cat(outs, 0)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(weight))
    loss = crit(logits.contiguous().view(-1, C), torch.from_numpy(lab).view(-1))
    loss.backward()
    for mod in replicas[1:]:
        for pb, pr in zip(base.parameters(), mod.parameters()):
            pb.grad += pr.grad
    out = {"C": C, "seed": seed, "n_points": np.array(n_points), "train": 1, "world": world,
           "bn_rand": int(bn_rand), "dropout": 1, "grid": 32, "weight": np.array(weight, np.float32),
           "logits": logits.detach().contiguous().numpy(), "loss": np.float64(loss.item())}
    names = [n for n, _ in base.named_parameters()]
    out["param_names"] = np.array(names)
    for i, (n, p) in enumerate(base.named_parameters()):
        g = p.grad.detach().numpy().reshape(-1)
        idx = sample_idx(1000 + i, g.size)
        out[f"gnorm/{n}"] = np.float64(np.linalg.norm(g.astype(np.float64)))
        out[f"gidx/{n}"] = idx
        out[f"gval/{n}"] = g[idx]
    opt = torch.optim.Adam(base.parameters(), lr=1e-3, weight_decay=1e-4)
    opt.step()
    for n, p in base.named_parameters():
        out[f"pval/{n}"] = p.detach().numpy().reshape(-1)[out[f"gidx/{n}"]]
    for k, v in base.state_dict().items():
        if "running" in k or "num_batches" in k:
            out[f"buf/{k}"] = v.numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)


def main(only=()):
    torch.set_num_threads(8)
    ref = load_reference()
    cases = {
        "eval_c2_bnrand": lambda: make_case(ref, "eval_c2_bnrand", C=2, n_points=[512, 512],
                                            seed=11, train=False, bn_rand=True, dropout=False),
        "train_c2": lambda: make_case(ref, "train_c2", C=2, n_points=[1024] * 4, seed=21,
                                      train=True, bn_rand=False, dropout=True),
        "train_c3_ragged_bnrand": lambda: make_case(ref, "train_c3_ragged_bnrand", C=3,
                                                    n_points=[600, 1024, 401, 800], seed=31,
                                                    train=True, bn_rand=True, dropout=True),
        "train_c2_nodrop_small": lambda: make_case(ref, "train_c2_nodrop_small", C=2,
                                                   n_points=[300, 300], seed=41, train=True,
                                                   bn_rand=False, dropout=False),
        "train_c3_dp2": lambda: make_dp_case(ref, "train_c3_dp2", C=3,
                                             n_points=[700, 1024, 512, 900], seed=51, world=2,
                                             bn_rand=True),
    }
    for name, fn in cases.items():
        if not only or name in only:
            fn()
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))     # optionally: names of the cases to (re)generate

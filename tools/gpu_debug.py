"""Per-layer comparison of the HIP path against the numpy oracle (debugging aid, GPU).

    python tools/gpu_debug.py [case] [fp32|bf16]

Runs one golden case through pcs_amd (train mode, replayed dropout masks), then prints the
max norm-relative error of every stored pre-BN activation, the logits, the loss and every
parameter gradient against oracle/pointnet_oracle.py.  Test infrastructure only.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]

import pcs_amd  # noqa: E402
from pcs_amd.model import PointNetSegmentation  # noqa: E402
import pointnet_oracle as orc  # noqa: E402
from golden_util import inputs, load, rel_err  # noqa: E402


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "train_c2_nodrop_small"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    g = load(case)
    sd, pts, lab, msk, masks = inputs(g)
    C = int(g["C"])
    train = bool(g["train"])
    dev = torch.device("cuda")
    model = PointNetSegmentation(C, compute_dtype=dtype).to(dev)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
    model.train(train)
    model._engine().flags = int(os.environ.get("PCS_FLAGS", "0"))   # e.g. 2 = no LDS-DMA kernel
    x = torch.from_numpy(pts).to(dev)
    if train:
        b1 = np.packbits(masks[0], axis=1, bitorder="little")
        b2 = np.packbits(masks[1], axis=1, bitorder="little")
        model.set_dropout_masks(torch.from_numpy(b1).to(dev), torch.from_numpy(b2).to(dev))
    out = model(x)
    torch.cuda.synchronize()
    ref_logits, cache = orc.forward(sd, pts, train=train, masks=masks)
    print(f"case={case} dtype={dtype} logits rel err = {rel_err(out.detach().cpu().numpy(), ref_logits):.3e}"
          f"  vs golden {rel_err(out.detach().cpu().numpy(), g['logits']):.3e}")
    if not train:
        return
    # intermediate activations saved by the last forward are not exposed by autograd; rerun engine
    eng = model._engine()
    P = model._param_dict()
    sv = eng.forward(P, {}, x, train=True, masks=model._masks or (
        torch.from_numpy(np.packbits(masks[0], axis=1, bitorder="little")).to(dev),
        torch.from_numpy(np.packbits(masks[1], axis=1, bitorder="little")).to(dev)), seed=0)
    torch.cuda.synchronize()
    for conv, ys in sv.ys.items():   # stored activations omit the per-channel BN offset
        if conv not in cache:          # a5 (stored post-BN/ReLU) has no pre-BN oracle entry
            continue
        yv = ys.float().cpu().numpy()
        ref = cache[conv]["y"]
        d = (yv - yv.mean(0)) - (ref - ref.mean(0))
        print(f"  y[{conv:12s}] centred rel err {np.abs(d).max() / np.abs(ref - ref.mean(0)).max():.3e}")
    print(f"  pooled g rel err {rel_err(sv.g.cpu().numpy(), cache['pool']['g']):.3e}")
    am = sv.am.cpu().numpy() - (np.arange(sv.B) * sv.N)[:, None]
    print(f"  argmax mismatches {(am != cache['pool']['idx']).sum()} / {am.size}")
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(g["weight"], device=dev))
    loss = crit(out.contiguous().view(-1, C), torch.from_numpy(lab).to(dev).view(-1))
    loss.backward()
    torch.cuda.synchronize()
    rloss, _, grads, _ = orc.train_step(sd, pts, lab, g["weight"], masks=masks)
    print(f"  loss {loss.item():.8f} oracle {rloss:.8f} golden {float(g['loss']):.8f}")
    gmax = max(np.linalg.norm(v) for v in grads.values())
    for n, p in model.named_parameters():
        gv = p.grad.detach().cpu().numpy().reshape(-1)
        rv = grads[n].reshape(-1)
        e = np.abs(gv - rv).max() / max(np.abs(rv).max(), 1e-3 * gmax)
        en = np.linalg.norm(gv - rv) / max(np.linalg.norm(rv), 1e-3 * gmax)
        cs = gv @ rv / (np.linalg.norm(gv) * np.linalg.norm(rv) + 1e-30)
        print(f"  grad[{n:22s}] max-rel {e:.3e} norm-rel {en:.3e} cos {cs:.6f} |g|={np.linalg.norm(rv):.3e}")


if __name__ == "__main__":
    main()

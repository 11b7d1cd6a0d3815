"""bf16 vs fp32 gradient agreement (1 - cosine per tensor) as the scene size grows:
python tools/bf16_scaling.py  (dense G^3 scenes, B = 4, one train-mode step, same dropout)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "oracle")]
import numpy as np
import torch
import pointnet_oracle as orc
from pcs_amd.data import class_weights, synthetic_batch
from pcs_amd.model import PointNetSegmentation

DEV = torch.device("cuda")
KEYS = ["conv2.weight", "conv5.weight", "global_feat.weight", "bn_global.weight", "bn_global.bias",
        "seg_conv1.weight", "seg_conv2.weight", "bn_seg1.bias"]
for G in (16, 32, 64, 128):
    pts, lab, _ = synthetic_batch(4321, [G ** 3] * 4, 2, grid=G, dense=True)
    w = class_weights([lab[b] for b in range(4)], num_classes=2)
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV).view(-1)
    sd = orc.init_params(2, 77)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1, weight=torch.tensor(w, device=DEV))
    grads = {}
    for dt in ("fp32", "bf16"):
        m = PointNetSegmentation(2, compute_dtype=dt).to(DEV)
        m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
        m.train(); m.seed_dropout(99)
        loss = crit(m(x).contiguous().view(-1, 2), y); loss.backward()
        grads[dt] = {n: p.grad.detach().double().cpu().flatten() for n, p in m.named_parameters()}
        del m, loss; torch.cuda.empty_cache()
    r = {k: 1 - float(grads["bf16"][k] @ grads["fp32"][k] / (grads["bf16"][k].norm() * grads["fp32"][k].norm()))
         for k in KEYS}
    print(f"N={G**3:8d}", " ".join(f"{k}={v:.4f}" for k, v in r.items()), flush=True)

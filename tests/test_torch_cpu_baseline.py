"""Pin the pure-PyTorch CPU restatement (oracle/torch_cpu.py, bench.py's cpu_baseline) to the
goldens written by the imported reference (tests/golden/make_golden.py): logits, loss, every
parameter gradient and the BN running statistics after one train step."""
import numpy as np
import pytest
import torch

import torch_cpu as tc
from golden_util import CASES, inputs, load, rel_err


@pytest.mark.parametrize("name", CASES)
def test_torch_cpu_forward_matches_reference_goldens(name):
    g = load(name)
    sd, pts, lab, msk, masks = inputs(g)
    T = tc.to_tensors(sd)
    with torch.no_grad():
        out = tc.forward(T, torch.from_numpy(pts), train=bool(g["train"]), masks=masks)
    assert rel_err(out.numpy(), g["logits"]) < 2e-5


@pytest.mark.parametrize("name", [c for c in CASES if not c.startswith("eval")])
def test_torch_cpu_train_step_matches_reference_goldens(name):
    g = load(name)
    sd, pts, lab, msk, masks = inputs(g)
    T = tc.to_tensors(sd)
    loss, _ = tc.train_step(T, torch.from_numpy(pts), torch.from_numpy(lab),
                            torch.tensor(g["weight"], dtype=torch.float32), masks=masks)
    assert abs(loss.item() - float(g["loss"])) < 1e-5 * max(1.0, abs(float(g["loss"])))
    names = [str(n) for n in g["param_names"]]
    gmax = max(float(g[f"gnorm/{n}"]) for n in names)
    for n in names:
        gv = T[n].grad.numpy().astype(np.float64).reshape(-1)
        # BN-followed conv biases have analytically zero gradients (fp32 noise on both sides)
        noisy = n.endswith(".bias") and not n.startswith(("bn", "seg_conv4"))
        scale = 0.05 * gmax if noisy else max(float(g[f"gnorm/{n}"]), 1e-3 * gmax)
        assert np.abs(gv[g[f"gidx/{n}"]] - g[f"gval/{n}"]).max() <= 2e-4 * scale + 1e-7, n
    for k in g.keys():
        if k.startswith("buf/") and "num_batches" not in k:
            np.testing.assert_allclose(T[k[4:]].numpy(), g[k], rtol=1e-5, atol=1e-6, err_msg=k)

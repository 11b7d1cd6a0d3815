"""Pin the numpy oracle against golden vectors produced by the reference itself.

The fixtures (tests/golden/*.npz) were written by tests/golden/make_golden.py from the
imported reference (torch CPU fp32 autograd); here the oracle recomputes every recorded
quantity in float64 and must agree to fp32 rounding.
"""
import numpy as np
import pytest

import pointnet_oracle as orc
from golden_util import CASES, assert_train_matches, inputs, load, rel_err


@pytest.mark.parametrize("name", CASES)
def test_oracle_logits(name):
    g = load(name)
    sd, pts, lab, msk, masks = inputs(g)
    logits, _ = orc.forward(sd, pts, train=bool(g["train"]), masks=masks)
    assert rel_err(logits, g["logits"]) < 2e-5


@pytest.mark.parametrize("name", [c for c in CASES if not c.startswith("eval")])
def test_oracle_train_step(name):
    g = load(name)
    sd, pts, lab, msk, masks = inputs(g)
    loss, logits, grads, cache = orc.train_step(sd, pts, lab, g["weight"], masks=masks)
    assert_train_matches(g, sd, loss, grads, orc.update_running_stats(sd, cache))


def test_oracle_dropout_masks_keep_rate():
    m1, m2 = orc.dropout_masks(5, 4096)
    assert abs(m1.mean() - 0.7) < 0.01 and abs(m2.mean() - 0.7) < 0.01


def test_state_dict_keys_match_golden_names():
    g = load("train_c2")
    names = [str(n) for n in g["param_names"]]
    keys = orc.state_dict_keys(2)
    assert len(keys) == 65
    assert [k for k in keys if "running" not in k and "num_batches" not in k] == names

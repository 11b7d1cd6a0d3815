"""Host side of SURVEY §8 f1/f3: metrics from a confusion matrix (vs sklearn, as the
reference computes them at P:343-346), checkpoint layout of P:373-382 with the module.
prefix handling of P:409-428, FusedAdam state compatible with torch.optim.Adam, StepLR."""
import numpy as np
import pytest
import torch

import pointnet_oracle as orc
from pcs_amd.checkpoint import CHECKPOINT_KEYS, load_checkpoint, save_checkpoint
from pcs_amd.metrics import f1_class2, metrics_from_confusion
from pcs_amd.model import PointNetSegmentation, load_reference_checkpoint
from pcs_amd.optim import FusedAdam

sklearn_metrics = pytest.importorskip("sklearn.metrics")


def _cm(t, p, C):
    cm = np.zeros((C, C), np.int64)
    np.add.at(cm, (t, p), 1)
    return cm


@pytest.mark.parametrize("C,drop", [(2, None), (3, None), (4, 2), (5, 0)])
def test_metrics_match_sklearn(C, drop):
    rng = np.random.default_rng(C)
    t = rng.integers(0, C, 5000)
    p = np.where(rng.random(5000) < 0.7, t, rng.integers(0, C, 5000))
    if drop is not None:          # a class absent from both y_true and y_pred
        keep = (t != drop) & (p != drop)
        t, p = t[keep], p[keep]
    m = metrics_from_confusion(_cm(t, p, C))
    f1 = sklearn_metrics.f1_score(t, p, average=None)
    np.testing.assert_allclose(m["f1_per_class"], f1, rtol=1e-12)
    assert m["accuracy"] == pytest.approx(sklearn_metrics.accuracy_score(t, p))
    assert m["f1_class2"] == (float(f1[2]) if len(f1) > 2 else 0.0)   # P:346
    assert m["miou"] == pytest.approx(orc.miou(orc.confusion(p, t, C)))


def test_f1_class2_binary_is_zero():
    assert f1_class2(np.array([[5, 1], [2, 7]])) == 0.0


def _model(C=2):
    torch.manual_seed(0)
    return PointNetSegmentation(C)


def test_checkpoint_layout_and_roundtrip(tmp_path):
    m = _model(3)
    opt = FusedAdam(m, lr=1e-3, weight_decay=1e-4)
    opt.exp_avg.uniform_()
    opt.exp_avg_sq.uniform_()
    opt.step_count = 7
    path = tmp_path / "best_model.pth"
    save_checkpoint(path, m, opt, epoch=4, train_loss=0.5, val_loss=0.25, f1_class2=0.1,
                    f1_per_class=[0.9, 0.8, 0.1])
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert tuple(ck.keys()) == CHECKPOINT_KEYS
    assert len(ck["model_state_dict"]) == 65
    assert ck["num_classes"] == 3 and ck["epoch"] == 4
    m2, ck2 = load_checkpoint(path, device="cpu")
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    # the optimizer state restores into a FusedAdam and into a plain torch.optim.Adam
    opt2 = FusedAdam(m2)
    opt2.load_state_dict(ck2["optimizer_state_dict"])
    assert opt2.step_count == 7 and torch.equal(opt2.exp_avg, opt.exp_avg)
    ref = torch.nn.Module()
    ref.ps = torch.nn.ParameterList([torch.nn.Parameter(p.detach().clone()) for p in m.parameters()])
    adam = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    adam.load_state_dict(ck2["optimizer_state_dict"])
    st0 = adam.state[next(iter(ref.parameters()))]
    o = m._flat_offsets()["conv1.weight"]   # flat buffers are in gradient-bucket order
    assert torch.equal(st0["exp_avg"].reshape(-1), opt.exp_avg[o:o + st0["exp_avg"].numel()])


def test_data_parallel_prefix(tmp_path):
    m = _model()
    path = tmp_path / "dp.pth"
    save_checkpoint(path, m, data_parallel=True)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert all(k.startswith("module.") for k in ck["model_state_dict"])
    sd, _ = load_reference_checkpoint(path)
    assert set(sd) == set(m.state_dict())


@pytest.mark.filterwarnings("ignore:Detected call of")   # no GPU: no Adam step
def test_step_lr_drives_fused_adam():
    m = _model()
    opt = FusedAdam(m, lr=1e-3)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=20, gamma=0.5)   # P:218
    lrs = []
    for _ in range(45):
        lrs.append(opt.param_groups[0]["lr"])
        sched.step()
    assert lrs[0] == 1e-3 and lrs[20] == 5e-4 and lrs[40] == 2.5e-4

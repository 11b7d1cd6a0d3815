"""Device side of SURVEY §8 f1/f3: pcs_confusion (vs numpy), predict() (vs the oracle's eval
forward on the reference golden case) and a save -> load -> predict round trip."""
import numpy as np
import pytest
import torch

import pointnet_oracle as orc
from golden_util import inputs, load

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.mark.parametrize("C", [2, 3, 13])
def test_confusion_matches_numpy(C):
    from pcs_amd.metrics import ConfusionMeter
    g = torch.Generator().manual_seed(C)
    meter = ConfusionMeter(C, DEV)
    ref = np.zeros((C, C), np.int64)
    for _ in range(2):
        z = torch.randn(3, 1001, C, generator=g)
        y = torch.randint(-1, C, (3, 1001), generator=g)
        meter.update(z.to(DEV), y.to(DEV))
        v = y.reshape(-1).numpy() >= 0
        np.add.at(ref, (y.reshape(-1).numpy()[v], z.reshape(-1, C).argmax(1).numpy()[v]), 1)
    assert np.array_equal(meter.cm.cpu().numpy(), ref)
    assert meter.compute()["points"] == int(ref.sum())


def test_predict_and_checkpoint_roundtrip(tmp_path):
    from pcs_amd.checkpoint import load_checkpoint, predict, save_checkpoint
    from pcs_amd.model import PointNetSegmentation
    g = load("eval_c2_bnrand")
    sd, pts, lab, msk, masks = inputs(g)
    m = PointNetSegmentation(int(g["C"])).to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in sd.items()})
    x = torch.from_numpy(pts).to(DEV)
    pred = predict(m, x).cpu().numpy()
    logits, _ = orc.forward(sd, pts, train=False)
    top2 = np.sort(logits, axis=-1)[..., -2:]
    clear = (top2[..., 1] - top2[..., 0]) > 1e-4 * np.abs(logits).max()
    assert np.array_equal(pred[clear], logits.argmax(-1)[clear])
    path = tmp_path / "best_model.pth"
    save_checkpoint(path, m, epoch=1, data_parallel=True)
    m2, _ = load_checkpoint(path, device=DEV)
    assert torch.equal(predict(m2, x).cpu(), torch.from_numpy(pred))

"""North-star mIoU parity (BASELINE north_star "mIoU within 1e-3 of reference"; SURVEY §0.4,
§8 c): the HIP path and the reference evaluate the SAME weights on the same synthetic clouds.

* device side: eval-mode forward through the C ABI, then the device confusion matrix
  (pcs_confusion via ConfusionMeter) and pcs_amd.metrics.miou;
* reference side: argmax of the logits the reference module itself wrote into the golden
  fixture (tests/golden/make_golden.py), or of the fp64 numpy oracle (pinned to those
  fixtures) on inputs no fixture covers, scored with sklearn's jaccard_score(average='macro')
  (the reference reports sklearn metrics, P:341-346; mIoU itself is build-defined).

Seeded random weights predict one class almost everywhere, which makes mIoU uninformative, so
the main case first trains the model for 300 fused steps on the device (weighted CE, P:216) and
then scores THOSE weights on both sides.  fp32 and bf16 are both held to the north star's 1e-3.

bf16 here is the bf16 model's eval forward as shipped (eval_trunk="fp32": conv1..conv4 in
fp32, conv5 fed a 16-bit split of a4; every layer from conv5 on in bf16).  On these trained
weights bf16 STORAGE of the narrow trunk alone moves mIoU by 1.27e-3 (81 flipped points,
logit-margin error p50 5.6e-2): the numpy restatement of that storage
(oracle/bf16_emulation.eval_logits) reproduces the device's error to p50 1.1e-3, so it is the
arithmetic's, not a kernel's (tools/miou_attr.py).
test_bf16_storage_eval_is_its_emulation pins exactly that and reports the number."""
import numpy as np
import pytest
import torch

import pointnet_oracle as orc
from golden_util import inputs, load

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
TOL = 1e-3


def _sk_miou(pred, lab):
    from sklearn.metrics import jaccard_score
    v = lab >= 0
    return float(jaccard_score(lab[v], pred[v], average="macro"))


def _device_eval(sd, pts, lab, C, dtype, eval_trunk="fp32"):
    from pcs_amd.metrics import ConfusionMeter
    from pcs_amd.model import PointNetSegmentation
    m = PointNetSegmentation(C, compute_dtype=dtype, eval_trunk=eval_trunk).to(DEV)
    m.load_state_dict({k: torch.as_tensor(np.array(v)) for k, v in sd.items()})
    m.eval()
    meter = ConfusionMeter(C, DEV)
    with torch.no_grad():
        lg = m(torch.from_numpy(pts).to(DEV))
        meter.update(lg, torch.from_numpy(lab).to(DEV))
    lgn = lg.float().cpu().numpy()
    return meter.compute()["miou"], lgn.argmax(-1).reshape(-1), lgn


def _device_miou(sd, pts, lab, C, dtype):
    return _device_eval(sd, pts, lab, C, dtype)[0]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_miou_matches_reference_golden(dtype):
    """eval_c2_bnrand: the logits in the fixture were written by the reference module."""
    g = load("eval_c2_bnrand")
    sd, pts, lab, _, _ = inputs(g)
    ref = _sk_miou(np.asarray(g["logits"]).argmax(-1).reshape(-1), lab.reshape(-1))
    got = _device_miou(sd, pts, lab, int(g["C"]), dtype)
    print(f"{dtype}: mIoU {got:.6f} vs reference {ref:.6f}")
    assert abs(got - ref) <= TOL


@pytest.fixture(scope="module")
def trained():
    """fp32 weights after 300 fused training steps (Adam, class-weighted CE) on seeded clouds."""
    import pcs_amd.data as pdata
    from pcs_amd.model import PointNetSegmentation
    from pcs_amd.optim import FusedAdam
    from pcs_amd.train import FusedTrainStep
    C = 2
    torch.manual_seed(7)
    m = PointNetSegmentation(C).to(DEV)
    pts, lab, _ = pdata.synthetic_batch(11, [4096] * 4, C, grid=32)
    w = pdata.class_weights([lab[b][lab[b] >= 0] for b in range(lab.shape[0])], num_classes=C)
    step = FusedTrainStep(m, FusedAdam(m, lr=3e-3), class_weight=w)
    x, y = torch.from_numpy(pts).to(DEV), torch.from_numpy(lab).to(DEV)
    for i in range(300):
        step(x, y, seed=1000 + i)
    torch.cuda.synchronize()
    return C, {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}


def _val_case(trained):
    import pcs_amd.data as pdata
    C, sd = trained
    pts, lab, _ = pdata.synthetic_batch(4242, [8192, 6000, 8192, 5000], C, grid=32)
    logits, _ = orc.forward({k: np.asarray(v, np.float64) if v.dtype.kind == "f" else v
                             for k, v in sd.items()}, pts, train=False)
    return C, sd, pts, lab, logits


def _margin(lg):
    return (lg[..., 1] - lg[..., 0]).reshape(-1)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_miou_of_trained_weights_matches_oracle(trained, dtype):
    """Ragged val batch (pads labelled -1 enter BN / max-pool as in collate_fn) scored with
    the trained weights by the device path and by the fp64 oracle."""
    C, sd, pts, lab, logits = _val_case(trained)
    pred = logits.argmax(-1).reshape(-1)
    v = lab.reshape(-1) >= 0
    hist = np.bincount(pred[v], minlength=C)
    ref = _sk_miou(pred, lab.reshape(-1))
    got, dpred, dlog = _device_eval(sd, pts, lab, C, dtype)
    flips = (dpred != pred) & v
    dm = np.abs(_margin(dlog) - _margin(logits))[v]
    print(f"trained {dtype}: mIoU {got:.6f} vs oracle {ref:.6f} (diff {got - ref:+.2e}), oracle prediction "
          f"histogram {hist}, flipped {int(flips.sum())}, margin error p50 {np.median(dm):.3e} "
          f"p99.9 {np.quantile(dm, 0.999):.3e} max {dm.max():.3e}, max |logit| {np.abs(logits).max():.3e}")
    assert hist.min() > 0.01 * v.sum(), "training left a degenerate (one-class) predictor"
    # the device confusion matrix and mIoU are exact for the predictions the path made
    assert abs(got - _sk_miou(dpred, lab.reshape(-1))) <= 1e-9
    assert abs(got - ref) <= TOL
    if dtype == "fp32":
        assert flips.sum() == 0


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_storage_eval_is_its_emulation(trained, dtype):
    """The eval forward on the training step's storage (eval_trunk="bf16": every layer bf16,
    fp8 a5 / global_feat weight rows for "fp8") and as shipped (eval_trunk="fp32") against the
    numpy restatement of exactly that storage (oracle/bf16_emulation.eval_logits): their logit
    margins agree to within 1/8 of what the storage itself costs, so a mIoU miss of the
    storage path is a property of its number format, not of a kernel.  Each path is held to
    its OWN format cost (the shipped fp32 trunk's is ~7x smaller than the all-bf16 one's); the
    emulation restates the shipped path's 16-bit split of a4 ("Asplit4") and the kernels'
    single-rounding fmaf, so the typical point agrees to fp32 rounding (p50 <= 1e-6; r06:
    2.4e-7 on both trunks).  The p99.9 tail is set by bf16 rounding-boundary flips that depend
    on the order of fp32 sums, and the emulation in float64 sums ("f64", another valid order)
    sits 7.7e-3 from the float32-sum emulation on the fp32 trunk, above that trunk's cost/8
    (4.8e-3): no implementation can be held below that floor, so the tail bound is the larger
    of cost/8 and 1.5x the floor (device 5.5e-3, r06).  The misses are reported, not bounded
    (fp8: ~100 flipped points either way, see the print)."""
    from bf16_emulation import eval_logits, eval_sites
    C, sd, pts, lab, logits = _val_case(trained)
    pred = logits.argmax(-1).reshape(-1)
    v = lab.reshape(-1) >= 0
    ref = _sk_miou(pred, lab.reshape(-1))
    p = lambda a: float(np.quantile(a, 0.999))   # noqa: E731
    fp8 = dtype == "fp8"
    for trunk in ("bf16", "fp32"):
        got, dpred, dlog = _device_eval(sd, pts, lab, C, dtype, eval_trunk=trunk)
        emu = eval_logits(sd, pts, eval_sites(trunk), fp8=fp8)
        emu64 = eval_logits(sd, pts, eval_sites(trunk), fp8=fp8, sums="f64")
        err = np.abs(_margin(emu) - _margin(logits))[v]        # what the storage costs
        cost = p(err)                                          # yardstick: this path's own format
        diff = np.abs(_margin(dlog) - _margin(emu))[v]         # device vs its restatement
        noise = np.abs(_margin(emu64) - _margin(emu))[v]       # the restatement in another sum order
        q = lambda a: f"p50 {np.median(a):.2e} p99 {np.quantile(a, 0.99):.2e} p99.9 {p(a):.2e}"   # noqa: E731
        print(f"{dtype} eval_trunk={trunk}: mIoU {got:.6f} vs oracle {ref:.6f} (diff {got - ref:+.2e}, "
              f"emulation {_sk_miou(emu.argmax(-1).reshape(-1), lab.reshape(-1)) - ref:+.2e}), flipped "
              f"{int(((dpred != pred) & v).sum())}; margin error: format {q(err)}; device vs emulation "
              f"{q(diff)}; emulation f64 sums vs f32 sums {q(noise)}; bound {max(cost / 8, 1.5 * p(noise)):.3e}")
        assert np.median(diff) <= 1e-6
        assert p(diff) <= max(cost / 8, 1.5 * p(noise))

"""The data-parallel gradient buckets (train.GradientBuckets, engine.bucket_ranges) are issued
from inside Engine.backward the moment their last writer is enqueued (§8 e).  An early issue
would all-reduce a partly written range -- invisible at world size 1, where the all-reduce is
an identity.  Here each issue point synchronises the device and snapshots its range of the flat
gradient buffer (prefilled with NaN); after the backward every snapshot must equal the final
range bit for bit, i.e. nothing wrote into a bucket after it was handed to the collective."""
import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

DEV = torch.device("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp8"])
def test_bucket_issue_points_follow_their_last_writer(dtype):
    import pcs_amd._lib as L
    from pcs_amd.data import synthetic_batch
    from pcs_amd.model import PointNetSegmentation
    from pcs_amd.optim import flat_buffers
    torch.manual_seed(5)
    model = PointNetSegmentation(2, compute_dtype=dtype).to(DEV)
    model.train()
    eng = model._engine()
    P, bufs = model._param_dict(), model._buffer_dict()
    _, gflat = flat_buffers(model)
    pts, lab, _ = synthetic_batch(11, [4096 + 17, 3000], 2, grid=32)
    x = torch.from_numpy(pts).to(DEV)
    y = torch.from_numpy(lab).to(DEV).reshape(-1)
    w = torch.tensor([0.7, 1.3], device=DEV)
    wsum = torch.empty(3, device=DEV)
    counts = torch.empty(16, dtype=torch.int64, device=DEV)
    L.call("pcs_ce_weight_sum", L.ptr(y), y.numel(), L.ptr(w), 2, L.ptr(counts), L.ptr(wsum), L.stream_ptr())
    sv = eng.forward(P, bufs, x, train=True, head_mode=L.HEAD_CE, labels=y, class_weight=w, wsum=wsum,
                     want_logits=False)
    gflat.fill_(float("nan"))
    gflat[eng.total_params:] = 0.0   # the loss tail is written by the caller, not the backward
    snaps, order = {}, []

    def on_bucket(name):
        torch.cuda.synchronize()
        lo, hi = eng.buckets[name]
        snaps[name] = gflat[lo:hi].clone()
        order.append(name)

    eng.backward(P, sv, gflat, on_bucket=on_bucket)
    torch.cuda.synchronize()
    assert sorted(order) == sorted(eng.buckets)
    assert torch.isfinite(gflat).all()
    for name, (lo, hi) in eng.buckets.items():
        assert torch.equal(snaps[name], gflat[lo:hi]), f"bucket {name} was written after its issue"

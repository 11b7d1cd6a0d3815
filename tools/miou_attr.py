"""Attribute the bf16 eval path's logit-margin error on trained weights to its rounding sites
(VERDICT r04 item 1).  CPU only: reads what tools/miou_dump.py wrote on the GPU box.

oracle/bf16_emulation.eval_logits restates the HIP bf16 EVAL forward in float32 with each
bf16 rounding site switchable; this script compares the device logits with it and with the
fp64 oracle, one site / one group of sites at a time, and reports the mIoU each leaves.

    python tools/miou_attr.py gpurun_out/miou_r05
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle")]

import pointnet_oracle as orc  # noqa: E402
from bf16_emulation import eval_logits, eval_sites  # noqa: E402

TRUNK = frozenset(f"{k}conv{i}" for k in "YAW" for i in (1, 2, 3, 4)) - {"Wconv1"}


def main(d):
    sd = dict(np.load(os.path.join(d, "trained_sd.npz")))
    v = dict(np.load(os.path.join(d, "val_logits.npz")))
    pts, lab = v["pts"], v["lab"].reshape(-1)
    valid = lab >= 0
    ref, _ = orc.forward({k: np.asarray(x, np.float64) if x.dtype.kind == "f" else x for k, x in sd.items()},
                         pts, train=False)
    rp = ref.argmax(-1).reshape(-1)
    rmarg = (ref[..., 1] - ref[..., 0]).reshape(-1)

    def miou(p):
        cm = np.zeros((2, 2), np.int64)
        np.add.at(cm, (lab[valid], p[valid]), 1)
        i = np.diag(cm)
        return float(np.mean(i / (cm.sum(0) + cm.sum(1) - i)))

    r0 = miou(rp)

    def report(tag, lg):
        p = lg.argmax(-1).reshape(-1)
        dm = np.abs((lg[..., 1] - lg[..., 0]).reshape(-1) - rmarg)[valid]
        print(f"{tag:46s} dmIoU {miou(p) - r0:+.2e}  flips {int(((p != rp) & valid).sum()):4d}  margin err "
              f"p50 {np.median(dm):.2e} p99.9 {np.quantile(dm, 0.999):.2e} max {dm.max():.2e}", flush=True)

    print(f"oracle mIoU {r0:.6f}, max |oracle logit| {np.abs(ref).max():.3f}, valid points {int(valid.sum())}")
    for dt in ("fp32", "bf16", "fp8"):
        if f"logits_{dt}" in v:
            report(f"device {dt}", v[f"logits_{dt}"])
    if "logits_bf16_trunk16" in v:
        report("device bf16, eval_trunk='bf16'", v["logits_bf16_trunk16"])
    allb = eval_sites("bf16")
    emu = eval_logits(sd, pts, allb)
    report("emulation: every bf16 site (eval_trunk='bf16')", emu)
    report("emulation: eval_trunk='fp32'", eval_logits(sd, pts, eval_sites("fp32")))
    report("emulation: no site", eval_logits(sd, pts, frozenset()))
    dev = v.get("logits_bf16_trunk16", v.get("logits_bf16"))
    dm = np.abs((dev[..., 1] - dev[..., 0]) - (emu[..., 1] - emu[..., 0])).reshape(-1)[valid]
    print(f"device bf16 storage path vs its emulation: margin diff p50 {np.median(dm):.2e} "
          f"p99.9 {np.quantile(dm, 0.999):.2e} max {dm.max():.2e}")
    for site in sorted(allb):
        report(f"  only {site}", eval_logits(sd, pts, frozenset({site})))
    report("  all but the trunk (conv1-4)", eval_logits(sd, pts, allb - TRUNK))
    report("  all but the trunk, a4 bf16", eval_logits(sd, pts, allb - TRUNK | {"Aconv4"}))
    report("  all but the trunk, W2-4 bf16", eval_logits(sd, pts, allb - TRUNK | {"Wconv2", "Wconv3", "Wconv4"}))
    report("  all but trunk weights", eval_logits(sd, pts, allb - {s for s in TRUNK if s[0] == "W"}))
    report("  all but trunk Y", eval_logits(sd, pts, allb - {s for s in TRUNK if s[0] == "Y"}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/miou_r05")

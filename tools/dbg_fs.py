"""Debug helper: where does the streaming forward kernel differ from fp64?"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
from test_gpu_fwd_stream import _run, SHAPES
for (K, C, kind) in SHAPES:
    for (B, N) in [(1, 4096), (2, 70005)]:
        out, st, ref, counts = _run(B, N, K, C, kind, 11)
        err = (out - ref).abs() / ref.abs().max()
        bad = (err > 8e-3) | ~torch.isfinite(out)
        print(K, C, kind, B, N, "bad frac", float(bad.double().mean()), "max", float(err.max()), flush=True)
        if bad.any():
            rows = bad.any(1).nonzero().flatten()
            cols = bad.any(0).nonzero().flatten()
            print("  bad rows", rows[:20].tolist(), "n", len(rows), " rows%64 hist", torch.bincount(rows % 64, minlength=64).tolist())
            print("  bad cols", cols[:40].tolist(), "n", len(cols))
            r0 = int(rows[0])
            print("  row", r0, "out", out[r0, :8].tolist(), "ref", ref[r0, :8].tolist())

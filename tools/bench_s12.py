"""Time the fused seg_conv1 + seg_conv2 forward (pcs_fwd_seg12) against the two pcs_gemm passes
it replaces at cfg2 size (4 x 128^3 rows), HIP events around 10 launches each (timing only;
tests/test_gpu_seg12.py checks the results).  PCS_LIB selects a variant build.

    python tools/bench_s12.py [--two-pass]"""
import ctypes as ct
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import pcs_amd._lib as L  # noqa: E402
from test_gpu_seg12 import _fused, _two_pass  # noqa: E402

DEV = torch.device("cuda")


def ops(B, N):
    M = B * N
    r = lambda *s: torch.randn(*s, device=DEV)   # noqa: E731
    return (r(M, 64).to(torch.bfloat16), r(64) * 0.5 + 1.0, r(64) * 0.3, (r(512, 64) * 0.15).to(torch.bfloat16),
            r(B, 512) * 0.2, r(512) * 0.3 + 0.8, r(512) * 0.2,
            torch.randint(0, 256, (M, 64), dtype=torch.uint8, device=DEV), (r(256, 512) * 0.05).to(torch.bfloat16))


def timed(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    B, N = 4, 128 ** 3
    o = ops(B, N)
    ks = 1.0 / 0.7
    tf = timed(lambda: _fused(L, B, N, *o, ks))
    line = f"{os.environ.get('PCS_LIB', 'in-tree')}: fused {tf:.3f} ms"
    if "--two-pass" in sys.argv:
        line += f", two passes {timed(lambda: _two_pass(L, B, N, *o, ks)):.3f} ms"
    print(line, flush=True)


if __name__ == "__main__":
    main()

"""Isolated duration of the dropout draw (pcs_dropout_bits, full grid) at the bench's two sizes
(M = 4 x 128^3 points: seg_conv1's 512 and seg_conv2's 256 channels), HIP events on the
launch stream, median of 20.  Timing only; PCS_LIB selects the library.

    python tools/bench_draw.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import pcs_amd._lib as L  # noqa: E402


def main():
    M = 4 * 128 ** 3
    s = L.stream_ptr()
    for C in (512, 256):
        bits = torch.empty(M, C // 8, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            L.call("pcs_dropout_bits", 7, 0, M, C, 0.3, L.ptr(bits), s)
        ts = []
        for i in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            L.call("pcs_dropout_bits", 7 + i, 0, M, C, 0.3, L.ptr(bits), s)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        keep = bits[: 1 << 16].cpu().numpy()
        import numpy as np
        rate = np.unpackbits(keep, axis=1, bitorder="little").mean()
        print(f"draw C={C}: {ts[len(ts) // 2]:.3f} ms (min {ts[0]:.3f}), keep rate {rate:.4f}", flush=True)


if __name__ == "__main__":
    main()

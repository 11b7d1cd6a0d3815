"""Micro-benchmark of the training step's head (pcs_head CE mode, bf16, C = 2, no logits out:
csrc/head_stream.hip) at cfg2 (4 x 128^3 rows).  Alternate builds: PCS_LIB=path.
    python tools/bench_head.py [reps]"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B, N, C = 4, 128 ** 3, 2
    M = B * N
    dev = torch.device("cuda")
    Y = torch.randn(M, 128, device=dev).to(torch.bfloat16)
    v = lambda n: torch.rand(n, device=dev) + 0.5   # noqa: E731
    s, t, mean, rstd, W, b, cw = v(128), v(128) - 1.0, v(128) - 1.0, v(128), v(C * 128) - 1.0, v(C), v(C)
    lab = torch.randint(-1, C, (M,), device=dev)
    wsum = torch.tensor([float(M)], device=dev)
    a = L.HeadArgs(num_scenes=B, scene_rows=N, Cin=128, num_classes=C, dtype=L.BF16, mode=L.HEAD_CE,
                   chunks_per_scene=0, Y=Y.data_ptr(), s=s.data_ptr(), t=t.data_ptr(), W=W.data_ptr(),
                   bias=b.data_ptr(), logits=None)
    L.load().pcs_head_geometry(ct.byref(a))
    nch = B * a.chunks_per_scene
    dZ = torch.empty(M, 128, dtype=torch.bfloat16, device=dev)
    stats, wp, lp = (torch.empty(nch, 128, 2, device=dev), torch.empty(nch, C * 129, device=dev),
                     torch.empty(nch, device=dev))
    a.labels, a.class_weight, a.wsum = lab.data_ptr(), cw.data_ptr(), wsum.data_ptr()
    a.dZ, a.mean, a.rstd = dZ.data_ptr(), mean.data_ptr(), rstd.data_ptr()
    a.stats, a.wpartial, a.loss_partial = stats.data_ptr(), wp.data_ptr(), lp.data_ptr()
    fn = lambda: L.call("pcs_head", ct.byref(a), L.stream_ptr())   # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"head CE (chunks {nch}): {ms:7.3f} ms  {M * (256 + 8 + 256) / 1e9 / ms:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()

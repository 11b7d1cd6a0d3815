"""Micro-benchmark of the channels-last Conv3d kernels (csrc/conv3d.hip): the
3x3x3 U-Net stencil forward, input gradient (transposed form) and weight gradient, plus the
2x2x2 stride-2 down / up convolutions, on B x G^3 voxel grids.  Prints ms and TF/s per launch
(algorithmic FLOPs 2 M taps Cin Cout) against the bf16 dense MFMA peak."""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402
import pcs_amd.voxel as V  # noqa: E402

PEAK = 2516.6


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    C = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    dev = torch.device("cuda")
    lib = L.load()
    st = L.stream_ptr()
    for (k, s, p, tr, cin, cout, name) in ((3, 1, 1, False, C, C, "stencil 3x3x3"),
                                           (2, 2, 0, False, C, 2 * C, "down 2x2x2/2"),
                                           (2, 2, 0, True, 2 * C, C, "up 2x2x2/2 (transposed)")):
        gin = (G, G, G) if not tr else (G // 2,) * 3
        g = V._geom(B, gin, cin, cout, k, s, p, tr)
        x = torch.randn(B, *gin, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(cout, k ** 3 * cin, device=dev) * 0.05).to(torch.bfloat16)
        M = B * g.Do * g.Ho * g.Wo
        y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, cout, device=dev).to(torch.bfloat16)
        flops = 2.0 * M * k ** 3 * cin * cout
        if tr:   # each output voxel of the 2x2x2/2 transposed form has one tap
            flops /= k ** 3
        ms = timeit(lambda: L.call("pcs_conv3d", ct.byref(g), L.ptr(x), L.ptr(w), None, L.ptr(y), L.BF16, st))
        print(f"{name:28s} fwd   {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s  ({flops / ms / 1e9 / PEAK:.3f} of peak)",
              flush=True)
        wt = torch.empty(cin, k ** 3 * cout, device=dev, dtype=torch.bfloat16)
        L.call("pcs_conv3d_weight_t", L.ptr(w), cout, k ** 3, cin, L.ptr(wt), st)
        gb = V._geom(B, (g.Do, g.Ho, g.Wo), cout, cin, k, s, p, not tr)
        dx = torch.empty_like(x)
        ms = timeit(lambda: L.call("pcs_conv3d", ct.byref(gb), L.ptr(dy), L.ptr(wt), None, L.ptr(dx), L.BF16, st))
        print(f"{name:28s} dgrad {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s", flush=True)
        nb = lib.pcs_conv3d_wgrad_workspace(ct.byref(g))
        ws = torch.empty(nb // 4, device=dev)
        dw = torch.empty(cout, k ** 3 * cin, device=dev)
        db = torch.empty(cout, device=dev)
        ms = timeit(lambda: L.call("pcs_conv3d_wgrad", ct.byref(g), L.ptr(x), L.ptr(dy), L.ptr(ws), nb, L.ptr(dw),
                                   L.ptr(db), st))
        print(f"{name:28s} wgrad {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()

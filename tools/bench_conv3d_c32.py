"""The 32-channel level of BASELINE configs[1]'s U-Net (128^3 grid, 32 -> 64 -> 128 channels) on
32-channel tiles against the same layers run on zero-padded 64-channel operands (the Python
layer's behaviour before 32-channel tiles): forward + backward (input, weight and bias
gradients) per layer through pcs_amd.voxel, median of 5 after a warm-up.  Timing only.

    python tools/bench_conv3d_c32.py [B] [G]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd.voxel as V  # noqa: E402


def step_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def layer(B, gin, cin, cout, k, s, p, tr, pad_to, dev):
    """fwd + bwd of one layer; pad_to = 64 emulates the zero-padded path (operands built padded,
    the padded output channels sliced off, as the old layer did)."""
    ci, co = (pad_to or cin), (pad_to or cout)
    ci, co = max(ci, cin), max(co, cout)
    x = torch.randn(B, *gin, ci, device=dev).to(torch.bfloat16).requires_grad_()
    w = torch.randn((ci, co, k, k, k) if tr else (co, ci, k, k, k), device=dev).mul_(0.05).requires_grad_()
    b = torch.zeros(co, device=dev, requires_grad=True)

    def run():
        f = V.conv_transpose3d if tr else V.conv3d
        y = f(x, w, b, s, p)
        y = y[..., :cout] if co != cout else y
        y.float().sum().backward()
    return step_ms(run)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    dev = torch.device("cuda")
    rows = ((3, 1, 1, False, (G,) * 3, 32, 32, "3x3x3 32->32"),
            (2, 2, 0, False, (G,) * 3, 32, 64, "2x2x2/2 down 32->64"),
            (2, 2, 0, True, (G // 2,) * 3, 64, 32, "2x2x2/2 up 64->32"),
            (3, 1, 1, False, (G,) * 3, 64, 32, "3x3x3 64->32 (after the skip concat)"))
    print(f"B={B} G={G}: fwd + bwd per layer, ms (32-channel tiles / zero-padded to 64)", flush=True)
    for k, s, p, tr, gin, cin, cout, name in rows:
        nat = layer(B, gin, cin, cout, k, s, p, tr, pad_to=None, dev=dev)
        pad = layer(B, gin, cin, cout, k, s, p, tr, pad_to=64, dev=dev)
        print(f"{name:40s} {nat:8.3f} / {pad:8.3f}  ({pad / nat:.2f}x)", flush=True)


if __name__ == "__main__":
    main()

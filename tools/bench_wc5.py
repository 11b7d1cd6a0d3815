"""Micro-benchmark of conv5's R = dz5^T relu(bn4(y4)) (pcs_wgrad RAW / BNRELU, Cin 128; the
LDS-DMA stream of csrc/wgrad_c5.hip) at cfg2.  Alternate builds: PCS_LIB=path."""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402

B, N = 4, 128 ** 3
M = B * N
dev = torch.device("cuda")
dz = (torch.randn(M, 1024, device=dev) * 0.1).to(torch.bfloat16)
y4 = torch.randn(M, 128, device=dev).to(torch.bfloat16)
s, t = torch.rand(128, device=dev) + 0.5, torch.randn(128, device=dev) * 0.3
R = torch.empty(1024, 128, device=dev)
a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=1024, Cin=128, dtype=L.BF16, splits_per_scene=0,
                dy_mode=L.PRO_RAW, x_mode=L.PRO_BNRELU, x_keep_scale=1.0, dW=R.data_ptr(), ldw=0, flags=0)
a.dZ, a.X, a.s, a.t = dz.data_ptr(), y4.data_ptr(), s.data_ptr(), t.data_ptr()
ws = torch.empty(L.load().pcs_wgrad_workspace(ct.byref(a)) // 4, device=dev)
a.partial = ws.data_ptr()
colsum = torch.empty(1024, device=dev)


def run(s1):
    a.dy_colsum = colsum.data_ptr() if s1 else None   # S1 of dz5 (the dy_colsum instantiation)
    fn = lambda: L.call("pcs_wgrad", ct.byref(a), L.stream_ptr())   # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"conv5 R{' + S1' if s1 else ''}: {ms:.3f} ms  {M * (1024 + 128) * 2 / 1e9 / ms:.2f} TB/s", flush=True)


for _ in range(3):
    run(False)
    run(True)

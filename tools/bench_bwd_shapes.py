"""Time the backward GEMMs of seg_conv2 / seg_conv3 / conv5 at cfg2 on the 256x256 kernels
(flags 0) and the generic 128-row kernels (FLAG_GENERIC):  python tools/bench_bwd_shapes.py"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402
from bench_shapes import timeit  # noqa: E402


def dgrad(B, N, cout, cin, mask, flags):
    dev = torch.device("cuda")
    M = B * N
    dz = (torch.randn(M, cout, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    yp = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    Wt = (torch.randn(cin, cout, device=dev) * 0.05).to(torch.bfloat16)
    out = torch.empty(M, cin, device=dev, dtype=torch.bfloat16)
    v = lambda n: torch.rand(n, device=dev) + 0.5   # noqa: E731
    bits = torch.randint(0, 256, (M, cin // 8), device=dev, dtype=torch.uint8) if mask else None
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=cout, Ncols=cin, dtype=L.BF16, prologue=L.PRO_BWD,
                   epilogue=L.EPI_DGRAD, chunks_per_scene=0, flags=flags, A=dz.data_ptr(), W=Wt.data_ptr(),
                   C=out.data_ptr(), a_keep_scale=1.0, c_keep_scale=1.0 / 0.7)
    L.load().pcs_gemm_geometry(ct.byref(a))
    st = torch.empty(B * a.chunks_per_scene, cin, 2, device=dev)
    keep = [v(cout), v(cout), v(cout), v(cin), v(cin), v(cin), v(cin)]
    a.A2, a.pa, a.pb, a.pc, a.Yp = y.data_ptr(), *(t.data_ptr() for t in keep[:3]), yp.data_ptr()
    a.es, a.et, a.emean, a.erstd = (t.data_ptr() for t in keep[3:])
    a.c_mask, a.stats = L.ptr(bits), st.data_ptr()
    ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
    gb = M * (2 * cout + 2 * cin) * 2 / 1e9
    print(f"dgrad {cout:4d}->{cin:4d} mask={int(mask)} flags={flags}: {ms:7.3f} ms {gb / ms * 1e3:7.1f} GB/s", flush=True)


def wgrad(B, N, cout, cin, mask, flags):
    dev = torch.device("cuda")
    M = B * N
    dz = (torch.randn(M, cout, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    v = lambda n: torch.rand(n, device=dev) + 0.5   # noqa: E731
    co = [v(cout), v(cout), v(cout), v(cin), v(cin)]
    bits = torch.randint(0, 256, (M, cin // 8), device=dev, dtype=torch.uint8) if mask else None
    dW = torch.empty(cout, cin, device=dev)
    a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=cout, Cin=cin, dtype=L.BF16, splits_per_scene=0,
                    dy_mode=L.PRO_BWD, x_mode=L.PRO_BNRELU, x_keep_scale=1.0 / 0.7, dW=dW.data_ptr(), ldw=0,
                    flags=flags, dZ=dz.data_ptr(), Y=y.data_ptr(), X=x.data_ptr())
    a.alpha, a.beta, a.gamma, a.s, a.t = (t.data_ptr() for t in co)
    a.x_mask = L.ptr(bits)
    nbytes = L.load().pcs_wgrad_workspace(ct.byref(a))
    ws = torch.empty(nbytes // 4, device=dev)
    a.partial = ws.data_ptr()
    ms = timeit(lambda: L.call("pcs_wgrad", ct.byref(a), L.stream_ptr()))
    gb = M * (2 * cout + cin) * 2 / 1e9
    print(f"wgrad {cout:4d}x{cin:4d} mask={int(mask)} flags={flags} sps={a.splits_per_scene}: {ms:7.3f} ms "
          f"{gb / ms * 1e3:7.1f} GB/s", flush=True)


def main():
    B, N = 4, 128 ** 3
    for cout, cin, mask in [(256, 512, True), (128, 256, True)]:
        for flags in (0, L.FLAG_GENERIC):
            dgrad(B, N, cout, cin, mask, flags)
        for flags in (0, L.FLAG_GENERIC):
            wgrad(B, N, cout, cin, mask, flags)


if __name__ == "__main__":
    main()

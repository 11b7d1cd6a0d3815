"""Micro-benchmark of the fused seg_conv2 / seg_conv3 input + weight gradient
(pcs_dgrad_wgrad_bn: csrc/fused_seg4.hip; SEG_SMALL=1 the conv2-4 shapes of csrc/fused_bwd.hip, SEG_ADD=1 with an addend) at cfg2 (4 x 128^3 rows), with dropout bits.
    python tools/bench_seg.py [reps]"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


def fused(B, N, cout, cin, reps, mask=True):
    dev = torch.device("cuda")
    M = B * N
    dz = (torch.randn(M, cout, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    yp = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    Wt = (torch.randn(cin, cout, device=dev) * 0.05).to(torch.bfloat16)
    out = torch.empty(M, cin, device=dev, dtype=torch.bfloat16)
    bits = torch.randint(0, 256, (M, cin // 8), device=dev, dtype=torch.uint8)
    v = lambda n: torch.rand(n, device=dev) + 0.5   # noqa: E731
    keep = [v(cout), v(cout), v(cout), v(cin), v(cin), v(cin), v(cin)]
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=cout, Ncols=cin, dtype=L.BF16, prologue=L.PRO_BWD,
                   epilogue=L.EPI_DGRAD, chunks_per_scene=0, A=dz.data_ptr(), W=Wt.data_ptr(), C=out.data_ptr(),
                   a_keep_scale=1.0, c_keep_scale=1.0 / 0.7, flags=int(os.environ.get("SEG_FLAGS", "0")))
    a.A2, a.pa, a.pb, a.pc, a.Yp = y.data_ptr(), *(t.data_ptr() for t in keep[:3]), yp.data_ptr()
    a.es, a.et, a.emean, a.erstd = (t.data_ptr() for t in keep[3:])
    if mask:
        a.c_mask = bits.data_ptr()
    elif os.environ.get("SEG_ADD"):   # conv3's backward: + seg_conv1's input gradient dA2
        add = torch.randn(M, cin, device=dev).to(torch.bfloat16)
        a.addend = add.data_ptr()
    nbytes = L.load().pcs_dgrad_wgrad_bn_workspace(ct.byref(a))
    st = torch.empty(B * a.chunks_per_scene, cin, 2, device=dev)
    ws = torch.empty(nbytes // 4, device=dev)
    dW = torch.empty(cout, cin, device=dev)
    a.stats = st.data_ptr()
    ms = timeit(lambda: L.call("pcs_dgrad_wgrad_bn", ct.byref(a), ws.data_ptr(), dW.data_ptr(), 0, L.stream_ptr()), reps)
    gb = M * (2 * cout + 2 * cin + cin / 8) * 2 / 1e9
    tf = 4.0 * M * cout * cin / 1e12
    print(f"fused {cout:4d}x{cin:4d}{' mask' if mask else ''}: {ms:7.3f} ms  {gb / ms:6.2f} TB/s  {tf / ms * 1e3:7.1f} TF/s", flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    B, N = 4, 128 ** 3
    shapes = [(256, 512, True), (128, 256, True)]
    if os.environ.get("SEG_SMALL"):   # conv4 (128 -> 64) / conv2-3 (64 -> 64) backward
        shapes = [(128, 64, False), (64, 64, False)]
    for cout, cin, mk in shapes:
        fused(B, N, cout, cin, reps, mk)


if __name__ == "__main__":
    main()

"""Micro-benchmark of conv5's folded input gradient (csrc/fused_c5.hip, the PRO_CAT / EPI_DGRAD
call of the training step) at cfg2 (4 x 128^3 rows): dz5 [M, 1024] and y4 [M, 128] bf16 in,
dA4 [M, 128] bf16 out, S1 / S2 per chunk.  Alternate builds: PCS_LIB=path.
    python tools/bench_c5.py [reps]"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B, N = 4, 128 ** 3
    M = B * N
    dev = torch.device("cuda")
    dz5 = torch.empty(M, 1024, device=dev, dtype=torch.bfloat16)
    for r0 in range(0, M, 1 << 20):
        dz5[r0:r0 + (1 << 20)] = torch.randn(min(1 << 20, M - r0), 1024, device=dev) * 0.1
    y4 = torch.randn(M, 128, device=dev).to(torch.bfloat16)
    Ws = (torch.randn(128, 1024, device=dev) * 0.03).to(torch.bfloat16)
    H4 = (torch.randn(128, 128, device=dev) * 0.05).to(torch.bfloat16)
    v = lambda o=0.0: torch.randn(128, device=dev) * 0.3 + o   # noqa: E731
    keep = [v(1.0), v(), v(), v(1.0), v(), v(), v(1.0).abs()]
    out = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=1152, Ncols=128, dtype=L.BF16, prologue=L.PRO_CAT,
                   epilogue=L.EPI_DGRAD, chunks_per_scene=0, A=dz5.data_ptr(), W=Ws.data_ptr(), C=out.data_ptr(),
                   a_keep_scale=1.0, c_keep_scale=1.0)
    a.K1 = 1024
    a.A2, a.W2, a.Yp = y4.data_ptr(), H4.data_ptr(), y4.data_ptr()
    a.pa, a.pb, a.bias, a.es, a.et, a.emean, a.erstd = (t.data_ptr() for t in keep)
    L.load().pcs_gemm_geometry(ct.byref(a))
    st = torch.empty(B * a.chunks_per_scene, 128, 2, device=dev)
    a.stats = st.data_ptr()
    fn = lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr())   # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gb = M * (1024 + 128 + 128) * 2 / 1e9
        print(f"c5 dgrad: {ms:7.3f} ms  {gb / ms:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()

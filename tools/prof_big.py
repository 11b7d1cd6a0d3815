"""One pcs_gemm variant at the cfg2 global_feat shape, for rocprofv3 counter passes:
    python tools/prof_big.py [fwd|dgrad|wgrad] [reps]"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    B, N, K, Nc = 4, 128 ** 3, 1024, 1024
    M = B * N
    dev = torch.device("cuda")
    lib = L.load()
    A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    X = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    W = (torch.randn(Nc, K, device=dev) * 0.03).to(torch.bfloat16)
    C = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    s, t = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
    be, ga = torch.randn(K, device=dev) * 1e-3, torch.randn(K, device=dev) * 1e-3
    am = (torch.randint(0, N, (B, K), device=dev, dtype=torch.int32)
          + (torch.arange(B, device=dev, dtype=torch.int32) * N)[:, None])
    sp = torch.randn(B, K, device=dev)
    if which == "wgrad":
        a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=Nc, Cin=K, dtype=L.BF16, splits_per_scene=0,
                        dy_mode=L.PRO_BWD_POOL, x_mode=L.PRO_BNRELU, x_keep_scale=1.0)
        ws = torch.empty(lib.pcs_wgrad_workspace(ct.byref(a)) // 4, device=dev)
        dW = torch.empty(Nc, K, device=dev)
        a.Y, a.X, a.beta, a.gamma, a.pool_idx, a.pool_coef = (L.ptr(v) for v in (A, X, be, ga, am, sp))
        a.s, a.t, a.partial, a.dW = L.ptr(s), L.ptr(t), L.ptr(ws), L.ptr(dW)
        fn = lambda: L.call("pcs_wgrad", ct.byref(a), L.stream_ptr())  # noqa: E731
    else:
        pro, epi = (L.PRO_BNRELU, L.EPI_FWD) if which == "fwd" else (L.PRO_BWD_POOL, L.EPI_RAW)
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=pro,
                       epilogue=epi, chunks_per_scene=0)
        lib.pcs_gemm_geometry(ct.byref(a))
        a.A, a.W, a.C = A.data_ptr(), W.data_ptr(), C.data_ptr()
        if which == "fwd":
            a.pa, a.pb = L.ptr(s), L.ptr(t)
        else:
            a.pb, a.pc, a.pool_idx, a.pool_coef = L.ptr(be), L.ptr(ga), L.ptr(am), L.ptr(sp)
        fn = lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr())  # noqa: E731
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("done", which, reps)


if __name__ == "__main__":
    main()

"""Time pcs_gemm at the cfg2 mid-layer shapes with epilogue features toggled:
    python tools/bench_shapes.py"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


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


def run(name, B, N, K, Nc, stats, store, flags=0, epi=None):
    dev = torch.device("cuda")
    lib = L.load()
    M = B * N
    A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    W = (torch.randn(Nc, K, device=dev) * 0.03).to(torch.bfloat16)
    C = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    s, t = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
    s2, t2 = torch.rand(Nc, device=dev) + 0.5, torch.randn(Nc, device=dev) * 0.1
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=L.PRO_BNRELU,
                   epilogue=L.EPI_FWD if epi is None else epi, chunks_per_scene=0, flags=flags)
    lib.pcs_gemm_geometry(ct.byref(a))
    st = torch.empty(B * a.chunks_per_scene, Nc, 2, device=dev)
    a.A, a.W, a.C, a.pa, a.pb = A.data_ptr(), W.data_ptr(), C.data_ptr() if store else None, L.ptr(s), L.ptr(t)
    a.stats = L.ptr(st) if stats else None
    if epi == L.EPI_BNRELU:
        a.es, a.et = L.ptr(s2), L.ptr(t2)
    ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
    gb = M * (K + (Nc if store else 0)) * 2 / 1e9
    print(f"{name:34s} K={K:5d} N={Nc:5d} stats={int(stats)} store={int(store)} gen={flags}: {ms:7.3f} ms "
          f"{2 * M * K * Nc / ms / 1e9:7.1f} TF/s {gb / ms * 1e3:7.1f} GB/s", flush=True)
    del A, W, C


def main():
    B, N = 4, 128 ** 3
    run("fwd bnrelu epilogue (conv5)", B, N, 128, 1024, 0, 1, epi=L.EPI_BNRELU)
    for K, Nc in [(128, 1024), (512, 256), (64, 512)]:
        for stats, store in [(1, 1), (0, 1), (0, 0)]:
            run("fwd", B, N, K, Nc, stats, store)
        run("fwd generic", B, N, K, Nc, 1, 1, flags=L.FLAG_GENERIC)


if __name__ == "__main__":
    main()

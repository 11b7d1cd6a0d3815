"""Micro-benchmark of conv5's BN+ReLU pass at the cfg2 shape (M = 4 x 128^3 rows, K = 128 ->
1024 columns, column sums on): the W-resident LDS-DMA stream (gemm_wres.hip) against the
register-staged 256x256 kernel (FLAG_NO_GLDS), bf16 and fp8 stores.  Prints ms and the
algorithmic HBM rate (y4 read once + a5 written)."""
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


def main():
    B, N, K, Nc = 4, 128 ** 3, 128, 1024
    M = B * N
    dev = torch.device("cuda")
    lib = L.load()
    Y = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(Nc, K, device=dev) * 0.1).to(torch.bfloat16)
    ps, pt = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.2
    es, et = torch.randn(Nc, device=dev), torch.randn(Nc, device=dev) * 0.3
    for c8 in (False, True):
        out = torch.empty(M, Nc, device=dev, dtype=torch.uint8 if c8 else torch.bfloat16)
        for fl, tag in ((0, "wres"), (L.FLAG_NO_GLDS, "big ")):
            flags = fl | (L.FLAG_C_FP8 if c8 else 0)
            a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=L.PRO_BNRELU,
                           epilogue=L.EPI_BNRELU, chunks_per_scene=0, flags=flags)
            lib.pcs_gemm_geometry(ct.byref(a))
            st = torch.empty(B * a.chunks_per_scene, Nc, 2, device=dev)
            a.A, a.W, a.C, a.pa, a.pb, a.es, a.et, a.stats = (Y.data_ptr(), W.data_ptr(), out.data_ptr(), ps.data_ptr(),
                                                               pt.data_ptr(), es.data_ptr(), et.data_ptr(), st.data_ptr())
            ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
            gb = (M * K * 2 + M * Nc * (1 if c8 else 2)) / 1e9
            print(f"[{tag}] conv5 BN+ReLU pass, {'fp8' if c8 else 'bf16'} store  {ms:7.3f} ms  {gb / ms:6.2f} TB/s",
                  flush=True)


if __name__ == "__main__":
    main()

"""Micro-benchmark of global_feat's two bf16 GEMMs at the cfg2 shape (M = 4 x 128^3 rows,
1024 x 1024, a5-like ReLU operand on random data): the four-wave 32x32x16 kernel
(csrc/gemm_w4.hip, the default) against the 8-wave 16x16x32 kernel (csrc/gemm_glds.hip,
the default), alternating, several rounds in one process.  Prints ms and TF/s per variant
and the agreement of the two input gradients.  PCS_LIB selects another build (ablations)."""
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
    B = int(os.environ.get("W4_B", "4"))
    N = 128 ** 3
    M = B * N
    K = Nc = 1024
    rounds = int(os.environ.get("W4_ROUNDS", "3"))
    dev = torch.device("cuda")
    lib = L.load()
    A = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    for r0 in range(0, M, 1 << 20):   # random a5-like operand, generated in slices
        A[r0:r0 + (1 << 20)] = torch.relu(torch.randn(min(1 << 20, M - r0), K, device=dev))
    W = (torch.randn(Nc, K, device=dev) * 0.03).to(torch.bfloat16)
    H = (torch.randn(K, K, device=dev) * 0.03).to(torch.bfloat16)
    gsign = torch.randn(Nc, device=dev)
    Ws = torch.empty_like(W)
    L.call("pcs_sign_rows", L.ptr(W), L.BF16, Nc, K, L.ptr(gsign), L.ptr(Ws), L.stream_ptr())
    c = torch.randn(Nc, device=dev) * 0.1
    C1 = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    C2 = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    flops = 2.0 * M * K * Nc

    def args(epi, flags):
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=L.PRO_RAW,
                       epilogue=epi, chunks_per_scene=0, flags=flags)
        lib.pcs_gemm_geometry(ct.byref(a))
        return a

    keep = []

    def fwd(flags):
        a = args(L.EPI_FWD, flags | L.FLAG_POOL_SIGNED_W)
        pool = torch.empty(B * a.chunks_per_scene, Nc, 4, device=dev)
        keep.append(pool)
        a.A, a.W, a.C, a.pool, a.es = A.data_ptr(), Ws.data_ptr(), None, pool.data_ptr(), gsign.data_ptr()
        return lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()), pool

    def dgrad(flags, out, stats=False):
        a = args(L.EPI_DGRAD, flags)
        a.A, a.W, a.C, a.Yp, a.bias = A.data_ptr(), H.data_ptr(), out.data_ptr(), A.data_ptr(), c.data_ptr()
        if stats:
            st = torch.empty(B * a.chunks_per_scene, Nc, 2, device=dev)
            keep.append(st)
            a.stats = st.data_ptr()
        return lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr())

    variants = [
        ("dgrad w4 (mask + store + bias)", dgrad(L.FLAG_W4, C1)),
        ("dgrad glds8 (mask + store + bias)", dgrad(0, C2)),
        ("dgrad glds8 + S1 (the r03 training call)", dgrad(0, C2, stats=True)),
    ]
    f4, p4 = fwd(L.FLAG_W4)
    f8, p8 = fwd(0)
    variants += [("fwd w4 (signed-W max-pool)", f4), ("fwd glds8 (signed-W max-pool)", f8)]
    if os.environ.get("W4_ONLY"):   # ablation builds: the two w4 calls only
        variants = [variants[0], variants[3]]
        rounds = 1
    for r in range(rounds):
        for name, fn in variants:
            ms = timeit(fn)
            print(f"[{r}] {name:44s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s  {flops / ms / 1e9 / 2516.6:6.3f}",
                  flush=True)
    if os.environ.get("W4_ONLY"):
        return
    variants[0][1]()   # w4 -> C1
    variants[1][1]()   # glds8 -> C2
    torch.cuda.synchronize()
    same = (C1.view(torch.int16) == C2.view(torch.int16)).float().mean().item()
    d = (C1.float() - C2.float()).abs().max().item()
    print(f"dgrad w4 vs glds8: bitwise-equal fraction {same:.5f}, max |diff| {d:.3e}, max |dz| "
          f"{C2.float().abs().max().item():.3e}")
    pos = gsign[None, :] > 0
    rw4 = torch.where(pos, p4[..., 1], p4[..., 3]).view(torch.int32)
    rg8 = torch.where(pos, p8[..., 1], p8[..., 3]).view(torch.int32)
    print(f"fwd pool rows equal: {(rw4 == rg8).float().mean().item():.5f}")


if __name__ == "__main__":
    main()

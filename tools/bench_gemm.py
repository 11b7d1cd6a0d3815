"""Micro-benchmark of single pcs_gemm / pcs_wgrad launches at the cfg2 global_feat shape
(M = 4 x 128^3, 1024 x 1024, bf16) with epilogue features switched off one by one."""
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    N = 128 ** 3
    M = B * N
    K = Nc = 1024
    dev = torch.device("cuda")
    lib = L.load()
    A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    W = (torch.randn(Nc, K, device=dev) * 0.03).to(torch.bfloat16)
    C = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    s = torch.rand(K, device=dev) + 0.5
    t = torch.randn(K, device=dev) * 0.1
    flops = 2.0 * M * K * Nc

    def make(flags=0, stats=True, pool=True, store=True, pro=L.PRO_BNRELU):
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=pro,
                       epilogue=L.EPI_FWD, chunks_per_scene=0, flags=flags)
        lib.pcs_gemm_geometry(ct.byref(a))
        nch = B * a.chunks_per_scene
        st = torch.empty(nch, Nc, 2, device=dev)
        pl = torch.empty(nch, Nc, 4, device=dev)
        a.A, a.W, a.C = A.data_ptr(), W.data_ptr(), C.data_ptr() if store else None
        a.pa, a.pb = s.data_ptr(), t.data_ptr()
        a.stats = st.data_ptr() if stats else None
        a.pool = pl.data_ptr() if pool else None
        keep = (st, pl)
        return a, keep

    for name, kw in [("big full (bnrelu+stats+pool+store)", {}),
                     ("big no pool", dict(pool=False)),
                     ("big no stats/pool", dict(pool=False, stats=False)),
                     ("big no stats/pool/store", dict(pool=False, stats=False, store=False)),
                     ("big raw prologue, nothing", dict(pool=False, stats=False, store=False, pro=L.PRO_RAW)),
                     ("generic full", dict(flags=L.FLAG_GENERIC))]:
        a, keep = make(**kw)
        try:
            ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
            print(f"{name:40s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s", flush=True)
        except L.PcsError as e:
            print(f"{name:40s} n/a ({e})")


if __name__ == "__main__":
    main()

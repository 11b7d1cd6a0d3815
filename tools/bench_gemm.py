"""Micro-benchmark of single pcs_gemm launches at the cfg2 global_feat shape (M = 4 x 128^3,
1024 x 1024, bf16): the 256x256 kernel with each epilogue feature on/off, against the
separate streaming passes (pcs_colstats, pcs_bnrelu_bwd) those features replace."""
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
    Y5 = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    W = (torch.randn(Nc, K, device=dev) * 0.03).to(torch.bfloat16)
    C = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    vK = lambda lo, sc: torch.rand(K, device=dev) * sc + lo  # noqa: E731
    s, t, al, be, ga = vK(0.5, 1), vK(-0.1, 0.2), vK(0.5, 1), vK(-1e-3, 2e-3), vK(-1e-3, 2e-3)
    em, er = vK(-0.1, 0.2), vK(1, 1)
    am = torch.randint(0, N, (B, K), device=dev, dtype=torch.int32) + \
        (torch.arange(B, device=dev, dtype=torch.int32) * N)[:, None]
    sp = torch.randn(B, K, device=dev)
    flops = 2.0 * M * K * Nc

    def run(name, pro, epi, flags=0, **kw):
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=pro,
                       epilogue=epi, chunks_per_scene=0, flags=flags)
        lib.pcs_gemm_geometry(ct.byref(a))
        nch = B * a.chunks_per_scene
        keep = {}
        if kw.pop("stats", False):
            keep["stats"] = torch.empty(nch, Nc, 2, device=dev)
        if kw.pop("pool", False):
            keep["pool"] = torch.empty(nch, Nc, 4, device=dev)
        kw.update(keep)
        a.A, a.W, a.C = A.data_ptr(), W.data_ptr(), C.data_ptr()
        for k, v in kw.items():
            setattr(a, k, L.ptr(v))
        try:
            ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
            print(f"{name:44s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s", flush=True)
        except L.PcsError as e:
            print(f"{name:44s} n/a ({e})")

    fwd = dict(pa=s, pb=t)
    run("fwd store", L.PRO_BNRELU, L.EPI_FWD, **fwd)
    run("fwd store, RAW prologue (no BN+ReLU)", L.PRO_RAW, L.EPI_FWD)
    run("fwd store+stats", L.PRO_BNRELU, L.EPI_FWD, stats=True, **fwd)
    run("fwd store+stats+pool", L.PRO_BNRELU, L.EPI_FWD, stats=True, pool=True, **fwd)
    run("fwd stats+pool (no store)", L.PRO_BNRELU, L.EPI_FWD, stats=True, pool=True, C=None, **fwd)
    cps = ct.c_int32(0)
    rpc = lib.pcs_colstats_geometry(B, N, Nc, ct.byref(cps))
    st = torch.empty(B * cps.value, Nc, 2, device=dev)
    pl = torch.empty(B * cps.value, Nc, 4, device=dev)
    ms = timeit(lambda: L.call("pcs_colstats", L.ptr(C), B, N, Nc, L.BF16, cps.value, rpc, L.ptr(st),
                               L.ptr(pl), L.stream_ptr()))
    print(f"{'colstats (stats+pool pass)':44s} {ms:8.3f} ms")
    pool = dict(pb=be, pc=ga, pool_idx=am, pool_coef=sp)
    run("dgrad raw (pool prologue)", L.PRO_BWD_POOL, L.EPI_RAW, **pool)
    run("dgrad fused DGRAD epilogue", L.PRO_BWD_POOL, L.EPI_DGRAD, stats=True, Yp=Y5, es=s, et=t,
        emean=em, erstd=er, **pool)
    ms = timeit(lambda: L.call("pcs_bnrelu_bwd", L.ptr(C), L.ptr(Y5), None, None, 1.0, L.ptr(s), L.ptr(t),
                               L.ptr(em), L.ptr(er), B, N, Nc, L.BF16, cps.value, rpc, L.ptr(st),
                               L.stream_ptr()))
    print(f"{'bnrelu_bwd pass':44s} {ms:8.3f} ms")
    run("generic fwd store+stats+pool", L.PRO_BNRELU, L.EPI_FWD, flags=L.FLAG_GENERIC, stats=True,
        pool=True, **fwd)


if __name__ == "__main__":
    main()

"""Micro-benchmark of the global_feat GEMMs at the cfg2 shape (M = 4 x 128^3 rows, 1024 x 1024,
bf16, a5-like operand) with each epilogue feature on/off: the LDS-DMA kernel (gemm_glds.hip)
against the register-staged 256x256 kernel (FLAG_NO_GLDS).  Prints ms and TF/s per variant.
GLDS_GRAM=1: the Gram of a5 instead; GLDS_FP8=1: the fp8 (MX-scaled MFMA) forms of the
LDS-DMA forward, input gradient and Gram."""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


def timeit(fn, reps=4):
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
    A = torch.relu(torch.randn(M, K, device=dev)).to(torch.bfloat16)
    W = (torch.randn(Nc, K, device=dev) * 0.03).to(torch.bfloat16)
    C = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    c = torch.randn(Nc, device=dev) * 0.1
    am = torch.randint(0, N, (B, K), device=dev, dtype=torch.int32) + \
        (torch.arange(B, device=dev, dtype=torch.int32) * N)[:, None]
    sp = torch.randn(B, K, device=dev)
    Wsp = torch.randn(K, Nc, device=dev) * 0.03
    gsign = torch.randn(Nc, device=dev)
    flops = 2.0 * M * K * Nc

    def run(name, epi, flags=0, **kw):
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=L.PRO_RAW,
                       epilogue=epi, chunks_per_scene=0, flags=flags)
        lib.pcs_gemm_geometry(ct.byref(a))
        nch = B * a.chunks_per_scene
        keep = {}
        if kw.pop("stats", False):
            keep["stats"] = torch.empty(nch, Nc, 2, device=dev)
        if kw.pop("pool", False):
            keep["pool"] = torch.empty(nch, Nc, 4, device=dev)
        kw.update(keep)
        a.A, a.W = A.data_ptr(), W.data_ptr()
        cc = kw.pop("C", None)
        a.C = cc.data_ptr() if cc is not None else None
        if kw.pop("sparse", False):
            a.pool_idx, a.pool_coef, a.pool_w, a.pool_ldw, a.pool_c = am.data_ptr(), sp.data_ptr(), Wsp.data_ptr(), Nc, K
        for k, v in kw.items():
            setattr(a, k, L.ptr(v))
        ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
        print(f"{name:52s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s", flush=True)

    if os.environ.get("GLDS_FP8"):
        A8 = A.float().clamp(max=448.0).to(torch.float8_e4m3fn).view(torch.uint8)
        del A
        W8 = torch.empty(Nc, K, dtype=torch.uint8, device=dev)
        wsc = torch.empty(Nc, dtype=torch.uint8, device=dev)
        Wf = W.float()
        L.call("pcs_quant_fp8_rows", L.ptr(Wf), Nc, K, K, L.ptr(W8), L.ptr(wsc), None, L.stream_ptr())

        def run8(name, epi, stats=True, pool=True, flags=0, **kw):
            a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=Nc, dtype=L.BF16, prologue=L.PRO_RAW,
                           epilogue=epi, chunks_per_scene=0, flags=L.FLAG_AW_FP8 | flags)
            lib.pcs_gemm_geometry(ct.byref(a))
            nch = B * a.chunks_per_scene
            keep = dict(stats=torch.empty(nch, Nc, 2, device=dev)) if stats else {}
            if epi == L.EPI_FWD and pool:
                keep["pool"] = torch.empty(nch, Nc, 4, device=dev)
            a.A, a.W, a.w_scale = A8.data_ptr(), W8.data_ptr(), wsc.data_ptr()
            for k, v in list(kw.items()) + list(keep.items()):
                setattr(a, k, L.ptr(v))
            ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
            print(f"{name:52s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s", flush=True)

        run8("[glds fp8] fwd, no epilogue work", L.EPI_FWD, stats=False, pool=False, es=gsign)
        run8("[glds fp8] fwd + stats", L.EPI_FWD, pool=False, es=gsign)
        W8u = W8
        W8s = torch.empty_like(W8)
        signed = hasattr(L, "FLAG_POOL_SIGNED_W")
        if signed:
            L.call("pcs_sign_rows", L.ptr(W8), L.FP8, Nc, K, L.ptr(gsign), L.ptr(W8s), L.stream_ptr())
        for _ in range(2):
            run8("[glds fp8] fwd + pool", L.EPI_FWD, stats=False, es=gsign)
            if signed:
                W8 = W8s
                run8("[glds fp8] fwd + pool, signed W (training path)", L.EPI_FWD, stats=False, es=gsign,
                     flags=L.FLAG_POOL_SIGNED_W)
                W8 = W8u
            run8("[glds fp8] fwd + stats + pool", L.EPI_FWD, es=gsign)
            run8("[glds fp8] dgrad: mask + store + bias + S1", L.EPI_DGRAD, C=C, Yp=A8, bias=c)
        nb2 = lib.pcs_gram_raw_workspace(M, K)
        ws2 = torch.empty(nb2 // 4, device=dev)
        G2 = torch.empty(K, K, device=dev)
        gfl = flops * 10 / 16
        for _ in range(2):
            ms = timeit(lambda: L.call("pcs_gram_raw", L.ptr(A8), M, K, L.FP8, L.ptr(ws2), nb2, L.ptr(G2),
                                       L.stream_ptr()))
            print(f"[gram fp8] LDS-DMA (pcs_gram_raw)               {ms:8.3f} ms  {gfl / ms / 1e9:8.1f} TF/s", flush=True)
        return
    if os.environ.get("GLDS_GRAM"):   # Gram of a5: register-staged 256x256 vs LDS-DMA persistent
        sps = ct.c_int32(0)
        nb = lib.pcs_gram_workspace(B, N, K, L.BF16, ct.byref(sps))
        ws = torch.empty(nb // 4, device=dev)
        G = torch.empty(K, K, device=dev)
        S = torch.empty(K, device=dev)
        nb2 = lib.pcs_gram_raw_workspace(M, K)
        ws2 = torch.empty(nb2 // 4, device=dev)
        G2 = torch.empty(K, K, device=dev)
        gfl = flops * 10 / 16
        for rep in range(3):
            ms = timeit(lambda: L.call("pcs_gram", L.ptr(A), None, None, B, N, K, L.BF16, sps.value, L.ptr(ws),
                                       L.ptr(G), L.ptr(S), L.stream_ptr()))
            print(f"[gram] register-staged (pcs_gram)                {ms:8.3f} ms  {gfl / ms / 1e9:8.1f} TF/s", flush=True)
            ms = timeit(lambda: L.call("pcs_gram_raw", L.ptr(A), M, K, L.BF16, L.ptr(ws2), nb2, L.ptr(G2), L.stream_ptr()))
            print(f"[gram] LDS-DMA persistent (pcs_gram_raw)         {ms:8.3f} ms  {gfl / ms / 1e9:8.1f} TF/s", flush=True)
        torch.cuda.synchronize()
        print("max |G - G2| / max |G|:", float((G - G2).abs().max() / G.abs().max()))
        return
    for fl, tag in ((0, "glds"), (L.FLAG_NO_GLDS, "big ")):
        run(f"[{tag}] fwd, no epilogue work", L.EPI_FWD, fl, es=gsign)
        run(f"[{tag}] fwd + stats", L.EPI_FWD, fl, stats=True, es=gsign)
        run(f"[{tag}] fwd + stats + pool", L.EPI_FWD, fl, stats=True, pool=True, es=gsign)
        run(f"[{tag}] fwd + pool", L.EPI_FWD, fl, pool=True, es=gsign)
    if hasattr(L, "FLAG_POOL_SIGNED_W"):   # the training path: W rows pre-multiplied by sign(es)
        Wu = W
        W = torch.empty_like(Wu)
        L.call("pcs_sign_rows", L.ptr(Wu), L.BF16, Nc, K, L.ptr(gsign), L.ptr(W), L.stream_ptr())
        run("[glds] fwd + pool, signed W (bf16 training path)", L.EPI_FWD, L.FLAG_POOL_SIGNED_W, pool=True,
            es=gsign)
        W = Wu
    run("[glds] dgrad: mask + store", L.EPI_DGRAD, 0, C=C, Yp=A)
    run("[glds] dgrad: mask + store + bias + S1", L.EPI_DGRAD, 0, C=C, Yp=A, bias=c, stats=True)
    run("[gen ] dgrad (generic kernel, FLAG_NO_GLDS)", L.EPI_DGRAD, L.FLAG_NO_GLDS, C=C, Yp=A, bias=c, stats=True,
        sparse=True)


if __name__ == "__main__":
    main()

"""global_feat's LDS-DMA GEMMs at the cfg2 shape (M = 4 x 128^3, K = Ncols = 1024, bf16 a5-like
operand): the input gradient (mask + store + bias + S1) and the forward (signed-W max-pool), as
the training step calls them.  Prints ms and TF/s; GF_FP8=1 runs the fp8 forms.  For A/B runs of
abtest builds (PCS_LIB) alternate processes: tools/ab_gf.sh."""
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
    B, N, K = 4, 128 ** 3, 1024
    M = B * N
    dev = torch.device("cuda")
    lib = L.load()
    fp8 = bool(os.environ.get("GF_FP8"))
    torch.manual_seed(0)
    A = torch.relu(torch.randn(M, K, device=dev)).to(torch.bfloat16)
    W = (torch.randn(K, K, device=dev) * 0.03)
    C = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    c = torch.randn(K, device=dev) * 0.1
    gsign = torch.randn(K, device=dev)
    flops = 2.0 * M * K * K
    if fp8:
        A = A.float().clamp(max=448.0).to(torch.float8_e4m3fn).view(torch.uint8)
        Wq = torch.empty(K, K, dtype=torch.uint8, device=dev)
        wsc = torch.empty(K, dtype=torch.uint8, device=dev)
        L.call("pcs_quant_fp8_rows", L.ptr(W), K, K, K, L.ptr(Wq), L.ptr(wsc), None, L.stream_ptr())
        Ws = torch.empty_like(Wq)
        L.call("pcs_sign_rows", L.ptr(Wq), L.FP8, K, K, L.ptr(gsign), L.ptr(Ws), L.stream_ptr())
        base = L.FLAG_AW_FP8
    else:
        Wq = W.to(torch.bfloat16)
        Ws = torch.empty_like(Wq)
        L.call("pcs_sign_rows", L.ptr(Wq), L.BF16, K, K, L.ptr(gsign), L.ptr(Ws), L.stream_ptr())
        wsc = None
        base = 0

    def args(epi, flags):
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=K, dtype=L.BF16, prologue=L.PRO_RAW,
                       epilogue=epi, chunks_per_scene=0, flags=base | flags)
        lib.pcs_gemm_geometry(ct.byref(a))
        return a, B * a.chunks_per_scene

    a, nch = args(L.EPI_DGRAD, 0)
    st = torch.empty(nch, K, 2, device=dev)
    a.A, a.Yp, a.W, a.C, a.bias, a.stats = A.data_ptr(), A.data_ptr(), Wq.data_ptr(), C.data_ptr(), c.data_ptr(), st.data_ptr()
    if fp8:
        a.w_scale = wsc.data_ptr()
    f, nchf = args(L.EPI_FWD, L.FLAG_POOL_SIGNED_W)
    pool = torch.empty(nchf, K, 4, device=dev)
    f.A, f.W, f.pool, f.es = A.data_ptr(), Ws.data_ptr(), pool.data_ptr(), gsign.data_ptr()
    if fp8:
        f.w_scale = wsc.data_ptr()
    for _ in range(2):
        ms = timeit(lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr()))
        print(f"dgrad {ms:8.3f} ms {flops / ms / 1e9:8.1f} TF/s", flush=True)
        ms = timeit(lambda: L.call("pcs_gemm", ct.byref(f), L.stream_ptr()))
        print(f"fwd   {ms:8.3f} ms {flops / ms / 1e9:8.1f} TF/s", flush=True)
    if os.environ.get("GF_DUMP"):
        torch.cuda.synchronize()
        torch.save({"C": C[:65536].cpu(), "st": st.cpu(), "pool": pool.cpu()}, os.environ["GF_DUMP"])


if __name__ == "__main__":
    main()

"""Run the stamped diagnostic build of global_feat's GEMMs (tools/variants/gf_stamps.py,
PCS_LIB=abtest/gf_stamps/libpcs.so) at the cfg2 shape and print each segment's share of the
wave cycles, per wave half, for the input gradient and the forward.  Diagnostic only."""
import ctypes as ct
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402

SEG = ["p1.lgkm", "prep2", "prep3", "prep4", "open1", "open2", "open3", "open4", "mfma", "close", "epi", "p1.Blo+mask", "p1.issue", "p1.vmcnt", "p1.loop", "p1.Alo"]


def main():
    B, N, K = 4, 128 ** 3, 1024
    M = B * N
    dev = torch.device("cuda")
    lib = L.load()
    lib.pcs_debug_stamps.restype = ct.c_int
    lib.pcs_debug_stamps.argtypes = [ct.c_void_p, ct.c_int64]
    fp8 = bool(os.environ.get("GF_FP8"))   # the e4m3 forms (MX-scaled MFMA)
    torch.manual_seed(0)
    A = torch.relu(torch.randn(M, K, device=dev)).to(torch.bfloat16)
    W32 = torch.randn(K, K, device=dev) * 0.03
    W = W32.to(torch.bfloat16)
    C = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    c = torch.randn(K, device=dev) * 0.1
    gsign = torch.randn(K, device=dev)
    wsc = None
    if fp8:
        A = A.float().clamp(max=448.0).to(torch.float8_e4m3fn).view(torch.uint8)
        W = torch.empty(K, K, dtype=torch.uint8, device=dev)
        wsc = torch.empty(K, dtype=torch.uint8, device=dev)
        L.call("pcs_quant_fp8_rows", L.ptr(W32), K, K, K, L.ptr(W), L.ptr(wsc), None, L.stream_ptr())
    Ws = torch.empty_like(W)
    L.call("pcs_sign_rows", L.ptr(W), L.FP8 if fp8 else L.BF16, K, K, L.ptr(gsign), L.ptr(Ws), L.stream_ptr())
    for mode in ("dgrad", "fwd"):
        epi = L.EPI_DGRAD if mode == "dgrad" else L.EPI_FWD
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=K, dtype=L.BF16, prologue=L.PRO_RAW, epilogue=epi,
                       chunks_per_scene=0, flags=(0 if mode == "dgrad" else L.FLAG_POOL_SIGNED_W) |
                       (L.FLAG_AW_FP8 if fp8 else 0))
        lib.pcs_gemm_geometry(ct.byref(a))
        nch = B * a.chunks_per_scene
        st = torch.empty(nch, K, 2, device=dev)
        pool = torch.empty(nch, K, 4, device=dev)
        if mode == "dgrad":
            a.A, a.Yp, a.W, a.C, a.bias, a.stats = A.data_ptr(), A.data_ptr(), W.data_ptr(), C.data_ptr(), c.data_ptr(), st.data_ptr()
        else:
            a.A, a.W, a.pool, a.es = A.data_ptr(), Ws.data_ptr(), pool.data_ptr(), gsign.data_ptr()
        if fp8:
            a.w_scale = wsc.data_ptr()
        for _ in range(2):
            L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
        torch.cuda.synchronize()
        nb = (K // 256) * nch
        buf = np.zeros((4096 * 8, 16), dtype=np.uint64)
        assert lib.pcs_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
        s = buf[:nb * 8].astype(np.float64).reshape(nb, 8, 16)   # [workgroup][wave][segment]
        for half, name in ((slice(0, 4), "half 0"), (slice(4, 8), "half 1")):
            tot = s[:, half, :].sum(axis=(0, 1))
            share = tot / tot.sum()
            per_wave_us = tot.sum() / (nb * 4) / 2.1e3
            print(f"{'fp8 ' if fp8 else ''}{mode} {name}: " + "  ".join(f"{SEG[i]} {share[i]:.3f}" for i in range(16)) +
                  f"  (mean wave {per_wave_us:.0f} us at 2.1 GHz)", flush=True)


if __name__ == "__main__":
    main()

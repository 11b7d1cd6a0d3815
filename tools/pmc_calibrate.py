"""Known-byte launches for calibrating rocprofv3 FETCH_SIZE / WRITE_SIZE on our access
patterns (MI355X guide: only 16 B/lane streaming reads are pre-calibrated):
  1) pcs_colstats over Y [M, 1024] bf16: reads exactly M*1024*2 bytes
  2) 256x256 GEMM with one column block (Ncols = 256): A [M, 1024] read once (+ 0.5 MB W),
     C [M, 256] written once
Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE)."""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402

B, N, K = 4, 128 ** 3, 1024
M = B * N
dev = torch.device("cuda")
lib = L.load()
Y = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
cps = ct.c_int32(0)
rpc = lib.pcs_colstats_geometry(B, N, K, ct.byref(cps))
st = torch.empty(B * cps.value, K, 2, device=dev)
pl = torch.empty(B * cps.value, K, 4, device=dev)
L.call("pcs_colstats", L.ptr(Y), B, N, K, L.BF16, cps.value, rpc, L.ptr(st), L.ptr(pl), L.stream_ptr())
W = (torch.randn(256, K, device=dev) * 0.03).to(torch.bfloat16)
C = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
s, t = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=256, dtype=L.BF16, prologue=L.PRO_BNRELU,
               epilogue=L.EPI_FWD, chunks_per_scene=0)
lib.pcs_gemm_geometry(ct.byref(a))
a.A, a.W, a.C, a.pa, a.pb = Y.data_ptr(), W.data_ptr(), C.data_ptr(), L.ptr(s), L.ptr(t)
L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
torch.cuda.synchronize()
print(f"colstats reads {M * K * 2 / 1e9:.3f} GB; gemm reads {M * K * 2 / 1e9:.3f} GB A, writes {M * 256 * 2 / 1e9:.3f} GB")

"""Micro-benchmark of pcs_gram at C = 128 (fwd_stats:conv5: the Gram of relu(bn4(y4)) and its column
sums) at cfg2 (4 x 128^3 rows).  Alternate builds: PCS_LIB=path.
    python tools/bench_gram128.py [reps]"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B, N, C = 4, 128 ** 3, 128
    dev = torch.device("cuda")
    Y = torch.randn(B * N, C, device=dev).to(torch.bfloat16)
    s, t = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3
    sps = ct.c_int32(0)
    nbytes = L.load().pcs_gram_workspace(B, N, C, L.BF16, ct.byref(sps))
    ws = torch.empty(nbytes // 4, device=dev)
    G, S = torch.empty(C, C, device=dev), torch.empty(C, device=dev)
    fn = lambda: L.call("pcs_gram", L.ptr(Y), L.ptr(s), L.ptr(t), B, N, C, L.BF16, sps.value,  # noqa: E731
                        L.ptr(ws), L.ptr(G), L.ptr(S), L.stream_ptr())
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"gram 128 (sps {sps.value}): {ms:7.3f} ms  {B * N * C * 2 / 1e9 / ms:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()

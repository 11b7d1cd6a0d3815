"""Micro-benchmark of the streaming forward kernel (csrc/fwd_stream.hip) at cfg2 (4 x 128^3 rows):
seg_conv1 (64 -> 512, scene bias), seg_conv2 (512 -> 256, dropout), seg_conv3 (256 -> 128,
dropout), conv5 (128 -> 1024, BN5 + ReLU, column sums).  Alternate builds: PCS_LIB=path.
    python tools/bench_fwd.py [reps]"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402


def run(B, N, K, C, kind, reps):
    dev = torch.device("cuda")
    M = B * N
    yp = (torch.randn(M, K, device=dev) + 0.2).to(torch.bfloat16)
    W = (torch.randn(C, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    c8 = kind == "bnrelu8"   # conv5 with the fp8 e4m3 a5 store (cfg5)
    out = torch.empty(M, C, device=dev, dtype=torch.uint8 if c8 else torch.bfloat16)
    v = lambda n: torch.rand(n, device=dev) + 0.5   # noqa: E731
    keep = [v(K), v(K) - 1.0, v(C), v(C) - 1.0, torch.randn(B, C, device=dev)]
    epi = L.EPI_BNRELU if kind in ("bnrelu", "bnrelu8") else L.EPI_FWD
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=C, dtype=L.BF16, prologue=L.PRO_BNRELU, epilogue=epi,
                   chunks_per_scene=0, A=yp.data_ptr(), W=W.data_ptr(), C=out.data_ptr(),
                   a_keep_scale=1.0 / 0.7 if kind == "mask" else 1.0, c_keep_scale=1.0,
                   flags=L.FLAG_C_FP8 if c8 else 0)
    a.pa, a.pb = keep[0].data_ptr(), keep[1].data_ptr()
    if kind in ("bnrelu", "bnrelu8"):
        a.es, a.et = keep[2].data_ptr(), keep[3].data_ptr()
    if kind == "bias":
        a.bias = keep[2].data_ptr()
    if kind == "scene":
        a.scene_bias = keep[4].data_ptr()
    bits = torch.randint(0, 256, (M, K // 8), device=dev, dtype=torch.uint8)
    if kind == "mask":
        a.a_mask = bits.data_ptr()
    L.load().pcs_gemm_geometry(ct.byref(a))
    st = torch.empty(B * a.chunks_per_scene, C, 2, device=dev)
    a.stats = st.data_ptr()
    fn = lambda: L.call("pcs_gemm", ct.byref(a), L.stream_ptr())   # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gb = M * (K * 2 + C * (1 if c8 else 2)) / 1e9 + (M * K / 8 / 1e9 if kind == "mask" else 0)
    print(f"{kind:7s} {K:4d}->{C:4d}: {ms:7.3f} ms  {gb / ms:6.2f} TB/s", flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B, N = 4, 128 ** 3
    shapes = [(64, 512, "scene"), (512, 256, "mask"), (256, 128, "mask"), (128, 1024, "bnrelu")]
    if os.environ.get("FS_SHAPES") == "small":   # conv4, conv2 / conv3
        shapes = [(64, 128, "bias"), (64, 64, "bias")]
    if os.environ.get("FS_SHAPES") == "all":   # the four wide shapes and conv5's fp8 store
        shapes.append((128, 1024, "bnrelu8"))
    if os.environ.get("FS_SHAPES") == "conv5":   # conv5 with the bf16 and the fp8 a5 store
        shapes = [(128, 1024, "bnrelu"), (128, 1024, "bnrelu8")]
    for K, C, kind in shapes:
        run(B, N, K, C, kind, reps)


if __name__ == "__main__":
    main()

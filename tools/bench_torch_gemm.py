"""What the vendor library reaches on global_feat's GEMM shapes (M = 4 x 128^3 rows, 1024 x 1024
weight), as a yardstick for the hand-written LDS-DMA kernel (no epilogue work here):

* bf16 a5 W^T (forward / dgrad shape) through torch.mm (hipBLASLt);
* fp8 e4m3 with per-tensor scales through torch._scaled_mm, when this build supports it.

    python tools/bench_torch_gemm.py
"""
import torch


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
    M, K, Nc = 4 * 128 ** 3, 1024, 1024
    dev = torch.device("cuda")
    flop = 2.0 * M * K * Nc
    A = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(Nc, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
    ms = timeit(lambda: torch.mm(A, W.t(), out=out))
    print(f"bf16 torch.mm  M={M} K={K} N={Nc}: {ms:7.3f} ms  {flop / ms / 1e9:7.1f} TF/s", flush=True)
    Wt = W.t().contiguous().t()
    ms = timeit(lambda: torch.mm(A, Wt, out=out))
    print(f"bf16 torch.mm (W col-major): {ms:7.3f} ms  {flop / ms / 1e9:7.1f} TF/s", flush=True)
    try:
        A8 = A.to(torch.float8_e4m3fn)
        W8 = W.to(torch.float8_e4m3fn)
        one = torch.ones((), device=dev)
        ms = timeit(lambda: torch._scaled_mm(A8, W8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
        print(f"fp8 torch._scaled_mm: {ms:7.3f} ms  {flop / ms / 1e9:7.1f} TF/s", flush=True)
    except Exception as e:  # noqa: BLE001 -- report what this build lacks
        print(f"fp8 torch._scaled_mm unavailable: {type(e).__name__}: {e}", flush=True)


if __name__ == "__main__":
    main()

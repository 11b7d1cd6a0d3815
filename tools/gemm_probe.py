"""Library ceiling for the wide layer's GEMM shapes: torch.matmul (hipBLASLt) on the global_feat
forward / dgrad shape, M = 4 x 128^3 rows, 1024 x 1024 bf16, no epilogue.  The hand-written
kernels are compared against this number.
    python tools/gemm_probe.py [reps]"""
import sys

import torch


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda")
    for M in (4 * 128 ** 3, 1 << 20):
        a = torch.randn(M, 1024, device=dev, dtype=torch.bfloat16)
        w = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
        for name, fn in [("a @ w^T", lambda: a @ w.t()), ("a @ w", lambda: a @ w)]:
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / reps
            tf = 2.0 * M * 1024 * 1024 / ms / 1e9
            print(f"M={M:9d} {name}: {ms:7.3f} ms  {tf:7.1f} TF/s  ({tf / 2516.6:.3f} of bf16 dense peak)", flush=True)
        del a, w
    # Gram a^T a (the Gram-form weight gradient's shape)
    a = torch.randn(4 * 128 ** 3, 1024, device=dev, dtype=torch.bfloat16)
    fn = lambda: a.t() @ a   # noqa: E731
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    tf = 2.0 * a.shape[0] * 1024 * 1024 / ms / 1e9
    print(f"Gram a^T a M={a.shape[0]}: {ms:7.3f} ms  {tf:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()

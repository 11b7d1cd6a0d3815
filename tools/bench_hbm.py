"""HBM stream rates on this box, as the yardstick for the write-heavy layer kernels (conv5's
BN+ReLU pass writes 17 GB of a5 and reads 2 GB): write-only (fill), read-only (sum), and copy
at 4 / 8 / 17 GB, through torch's own kernels (bandwidth = bytes moved / time).

    python tools/bench_hbm.py
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
    dev = torch.device("cuda")
    for gb in (4, 8, 17):
        n = gb * 2 ** 30 // 2
        x = torch.empty(n, dtype=torch.bfloat16, device=dev)
        ms = timeit(lambda: x.fill_(1.0))
        print(f"write-only {gb:3d} GiB: {ms:7.3f} ms  {x.numel() * 2 / ms / 1e9:6.2f} TB/s", flush=True)
        ms = timeit(lambda: x.sum(dtype=torch.float32))
        print(f"read-only  {gb:3d} GiB: {ms:7.3f} ms  {x.numel() * 2 / ms / 1e9:6.2f} TB/s", flush=True)
        if gb <= 8:
            y = torch.empty_like(x)
            ms = timeit(lambda: y.copy_(x))
            print(f"copy       {gb:3d} GiB: {ms:7.3f} ms  {2 * x.numel() * 2 / ms / 1e9:6.2f} TB/s (read + write)",
                  flush=True)
            del y
        del x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

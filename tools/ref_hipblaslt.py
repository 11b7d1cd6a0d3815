import torch, time
M, K, N = 4 * 128**3, 1024, 1024
A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
W = torch.randn(N, K, device="cuda").to(torch.bfloat16)
for name, fn in [("A @ W^T (NT, like our fwd)", lambda: A @ W.t()), ("A^T @ A (Gram-like, TN)", lambda: A.t() @ A[:, :K])]:
    fn(); torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(5): fn()
    en.record(); torch.cuda.synchronize()
    ms = st.elapsed_time(en) / 5
    print(f"{name}: {ms:.3f} ms  {2*M*K*N/ms/1e9:.1f} TF/s", flush=True)

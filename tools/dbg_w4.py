"""Diagnostics for csrc/gemm_w4.hip: the input gradient with H = I and c = 0 must return the
masked operand itself; integer-coded operands show where a wrong element came from."""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcs_amd._lib as L  # noqa: E402

DEV = torch.device("cuda")


def run(B, N, K, cps, flags=0, H=None, c=None, A=None):
    lib = L.load()
    a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=K, dtype=L.BF16, prologue=L.PRO_RAW,
                   epilogue=L.EPI_DGRAD, chunks_per_scene=cps, flags=flags)
    lib.pcs_gemm_geometry(ct.byref(a))
    out = torch.full((B * N, K), -7.0, dtype=torch.bfloat16, device=DEV)
    a.A, a.W, a.C, a.Yp, a.bias = A.data_ptr(), H.data_ptr(), out.data_ptr(), A.data_ptr(), c.data_ptr()
    print("selected w4:", lib.pcs_gemm_w4_selected(ct.byref(a)), "cps", a.chunks_per_scene)
    L.call("pcs_gemm", ct.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    return out


def main():
    B, N, K, cps = [int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (1, 512, 512, 1))]
    M = B * N
    r = torch.arange(M)[:, None]
    k = torch.arange(K)[None, :]
    A = (((r % 16) * 16 + (k % 16)) + 1).float().to(torch.bfloat16).to(DEV)
    H = torch.eye(K, dtype=torch.bfloat16, device=DEV)
    c = torch.zeros(K, device=DEV)
    out = run(B, N, K, cps, 0, H, c, A)
    bad = (out != A)
    nb = int(bad.sum())
    print(f"identity case: {nb} of {M * K} wrong")
    if nb:
        idx = bad.nonzero()[:12].tolist()
        for rr, cc in idx:
            v = float(out[rr, cc])
            dec = (int(v) - 1) if v >= 1 else -1
            print(f"  row {rr} col {cc}: got {v} (r%16={dec // 16}, k%16={dec % 16}) want {float(A[rr, cc])}")
        br = bad.view(M // 32 if M % 32 == 0 else 1, -1).any(1) if M % 32 == 0 else None
        rows_bad = bad.any(1).nonzero().flatten()
        cols_bad = bad.any(0).nonzero().flatten()
        print("  bad rows:", rows_bad.numel(), rows_bad[:20].tolist())
        print("  bad cols:", cols_bad.numel(), cols_bad[:40].tolist())
        print("  by col%32:", bad.sum(0).view(-1, 32).sum(0).tolist())
        print("  by row%32:", bad.sum(1)[: (M // 32) * 32].view(-1, 32).sum(0).tolist())
        print("  by col-block 32:", bad.sum(0).view(-1, 32).sum(1).tolist())
        print("  by row tile 256:", bad.sum(1)[: (M // 256) * 256].view(-1, 256).sum(1).tolist())
    # mask: H a permutation (column c takes k = c ^ 1), operand with zeros, -0 and exact codes
    P = torch.zeros(K, K, dtype=torch.bfloat16, device=DEV)
    P[torch.arange(K), torch.arange(K) ^ 1] = 1.0
    Am = A.clone()
    zr = ((r * 7 + k * 3) % 5 == 0).to(DEV)
    Am[zr] = 0.0
    Am[(((r * 5 + k) % 11) == 0).to(DEV)] = -0.0
    outm = run(B, N, K, cps, 0, P, c, Am)
    wantm = torch.where(Am > 0, Am[:, torch.arange(K, device=DEV) ^ 1], torch.zeros_like(Am))
    badm = outm != wantm
    print(f"mask case: {int(badm.sum())} wrong")
    if int(badm.sum()):
        for rr, cc in badm.nonzero()[:10].tolist():
            print(f"  row {rr} col {cc}: got {float(outm[rr, cc])} want {float(wantm[rr, cc])} a={float(Am[rr, cc])}")
        print("  by col%32:", badm.sum(0).view(-1, 32).sum(0).tolist())
        print("  by col-block 32:", badm.sum(0).view(-1, 32).sum(1).tolist())
        print("  by row%32:", badm.sum(1)[: (M // 32) * 32].view(-1, 32).sum(0).tolist())
        print("  by row tile 256:", badm.sum(1)[: (M // 256) * 256].view(-1, 256).sum(1).tolist())
    # bias only
    Hz = torch.zeros_like(H)
    cb = (torch.arange(K, device=DEV) % 13 + 1).float()
    Ap = torch.ones_like(A)
    out2 = run(B, N, K, cps, 0, Hz, cb, Ap)
    want = cb.to(torch.bfloat16)[None, :].expand(M, K)
    bad2 = out2 != want
    print(f"bias case: {int(bad2.sum())} wrong")
    if int(bad2.sum()):
        idx = bad2.nonzero()[:8].tolist()
        for rr, cc in idx:
            print(f"  row {rr} col {cc}: got {float(out2[rr, cc])} want {float(want[rr, cc])}")
        print("  by col%32:", bad2.sum(0).view(-1, 32).sum(0).tolist())


if __name__ == "__main__":
    main()

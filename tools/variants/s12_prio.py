# fwd_s12: the wave in the interleaved stage-2 / stage-1 MFMA section at raised issue priority
# (s_setprio 1), back to 0 for the transform, the epilogue and the DMA issue
NAME = "s12_prio"
SRC = "fwd_s12"
EDITS = [
    ("""      uint32_t pa[2][2], pb[2][2];
      stage2(xr, 0, 3, acc2);""",
     """      uint32_t pa[2][2], pb[2][2];
      __builtin_amdgcn_s_setprio(1);
      stage2(xr, 0, 3, acc2);"""),
    ("""      store1(pa, pb, 1, out1);
      __builtin_amdgcn_sched_barrier(0);
    }""",
     """      store1(pa, pb, 1, out1);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
    }"""),
]

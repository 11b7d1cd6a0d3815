# fwd_s12: interleave each loop part's VALU (epilogue 1) with its 16 MFMAs by sched_group_barrier
NAME = "s12_sgb"
SRC = "fwd_s12"
_P = """
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      }
      __builtin_amdgcn_sched_barrier(0);"""
EDITS = [
    ("""      epi1(st1, xw, 0, acc1, pa);
      stage1(st1, 1, acc1);
      __builtin_amdgcn_sched_barrier(0);""",
     """      epi1(st1, xw, 0, acc1, pa);
      stage1(st1, 1, acc1);""" + _P),
    ("""      store1(pa, pb, 0, out1);
      stage1(st1, 2, acc1);
      __builtin_amdgcn_sched_barrier(0);""",
     """      store1(pa, pb, 0, out1);
      stage1(st1, 2, acc1);""" + _P),
    ("""      epi1(st1, xw, 2, acc1, pa);
      stage1(st1, 3, acc1);
      __builtin_amdgcn_sched_barrier(0);""",
     """      epi1(st1, xw, 2, acc1, pa);
      stage1(st1, 3, acc1);""" + _P),
    ("""      store1(pa, pb, 1, out1);
      __builtin_amdgcn_sched_barrier(0);
    }""",
     """      store1(pa, pb, 1, out1);""" + _P + """
    }"""),
]

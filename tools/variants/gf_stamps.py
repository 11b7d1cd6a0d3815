# Diagnostic build (never shipped, never timed as a result): s_memtime stamps in gemm_glds's
# K-tile loop, summed per wave into a device buffer that tools/stamps_gf.py reads back through
# pcs_debug_stamps.  Segments (cycles, per wave, summed over the launch):
#   0 prep   : each phase's part before its first barrier (fragment reads, mask, DMA issue, waits)
#   1 open   : waiting at the phases' first barriers
#   2 mfma   : the MFMA sections
#   3 close  : waiting at the phases' second barriers
#   4 ealign : waiting at the epilogue's aligning barrier
#   5 ebody  : the epilogue up to its stores (mask / pool / statistics arithmetic)
#   6 estore : the DGRAD stores and S1 (FWD: 0)
#   7 erest  : the stagger-restoring barrier and the accumulator reset
# Read SHARES (the stamps' own lgkmcnt(0) waits and ~40 cycles each distort lengths).
NAME = "gf_stamps"
SRC = "gemm_glds"
STAMP = '''__builtin_amdgcn_sched_barrier(0); asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(STV) :: "memory"); __builtin_amdgcn_sched_barrier(0);'''


def st(seg):
    """close the running segment into sum[seg] and start the next one"""
    return ("{ unsigned long long STV; " + STAMP + " ssum[" + str(seg) + "] += STV - tlast; tlast = STV; }")


EDITS = [
    ("""constexpr int LDS_BYTES = OFF_UNI + 2 * 256 * 8 * 4;""",
     """constexpr int LDS_BYTES = OFF_UNI + 2 * 256 * 8 * 4;
__device__ unsigned long long g_stamps[4096 * 8][16];"""),
    ("""  for (int qs = 0; qs < total; ++qs, kt = ka, tcur = ta, pcur = pa) {""",
     """  unsigned long long ssum[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tlast;
  { unsigned long long STV; """ + STAMP + """ tlast = STV; }
  for (int qs = 0; qs < total; ++qs, kt = ka, tcur = ta, pcur = pa) {"""),
]
# per phase: prep | open barrier | mfma | close barrier
for ph, quad in enumerate(("mfma_quad(0, 0);", "mfma_quad(0, 2);", "mfma_quad(4, 0);", "mfma_quad(4, 2);")):
    EDITS.append(("""    barrier_raw();
    """ + quad + """
    barrier_raw();""", "    " + st(ph) + """
    barrier_raw();
    """ + st(4 + ph) + """
    """ + quad + """
    """ + st(8) + """
    barrier_raw();
    """ + st(9)))
EDITS += [
    ("""    u32x4 mv0, mv1;
    read_a(buf, 0);
    read_b(buf, 2, 0);""", """    u32x4 mv0, mv1;
    """ + st(14) + """
    read_a(buf, 0);
    """ + st(15) + """
    read_b(buf, 2, 0);"""),
    ("""    if (xmask) {
      mask_load(buf, 0, mv0, mv1);
      mask_bits(0, kt - kq0, tcur & 1, mv0, mv1);
    }
    issue(qs + 1, pa, ka, 1);""", """    if (xmask) {
      mask_load(buf, 0, mv0, mv1);
      mask_bits(0, kt - kq0, tcur & 1, mv0, mv1);
    }
    """ + st(11) + """
    issue(qs + 1, pa, ka, 1);
    """ + st(12)),
    ("""    if (qs + 1 < total) wait_vm<10>(); else wait_vm<2>();
    wait_lgkm0();""", """    if (qs + 1 < total) wait_vm<10>(); else wait_vm<2>();
    """ + st(13) + """
    wait_lgkm0();"""),
    ("""    bias_init(acc);
    if (wm == 1) barrier_raw();   // the stagger again (see the epilogue's first barrier)
  }""", """    bias_init(acc);
    if (wm == 1) barrier_raw();   // the stagger again (see the epilogue's first barrier)
    """ + st(10) + """
  }
  if (lane == 0) {
    const int gw = blockIdx.x * 8 + wid;
    if (gw < 4096 * 8)
      for (int s = 0; s < 16; ++s) g_stamps[gw][s] = ssum[s];
  }"""),
    ("""extern "C" int pcs_pool_rows_add(""", """extern "C" int pcs_debug_stamps(void *host, int64_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes < (int64_t)sizeof(g_stamps) ? bytes : sizeof(g_stamps)) == hipSuccess ? 0 : -1;
}

extern "C" int pcs_pool_rows_add("""),
]

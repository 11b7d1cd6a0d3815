// Fused input + weight gradient of seg_conv2 (512 -> 256) and seg_conv3 (256 -> 128)
// (autograd of P:125-127 at P:254), on an LDS-DMA stream:
//
//   dy   = alpha * dZ + beta + gamma * Y                 ([M, COUT], bn_seg{2,3} backward)
//   g    = dy . W                                        ([M, CIN])
//   dz'  = (es * Yp + et > 0) * keep * ks * g             (stored; S1 = sum dz', S2 = sum dz' Yp)
//   dW  += dy^T . x,   x = relu(es * Yp + et) * keep * ks ([COUT, CIN])
//
// Separately (pcs_gemm DGRAD + pcs_wgrad) the pair reads dZ, Y and Yp twice and measured
// 10.4 ms (seg_conv2) / 4.6 ms (seg_conv3) at cfg2, 4.1-4.3 TB/s each.  Here one pass moves
// dZ, Y, Yp and the dropout bits in and dz' out.
//
// * A workgroup (8 waves) owns a CB = 128 column block of CIN for a scene-aligned row slice:
//   the CIN / CB workgroups of a slice are consecutive, so they run on one XCD and the dZ / Y
//   rows they all stream come from that XCD's L2 after the first read.
// * Rows stream in MS = 32-row steps through an NST-stage LDS ring filled by LDS-DMA
//   (global_load_lds): dZ and Y (COUT wide), the block's Yp (128 wide) and its dropout bits.
//   Every wave issues the same number of pieces per step (5 or 3 of 1 KB, plus one 256-B
//   piece of the bits), always -- past the slice end the rows are clamped and the data never
//   read -- so one compile-time vmcnt count serves every wave and every step.  The 16-B slots
//   of an LDS row hold the source chunks XOR-permuted by (row & 15) (the permutation is put on
//   the DMA source address, since the DMA writes LDS linearly): the fragment reads and the
//   transposed reads below are then bank-conflict free.
// * Per step: the transform of step t+1 (dy, in place over its dZ slab; x into a double
//   buffer) by all 512 threads, each element once; the input gradient of step t from the
//   registers' W^T block (loaded once) and dy fragments; the weight gradient of step t from
//   transposed reads (ds_read_b64_tr_b16) of dy and x; then the epilogue in registers (mask,
//   S1 / S2, 16-B stores widened with v_permlane16_swap).  One barrier per step: the wait for
//   step t+1 and the barrier at the top of step t, the DMA after it (a two-barrier form, with
//   the wait between the phases, measured 0.05-0.1 ms slower and was removed).
// * dW partial per workgroup (fp32, the slice's slab) and per-slice S1 / S2, reduced by the
//   caller's pcs_reduce_partials as pcs_dgrad_wgrad_bn's other shapes.
#include "common.h"


namespace {

constexpr int THREADS = 512;
constexpr int CB = 128;   // CIN columns per workgroup
constexpr int MS = 32;    // rows per step

template <int COUT> struct SegCfg {
  static constexpr int NST = COUT == 256 ? 3 : 4;          // ring stages
  static constexpr int DZB = MS * COUT * 2;                 // dZ (-> dy in place) / Y slab bytes
  static constexpr int YPB = MS * CB * 2;                   // Yp slab
  static constexpr int MKB = MS * CB / 8;                   // dropout bits (512 B)
  static constexpr int STAGE = 2 * DZB + YPB + MKB;
  static constexpr int XR = CB * 2 + 32;                    // x row stride (32-B pad, prow rows)
  static constexpr int XB = MS * XR;                        // one x buffer
  static constexpr int OFF_X = NST * STAGE;                 // x [2][MS][XR]
  static constexpr int OFF_CF = OFF_X + 2 * XB;             // alpha | beta | gamma [COUT], es | et [CB]
  static constexpr int OFF_LUT = OFF_CF + (3 * COUT + 2 * CB) * 4;   // dropout-bit masks, [256][4] u32
  static constexpr int BYTES = OFF_LUT + 256 * 16;
  static_assert(BYTES <= 160 * 1024, "LDS budget");
  static constexpr int KS = COUT / 32;                      // dgrad k-steps (32 deep)
  static constexpr int OBW = COUT / 128;                    // wgrad 16-row output tiles per wave
  static constexpr int SPR = COUT / 8;                      // 16-B slots per dZ row
  static constexpr int DZP = DZB / 1024;                    // 1-KB pieces per dZ slab
  static constexpr int YPP = YPB / 1024;                    // 1-KB pieces per Yp slab (8)
  static constexpr int NPW = (2 * DZP + YPP) / 8;           // 1-KB pieces per wave per step
  static_assert((2 * DZP + YPP) % 8 == 0, "uniform pieces per wave");
  static constexpr int VM_STEP = NPW + 1;                   // vector-memory loads per wave per step
  static constexpr int DY_RPT = MS * SPR / THREADS;         // dy slots per thread per step
  static_assert(DY_RPT == 1 || DY_RPT == 2, "transform passes");
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// LDS-DMA: 64 lanes x 16 B (or x 4 B) from sbase + voff (per lane) to the LDS address in M0
// (+ lane * size).  Inline asm so that the compiler's own wait insertion neither drains these
// loads before unrelated LDS reads nor spills their addresses: the kernel counts them itself.
// M0 is set from a per-step SGPR base plus an immediate (one SALU per piece); the caller
// saves M0 before a group of pieces and restores it after (m0_save / m0_restore).
template <int OFF> PCS_DEV void glds16o(const char *sbase, uint32_t voff, uint32_t m0base) {
  asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0base), "n"(OFF) : "memory", "scc");
}
template <int OFF> PCS_DEV void glds4o(const char *sbase, uint32_t voff, uint32_t m0base) {
  asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0base), "n"(OFF) : "memory", "scc");
}
PCS_DEV uint32_t m0_save() {
  uint32_t k;
  asm volatile("s_mov_b32 %0, m0" : "=s"(k));
  return k;
}
PCS_DEV void m0_restore(uint32_t k) { asm volatile("s_mov_b32 m0, %0" ::"s"(k)); }
template <int N> PCS_DEV void wait_vm() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
PCS_DEV void barrier_lds() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS layouts.  The ring stages are written by LDS-DMA (linear per 1-KB piece), so the slot
// permutations go on the DMA source addresses:
// * dZ / Y rows (unpadded): 16-B chunk c of row r at chunk c ^ ftr(r), ftr an even value
//   distinct over each row set a fragment read or a transposed read touches -- the dgrad's
//   ds_read_b128 (16 rows, one chunk) and the wgrad's ds_read_b64_tr_b16 (rows {0-3, 8-11} or
//   {4-7, 12-15}, two chunks) are both bank-conflict free (checked with the guide's bank model).
//   The transform reads dZ and Y lane-linearly and writes dy back in place, so dy keeps it.
// * Yp: chunk c of row r at c ^ (r & 15): the epilogue's 8-B reads of 16 rows at one column
//   hit 16 distinct chunks.
// * x (written by the transform): rows padded by 32 B and permuted (row bits 2 <-> 3), the
//   layout of fused_bwd.hip, conflict free for the transposed reads.
PCS_DEV int ftr(int row) { return ((row & 3) << 1) | (row & 8); }
PCS_DEV int prow(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }
PCS_DEV int fyp(int row) { return row & 15; }

PCS_DEV bf16x8 tr_frag2(const char *p0, const char *p1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)p0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)p1);
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// 8 coefficients of one 16-B data slot from the split LDS layout: elements 0-3 of every slot
// first, then elements 4-7 (lanes reading consecutive slots then read consecutive 16 B: no bank
// conflicts; the interleaved [slot][8] layout would put two lanes on every bank)
PCS_DEV void lds_vec8(const char *p, int half_bytes, float (&v)[8]) {
  const u32x4 x = *reinterpret_cast<const u32x4 *>(p);
  const u32x4 y = *reinterpret_cast<const u32x4 *>(p + half_bytes);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = __uint_as_float(x[e]);
    v[4 + e] = __uint_as_float(y[e]);
  }
}
PCS_DEV int split_idx(int i, int n) { return ((i & 7) >> 2) * (n / 2) + (i >> 3) * 4 + (i & 3); }
PCS_DEV float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
PCS_DEV float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

template <int COUT, int CIN, bool MASK>
__global__ __launch_bounds__(THREADS) void seg_bwd_kernel(pcs_gemm_args a, float *__restrict__ wpart,
                                                          int64_t rows_per_split) {
  typedef SegCfg<COUT> F;
  constexpr int NBLK = CIN / CB;
  constexpr int ROWB = COUT * 2;   // dZ / Y / dy row bytes
  __shared__ __attribute__((aligned(16))) char lds[F::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (divisions by runtime values run on the VALU: the results are made provably uniform, so
  // the DMA bases below stay in SGPRs instead of waterfall loops around every piece)
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = __builtin_amdgcn_readfirstlane(L / NBLK), n0 = __builtin_amdgcn_readfirstlane((L % NBLK) * CB);
  const int sps = a.chunks_per_scene;
  const int scene = __builtin_amdgcn_readfirstlane(chunk / sps), sis = __builtin_amdgcn_readfirstlane(chunk % sps);
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int64_t sbase = (int64_t)scene * N;
  const int nsteps = (int)((hi - lo + MS - 1) / MS);   // >= 1 (no empty slices)
  const char *dZg = reinterpret_cast<const char *>(a.A);
  const char *Yg = reinterpret_cast<const char *>(a.A2);
  const char *Ypg = reinterpret_cast<const char *>(a.Yp) + n0 * 2;
  const char *Mkg = MASK ? reinterpret_cast<const char *>(a.c_mask) + n0 / 8 : nullptr;
  const bf16_t *Wt = reinterpret_cast<const bf16_t *>(a.W);   // W^T [CIN][COUT]
  bf16_t *Cg = reinterpret_cast<bf16_t *>(a.C);
  const float ks = MASK ? a.c_keep_scale : 1.f;

  // ---- DMA of step s into ring stage sidx.  Piece j = wid + 8 i of the step, 1 KB each, laid
  // out contiguously in the stage: dZ [0, DZP), Y [DZP, 2 DZP), Yp [2 DZP, 2 DZP + YPP) (a
  // round i has one kind for every wave: DZP is a multiple of 8), then one dword piece of the
  // dropout bits (waves 0 / 1 take its two halves; the others repeat them, writing the same
  // bytes, so that every wave issues the same count; without bits they read Yp's rows, never
  // used).  Per-lane source offsets relative to the step's first row, carrying the slot
  // swizzles; rows past the slice clamp to its last row (their LDS rows are never used).
  static_assert(F::DZP % 8 == 0, "piece rounds of one kind");
  auto piece_off = [&](int i, int lastr) -> uint32_t {
    if (8 * i < 2 * F::DZP) {
      const int pj = (8 * i < F::DZP ? 8 * i : 8 * i - F::DZP) + wid;
      const int r = pj * (1024 / ROWB) + lane / F::SPR;
      return (uint32_t)(min(r, lastr) * ROWB + (((lane % F::SPR) ^ ftr(r)) << 4));
    }
    const int r = (8 * i - 2 * F::DZP + wid) * 4 + (lane >> 4);
    return (uint32_t)(min(r, lastr) * CIN * 2 + (((lane & 15) ^ fyp(r)) << 4));
  };
  auto mask_off = [&](int lastr) -> uint32_t {
    const int r = 16 * (wid & 1) + (lane >> 2);
    return (uint32_t)(min(r, lastr) * (MASK ? CIN / 8 : CIN * 2) + (lane & 3) * 4);
  };
  uint32_t voff[F::NPW + 1];
#pragma unroll
  for (int i = 0; i < F::NPW; ++i) voff[i] = piece_off(i, MS - 1);
  voff[F::NPW] = mask_off(MS - 1);
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  auto dma_issue = [&](int sidx, int64_t m0, const uint32_t (&vo)[F::NPW + 1]) {
    const uint32_t mb = lds_m0 + sidx * F::STAGE + wid * 1024;
    const char *bdz = dZg + (sbase + m0) * ROWB;
    const char *by = Yg + (sbase + m0) * ROWB;
    const char *byp = Ypg + (sbase + m0) * (CIN * 2);
    const char *bmk = MASK ? Mkg + (sbase + m0) * (CIN / 8) : byp;
    const uint32_t keep = m0_save();
    glds16o<0>(bdz, vo[0], mb);
    if constexpr (F::NPW == 5) {   // COUT 256: dZ dZ Y Y Yp
      glds16o<8192>(bdz, vo[1], mb);
      glds16o<16384>(by, vo[2], mb);
      glds16o<24576>(by, vo[3], mb);
      glds16o<32768>(byp, vo[4], mb);
    } else {                       // COUT 128: dZ Y Yp
      static_assert(F::NPW == 3, "piece rounds");
      glds16o<8192>(by, vo[1], mb);
      glds16o<16384>(byp, vo[2], mb);
    }
    glds4o<2 * F::DZB + F::YPB>(bmk, vo[F::NPW], lds_m0 + sidx * F::STAGE + (wid & 1) * 256);
    m0_restore(keep);
  };
  auto dma_step = [&](int s, int sidx) {
    const int64_t m0 = pcs_min64(lo + (int64_t)s * MS, hi - 1);
    const int lastr = (int)pcs_min64(hi - 1 - m0, MS - 1);
    if (lastr == MS - 1) {   // uniform: a full step
      dma_issue(sidx, m0, voff);
    } else {
      uint32_t vt[F::NPW + 1];
#pragma unroll
      for (int i = 0; i < F::NPW; ++i) vt[i] = piece_off(i, lastr);
      vt[F::NPW] = mask_off(lastr);
      dma_issue(sidx, m0, vt);
    }
  };

  // ---- transform coefficients in LDS (split layout), W^T fragments of this wave's dgrad
  // column tile (ct = wave) in registers, epilogue coefficients of this lane's 4 columns
  {
    float *cf = reinterpret_cast<float *>(lds + F::OFF_CF);
    for (int i = tid; i < COUT; i += THREADS) {
      const int j = split_idx(i, COUT);
      cf[j] = a.pa[i];
      cf[COUT + j] = a.pb[i];
      cf[2 * COUT + j] = a.pc[i];
    }
    if (tid < CB) {   // x = relu(es y + et) ks = relu((es ks) y + et ks): the keep scale folded in (ks > 0)
      const int j = split_idx(tid, CB);
      cf[3 * COUT + j] = a.es[n0 + tid] * ks;
      cf[3 * COUT + CB + j] = a.et[n0 + tid] * ks;
    }
    // dropout byte -> the AND masks of 8 packed bf16 values (dword d: bits 2d, 2d+1 as halves)
    if (tid < 256) {
      uint32_t *lut = reinterpret_cast<uint32_t *>(lds + F::OFF_LUT) + tid * 4;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        lut[d] = (((tid >> (2 * d)) & 1) ? 0x0000FFFFu : 0u) | (((tid >> (2 * d + 1)) & 1) ? 0xFFFF0000u : 0u);
    }
  }
  const int dlc = tid % F::SPR, drr = tid / F::SPR;   // dy: physical slot, first row
  const int xlc = tid & 15, xrr = tid >> 4;             // x: chunk, row
  // the dy slot's logical chunk is the same for all its rows (they differ by 16 rows: ftr is
  // periodic in 16), so one set of coefficients serves every pass
  const char *cfd = lds + F::OFF_CF + (dlc ^ ftr(drr)) * 16;
#ifndef SEG_CREG
#define SEG_CREG 1
#endif
  // SEG_CREG: the thread's 24 dy-transform coefficients held in registers (read from LDS once,
  // after the barrier below) instead of 6 ds_read_b128 per transform pass
  float rca[8], rcb[8], rcg[8];
  const char *cfx = lds + F::OFF_CF + 3 * COUT * 4 + xlc * 16;
  const int l16 = lane & 15, g = lane >> 4;
  const int ct = wid;
  const int cc = 16 * ct + 4 * g;   // block-local column of this lane's 4 (epilogue)
  float es4[4], et4[4];
  load_vec<4>(a.es, n0 + cc, es4);
  load_vec<4>(a.et, n0 + cc, et4);
  u32x4 wfr[F::KS];
#pragma unroll
  for (int kk = 0; kk < F::KS; ++kk)
    wfr[kk] = *reinterpret_cast<const u32x4 *>(Wt + (int64_t)(n0 + ct * 16 + l16) * COUT + (4 * kk + g) * 8);

  // loop-invariant LDS offsets, relative to a stage (or an x buffer); the k-steps / tiles /
  // passes then differ by immediates
  const int o_tr = tid * 16;                        // dZ / Y / dy of the transform, pass i: + i 8 KB
  const int o_ypx = 2 * F::DZB + xrr * (CB * 2) + ((xlc ^ fyp(xrr)) << 4);
  const int o_mkx = 2 * F::DZB + F::YPB + xrr * 16 + xlc;
  const int o_xw = prow(xrr) * F::XR + xlc * 16;
  const int o_ype = 2 * F::DZB + l16 * (CB * 2) + ((((cc >> 3) ^ l16) << 4) | ((cc & 7) << 1));   // + u 4 KB
  const int o_mke = 2 * F::DZB + F::YPB + l16 * 16 + (cc >> 3);                                     // + u 256
  // dgrad fragment of k-step kk: logical chunk 4 kk + g of row 16 u + l16 sits at chunk
  // (4 kk + g) ^ ftr(l16) = 16 (kk >> 2) + ((4 (kk & 3) + g) ^ ftr(l16))
  int o_dg[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) o_dg[b] = l16 * ROWB + (((4 * b + g) ^ ftr(l16)) << 4);
  const int q = (lane >> 2) & 3, p = lane & 3;      // transposed-read lane roles
  const int tr0 = 8 * g + q, tr1 = 8 * g + 4 + q;   // dy rows (k) of the two 4-row halves
  int o_ty[F::OBW][2];
#pragma unroll
  for (int ob = 0; ob < F::OBW; ++ob) {
    const int s = 2 * (F::OBW * wid + ob) + (p >> 1);   // logical chunk of columns 16 (..) + 4 p
    o_ty[ob][0] = tr0 * ROWB + ((s ^ ftr(tr0)) << 4) + 8 * (p & 1);
    o_ty[ob][1] = tr1 * ROWB + ((s ^ ftr(tr1)) << 4) + 8 * (p & 1);
  }
  const int o_tx0 = prow(tr0) * F::XR + 8 * p;   // + u 32 B
  const int o_tx1 = prow(tr1) * F::XR + 8 * p;

  f32x4 accw[F::OBW][8];
#pragma unroll
  for (int o = 0; o < F::OBW; ++o)
#pragma unroll
    for (int u = 0; u < 8; ++u) accw[o][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s1[4], s2[4];   // this lane's 4 columns, both row tiles
#pragma unroll
  for (int r = 0; r < 4; ++r) { s1[r] = 0.f; s2[r] = 0.f; }

  // ---- transform of step s (landed, barrier passed): dy in place over dZ, x into buffer s & 1;
  // zeros past the slice.  Split in pieces so phase 2 can put the weight-gradient MFMAs of the
  // previous step between them.
  auto transform_dy = [&](int s, int sidx, int i) {
    char *st = lds + sidx * F::STAGE;
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)s * MS), MS);   // rows of the step
    float ca[8], cb[8], cg[8], v[8], y[8];
    const u32x4 dz = *reinterpret_cast<const u32x4 *>(st + o_tr + i * THREADS * 16);
    const u32x4 yy = *reinterpret_cast<const u32x4 *>(st + F::DZB + o_tr + i * THREADS * 16);
    if constexpr (SEG_CREG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { ca[e] = rca[e]; cb[e] = rcb[e]; cg[e] = rcg[e]; }
    } else {
      lds_vec8(cfd, COUT * 2, ca);
      lds_vec8(cfd + COUT * 4, COUT * 2, cb);
      lds_vec8(cfd + 2 * COUT * 4, COUT * 2, cg);
    }
    unpack_chunk(dz, v);
    unpack_chunk(yy, y);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaf(ca[e], v[e], fmaf(cg[e], y[e], cb[e]));
    u32x4 out = pack_chunk(v);
    if (rem < MS && drr + i * (THREADS / F::SPR) >= rem) out = mk_u32x4(0, 0, 0, 0);   // (uniform test first)
    *reinterpret_cast<u32x4 *>(st + o_tr + i * THREADS * 16) = out;
  };
  auto transform_x = [&](int s, int sidx) {
    const char *st = lds + sidx * F::STAGE;
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)s * MS), MS);
    float v[8], xs[8], xt[8];
    lds_vec8(cfx, CB * 2, xs);
    lds_vec8(cfx + CB * 4, CB * 2, xt);
    unpack_chunk(*reinterpret_cast<const u32x4 *>(st + o_ypx), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = relu(fmaf(v[e], xs[e], xt[e]));
    u32x4 out = pack_chunk(v);
    if constexpr (MASK) {   // dropout: AND with the byte's masks (one LDS read for 8 values)
      const u32x4 m = *reinterpret_cast<const u32x4 *>(lds + F::OFF_LUT + (uint32_t)(uint8_t)st[o_mkx] * 16);
      out = mk_u32x4(out[0] & m[0], out[1] & m[1], out[2] & m[2], out[3] & m[3]);
    }
    if (rem < MS && xrr >= rem) out = mk_u32x4(0, 0, 0, 0);
    *reinterpret_cast<u32x4 *>(lds + F::OFF_X + (s & 1) * F::XB + o_xw) = out;
  };

  // ---- output rows through one buffer descriptor for the slice (range: its rows): a store's
  // rows past the slice are dropped by the hardware, so every wave issues exactly one store per
  // step (the counted waits); the prologue's placeholder stores lie wholly out of range
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char *>(Cg + (sbase + lo) * CIN + n0), 0,
      (int)(uint32_t)((hi - lo - 1) * CIN * 2 + CB * 2), 0x00020000);
  const uint32_t o_st = (uint32_t)((16 * (g & 1) + l16) * (CIN * 2) + (16 * ct + 8 * (g >> 1)) * 2);
  auto store_rows = [&](uint32_t vo, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, rs_out, (int)vo, 0, 0); };

  // ---- prologue: steps 0 .. NST-2 in flight (each followed by a store the range check drops,
  // as every loop step's DMA is followed by its epilogue store), step 0 landed and transformed
#pragma unroll
  for (int s = 0; s < F::NST - 1; ++s) {
    dma_step(s, s);
    store_rows(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
  }
  wait_vm<1 + (F::NST - 2) * (F::VM_STEP + 1)>();
  barrier_lds();
  if constexpr (SEG_CREG) {   // (the coefficients were written to LDS before this barrier)
    lds_vec8(cfd, COUT * 2, rca);
    lds_vec8(cfd + COUT * 4, COUT * 2, rcb);
    lds_vec8(cfd + 2 * COUT * 4, COUT * 2, rcg);
  }
#pragma unroll
  for (int i = 0; i < F::DY_RPT; ++i) transform_dy(0, 0, i);
  transform_x(0, 0);
  barrier_lds();

  // Per step t, two phases split by barriers:
  //   phase 1: DMA of step t+NST-1; input gradient of step t (dy in stage t, W^T in registers)
  //            and its epilogue (masks, S1 / S2, store);
  //   phase 2: the weight gradient of step t (dy in stage t, x in buffer t & 1) interleaved
  //            with the transform of step t+1 (stage t+1 in place, x into buffer (t+1) & 1):
  //            MFMAs and VALU work of one wave with no dependence between them.
  int sc = 0, sn = 1, sd = F::NST - 1;   // stages of steps t, t+1 and t+NST-1 (= t-1's)
  uint32_t o_out = o_st;                 // this lane's store offset at step t
  for (int t = 0; t < nsteps; ++t) {
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)t * MS), MS);
    // one barrier per step: step t+1 landed (newer: the stores and DMAs of the NST-3 steps in
    // between, and step t-1's store), visible to every wave; every wave done with step t-1
    wait_vm<1 + (F::NST - 3) * (F::VM_STEP + 1)>();
    barrier_lds();
    dma_step(t + F::NST - 1, sd);   // into the stage step t-1 used (free since the last barrier)
    const char *st = lds + sc * F::STAGE;
    const char *xb = lds + F::OFF_X + (t & 1) * F::XB;
    // (the epilogue's Yp values and dropout bits, read up front)
    uint2 ype[2];
    uint32_t kbe[2] = {0xFu, 0xFu};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      ype[u] = *reinterpret_cast<const uint2 *>(st + o_ype + u * 16 * (CB * 2));
      if constexpr (MASK) kbe[u] = (uint32_t)(uint8_t)st[o_mke + u * 256];
    }
    // input gradient out[m = 16 u + l16][c = 16 ct + 4 g + r] (both row tiles u); the LDS
    // operand reads run PD k-steps ahead of the MFMAs
    f32x4 accd[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    {
#ifndef SEG_PD
#define SEG_PD 3
#endif
      constexpr int PD = SEG_PD;
      bf16x8 yf[PD + 1][2];
      auto rd_dg = [&](int kk, bf16x8 (&d)[2]) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
          d[u] = *reinterpret_cast<const bf16x8 *>(st + o_dg[kk & 3] + (kk >> 2) * 256 + u * 16 * ROWB);
      };
#pragma unroll
      for (int kk = 0; kk < PD; ++kk) rd_dg(kk, yf[kk]);
#pragma unroll
      for (int kk = 0; kk < F::KS; ++kk) {
        if (kk + PD < F::KS) rd_dg(kk + PD, yf[(kk + PD) % (PD + 1)]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2; ++u)
          accd[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wfr[kk]), yf[kk % (PD + 1)][u],
                                                           accd[u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // epilogue: previous layer's ReLU / dropout masks, S1 / S2, 16-B stores
    {
      uint32_t pk[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint2 yp = ype[u];
        const float y[4] = {bf_lo(yp.x), bf_hi(yp.x), bf_lo(yp.y), bf_hi(yp.y)};
        // dropout bits of the lane's 4 columns, cleared for rows past the slice
        const int kb = (int)((16 * u + l16 < rem ? 0xFu : 0u) & (MASK ? (kbe[u] >> (cc & 7)) : 0xFu));
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // keep <=> bit set and z > 0: all-ones masks from the bit (sign-extended) and from the
          // comparison, applied to the bits of the scaled gradient (VALU only, no SGPR masks)
          const float z = fmaf(y[r], es4[r], et4[r]);
          const int m = __builtin_amdgcn_sbfe(kb, r, 1) & (z > 0.f ? -1 : 0);
          v[r] = __int_as_float(__float_as_int(accd[u][r] * ks) & m);
          s1[r] += v[r];
          s2[r] = fmaf(v[r], y[r], s2[r]);
        }
        pk[u][0] = pack2bf(v[0], v[1]);
        pk[u][1] = pack2bf(v[2], v[3]);
      }
      // lane groups 2h / 2h+1 trade row tiles: each lane then holds 8 consecutive columns
      // (8 (g >> 1) ..) of row 16 (g & 1) + l16
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][h], pk[1][h], false, false);
        pk[0][h] = sw[0];
        pk[1][h] = sw[1];
      }
      // a buffer store whose range ends at the slice's last row: rows past it are dropped by
      // the hardware, so every wave issues exactly one store per step (the counted waits)
      store_rows(o_out, mk_u32x4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]));
      o_out += MS * CIN * 2;
    }
    // phase 2: weight gradient dW[o = 16 (OBW wid + ob) + l16][c = 16 u + 4 g + r] over the 32
    // rows of step t, with the transform of step t+1 between its MFMA groups
    {
      const bool more = t + 1 < nsteps;
      bf16x8 yt[F::OBW], xf[2];
#pragma unroll
      for (int ob = 0; ob < F::OBW; ++ob) yt[ob] = tr_frag2(st + o_ty[ob][0], st + o_ty[ob][1]);
      xf[0] = tr_frag2(xb + o_tx0, xb + o_tx1);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u + 1 < 8) xf[(u + 1) & 1] = tr_frag2(xb + o_tx0 + (u + 1) * 32, xb + o_tx1 + (u + 1) * 32);
#pragma unroll
        for (int ob = 0; ob < F::OBW; ++ob)
          accw[ob][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[u & 1], yt[ob], accw[ob][u], 0, 0, 0);
        // transform pieces after the MFMA groups 1, 3 (dy passes) and 5 (x)
        if (more) {
          if (u == 1) transform_dy(t + 1, sn, 0);
          if (F::DY_RPT > 1 && u == 3) transform_dy(t + 1, sn, F::DY_RPT - 1);
          if (u == 5) transform_x(t + 1, sn);
        }
      }
    }
    sd = sc;
    sc = sn;
    sn = sn + 1 == F::NST ? 0 : sn + 1;
  }
  wait_vm<0>();   // the clamped DMAs past the end

  // ---- dW partial (this slice's slab, columns n0 ..)
  float *out = wpart + (int64_t)chunk * COUT * CIN + n0;
#pragma unroll
  for (int ob = 0; ob < F::OBW; ++ob)
#pragma unroll
    for (int u = 0; u < 8; ++u)
      *reinterpret_cast<float4 *>(out + (int64_t)(16 * (F::OBW * wid + ob) + l16) * CIN + 16 * u + 4 * g) =
          make_float4(accw[ob][u][0], accw[ob][u][1], accw[ob][u][2], accw[ob][u][3]);

  // ---- S1 / S2: over the 16 lanes (rows) of each column; the wave owns its columns
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s1[r] += __shfl_xor(s1[r], o);
      s2[r] += __shfl_xor(s2[r], o);
    }
  if (l16 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * ct + 4 * g + r;
      *reinterpret_cast<float2 *>(a.stats + ((int64_t)chunk * CIN + n0 + c) * 2) =
          make_float2(s1[r], a.erstd[n0 + c] * (s2[r] - a.emean[n0 + c] * s1[r]));
    }
  }
}

}  // namespace

// Shapes served: (Cout, Cin) = K x Ncols in {256 x 512 (seg_conv2), 128 x 256 (seg_conv3)}, bf16,
// PRO_BWD / EPI_DGRAD with dropout bits and no addend.
int64_t pcs_seg_bwd_geometry(pcs_gemm_args *a);
bool pcs_seg_bwd_applicable(const pcs_gemm_args &a) {
  if (!(a.dtype == PCS_BF16 && !(a.flags & PCS_FLAG_GENERIC) && !a.addend &&
        ((a.K == 256 && a.Ncols == 512) || (a.K == 128 && a.Ncols == 256))))
    return false;
  // the buffer-store ranges and per-lane row offsets are 32-bit: a slice of the widest rows
  // (Ncols bf16) must stay below 2 GB, else the generic kernels run it
  pcs_gemm_args g = a;
  const int64_t rps = pcs_seg_bwd_geometry(&g);
  return rps * (int64_t)a.Ncols * 2 < ((int64_t)1 << 31);
}

int64_t pcs_seg_bwd_geometry(pcs_gemm_args *a) {
  const int nblk = a->Ncols / CB;
  int64_t sps = (256 + a->num_scenes * nblk - 1) / (a->num_scenes * nblk);   // one WG per CU
  const int64_t max_sps = (a->scene_rows + 4 * MS - 1) / (4 * MS);
  if (sps > max_sps) sps = max_sps;
  if (sps < 1) sps = 1;
  const int64_t rps = ((a->scene_rows + sps - 1) / sps + MS - 1) / MS * MS;
  a->chunks_per_scene = (int32_t)((a->scene_rows + rps - 1) / rps);   // no empty slices
  return rps;
}

int pcs_seg_bwd_launch(const pcs_gemm_args &a, float *wpart, hipStream_t s) {
  pcs_gemm_args g = a;
  const int64_t rps = pcs_seg_bwd_geometry(&g);
  if (g.chunks_per_scene != a.chunks_per_scene)
    return pcs_set_einval("pcs_dgrad_wgrad_bn", "chunks_per_scene must come from pcs_dgrad_wgrad_bn_workspace");
  const int nb = (int)(a.num_scenes * a.chunks_per_scene) * (a.Ncols / CB);
#define PCS_SEG(CO, CI, MK) \
  hipLaunchKernelGGL((seg_bwd_kernel<CO, CI, MK>), dim3(nb), dim3(THREADS), 0, s, a, wpart, rps)
  if (a.K == 256) {
    if (a.c_mask) PCS_SEG(256, 512, true); else PCS_SEG(256, 512, false);
  } else {
    if (a.c_mask) PCS_SEG(128, 256, true); else PCS_SEG(128, 256, false);
  }
#undef PCS_SEG
  PCS_CHECK_LAUNCH();
  return 0;
}

// Fused input + weight gradient of seg_conv2 (512 -> 256) and seg_conv3 (256 -> 128) at one
// wave per SIMD (autograd of P:125-127 at P:254), the same operation as the r03 8-wave kernel (fused_seg.hip, removed in r06):
//
//   dy   = alpha * dZ + beta + gamma * Y                 ([M, COUT], bn_seg{2,3} backward)
//   g    = dy . W                                        ([M, CIN])
//   dz'  = (es * Yp + et > 0) * keep * ks * g             (stored; S1 = sum dz', S2 = sum dz' Yp)
//   dW  += dy^T . x,   x = relu(es * Yp + et) * keep * ks ([COUT, CIN])
//
// that kernel's 8-wave workgroups own 128 CIN columns each, so the four (seg_conv2) or two
// (seg_conv3) workgroups of a row slice all recompute the slice's dy, and every wave reads the
// whole dy slab for its 16 dgrad columns: vector-ALU- and LDS-bound at 3.2 TB/s.  Here four
// waves (one per SIMD, 512 registers each) own 256 columns:
//
// * wave w owns CIN columns 64 w .. 64 w + 63 of the block for everything: its W^T block in
//   VGPRs (64 x COUT bf16: 128 / 64 registers), its dW block [COUT x 64] in AGPRs (256 / 128),
//   the input gradient of those columns (16x16x32, W^T as A: each lane ends with 4 consecutive
//   columns of one row), the epilogue of those columns, which also forms x, and the weight
//   gradient from x (the wave's own LDS tile: no barrier between them) and dy (32x32x16);
// * rows stream in MS = 16-row steps through an NST-stage LDS ring filled by LDS-DMA: dZ and Y
//   (COUT wide), the block's Yp (256 wide) and its dropout bits.  Every wave issues the same
//   pieces every step (rows past the slice clamp to its last row), one compile-time vmcnt
//   serves every wait, and the pieces issue between the input gradient's MFMAs;
// * the dy transform of step t+1 (all 256 threads, each element once per workgroup) runs
//   between the weight gradient MFMAs of step t; one barrier per step.
//
// LDS images (the DMA writes linearly, so each permutation goes on its source address):
// * dZ / Y / dy rows: 16-B chunk c of row r at slot c ^ fdz(r), fdz(r) = 4 (r & 3) + tau(r >> 2 & 3),
//   tau = (0, 2, 3, 1): the transposed reads (4 aligned rows x 4 chunks per 32-lane half) and the
//   input gradient's ds_read_b128 (16 rows, chunks c0 / c0 + 1 across its lane groups) are both
//   conflict-free by the bank rule of MI355X_MICROARCH.md section LDS;
// * Yp rows: chunk c at c ^ (r & 15) (16 rows at one column: 16 distinct slots);
// * x tile of a wave: [16 rows][64 columns], 128-B rows, chunk c at c ^ (4 ((r >> 1) & 1)).
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int CB = 256;   // CIN columns per workgroup
constexpr int MS = 16;    // rows per step

template <int COUT> struct S4 {
  static constexpr int NST = COUT == 256 ? 3 : 4;    // ring stages (NST - 1 steps in flight)
  static constexpr int WLK = COUT == 256 ? 4 : 0;    // input-gradient k-steps whose W^T is staged in LDS
  static constexpr int ROWB = COUT * 2;
  static constexpr int DZB = MS * ROWB;              // dZ (-> dy in place) / Y slab
  static constexpr int YPB = MS * CB * 2;            // Yp slab (8 KB)
  static constexpr int MKB = MS * CB / 8;            // dropout bits (512 B)
  static constexpr int STAGE = 2 * DZB + YPB + MKB;
  static constexpr int TILE = 64 * 32;               // a wave's x^T or v^T tile: [64 columns][16 rows] bf16
  static constexpr int XWB = 2 * TILE;
  static constexpr int WROWB = WLK * 64;             // staged W^T row: WLK k-steps of 32 bf16
  static constexpr int OFF_X = NST * STAGE;
  static constexpr int OFF_W = OFF_X + 4 * XWB;
  static constexpr int OFF_CF = OFF_W + CB * WROWB;  // alpha | beta | gamma [COUT] (split)
  static constexpr int BYTES = OFF_CF + 3 * COUT * 4;
  static_assert(BYTES <= 160 * 1024, "LDS budget");
  static constexpr int KSD = COUT / 32;              // input-gradient k-steps
  static constexpr int NO = COUT / 32;               // weight-gradient 32-row (COUT) blocks
  static constexpr int CPR = COUT / 8;               // 16-B chunks per dZ row
  static constexpr int NPD = DZB / 1024;             // 1-KB pieces per dZ slab
  static constexpr int NPW = (2 * NPD + YPB / 1024) / 4;   // 1-KB pieces per wave per step
  static_assert(NPD % 4 == 0, "piece rounds of one kind");
  static constexpr int VM_STEP = NPW + 1;            // + the dropout-bit piece
  static constexpr int TPASS = MS * CPR / THREADS;   // transform chunks per thread
  static_assert(TPASS == 1 || TPASS == 2, "transform passes");
  static constexpr bool DACC_V = true;   // input gradient D in VGPRs (see the k-step loop)
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
// LDS-DMA through a buffer descriptor (su32x4 in SGPRs): rows past the descriptor's range
// read as zeros (and are never used), so no row clamping and no per-step branches.  M0 is
// set per piece and not restored: hipcc never reads M0 in this file's kernels
// (tests/test_asm_audit.py checks the compiled code)
typedef unsigned int su32x4 __attribute__((ext_vector_type(4)));
template <int OFF> PCS_DEV void blds16o(const su32x4 &rs, uint32_t voff, uint32_t soff, uint32_t m0base) {
  asm volatile("s_add_u32 m0, %3, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               :: "v"(voff), "s"(rs), "s"(soff), "s"(m0base), "n"(OFF) : "memory", "scc");
}
// the same loads with M0 already set (by set_m0, at least one instruction earlier)
template <int OFF> PCS_DEV void set_m0(uint32_t base) { asm volatile("s_add_u32 m0, %0, %1" ::"s"(base), "n"(OFF) : "scc"); }
PCS_DEV void blds16_m0(const su32x4 &rs, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rs), "s"(soff) : "memory");
}
PCS_DEV void blds4_m0(const su32x4 &rs, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dword %0, %1, %2 offen lds" ::"v"(voff), "s"(rs), "s"(soff) : "memory");
}
template <int OFF> PCS_DEV void blds4o(const su32x4 &rs, uint32_t voff, uint32_t soff, uint32_t m0base) {
  asm volatile("s_add_u32 m0, %3, %4\n\ts_nop 0\n\tbuffer_load_dword %0, %1, %2 offen lds"
               :: "v"(voff), "s"(rs), "s"(soff), "s"(m0base), "n"(OFF) : "memory", "scc");
}
PCS_DEV su32x4 rsrc_of(const void *base, uint32_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  su32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((uint32_t)b);
  r.y = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xffffu);
  r.z = __builtin_amdgcn_readfirstlane(bytes);
  r.w = 0x00020000u;
  return r;
}
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
PCS_DEV void wait_lgkm0() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

PCS_DEV int fdz(int r) { return ((r & 3) << 2) | ((0x1320 >> (4 * ((r >> 2) & 3))) & 3); }
PCS_DEV int fyp(int r) { return 2 * (r & 7); }
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

PCS_DEV bf16x8 tr_frag2(const char *p0, const char *p1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)p0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)p1);
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// split coefficient layout: elements 0-3 of every chunk first, then elements 4-7
PCS_DEV int split_idx(int i, int n) { return ((i & 7) >> 2) * (n / 2) + (i >> 3) * 4 + (i & 3); }
PCS_DEV float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
PCS_DEV float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// the coefficients of 8 channels as 4 packed pairs (channels 2 i, 2 i + 1)
PCS_DEV void lds_pairs8(const char *p, int half_bytes, f32x2 (&v)[4]) {
  const u32x4 x = *reinterpret_cast<const u32x4 *>(p);
  const u32x4 y = *reinterpret_cast<const u32x4 *>(p + half_bytes);
  v[0] = f32x2{__uint_as_float(x[0]), __uint_as_float(x[1])};
  v[1] = f32x2{__uint_as_float(x[2]), __uint_as_float(x[3])};
  v[2] = f32x2{__uint_as_float(y[0]), __uint_as_float(y[1])};
  v[3] = f32x2{__uint_as_float(y[2]), __uint_as_float(y[3])};
}
// the bn backward of one 16-B chunk, dy = alpha dz + (gamma y + beta), in packed fp32 pairs
// (v_pk_fma_f32: two channels per issue; the same roundings as two fmaf)
PCS_DEV u32x4 bnb_chunk(const u32x4 &dz, const u32x4 &y, const f32x2 (&ca)[4], const f32x2 (&cb)[4],
                        const f32x2 (&cg)[4]) {
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 d = {bf_lo(dz[i]), bf_hi(dz[i])}, yy = {bf_lo(y[i]), bf_hi(y[i])};
    const f32x2 r = __builtin_elementwise_fma(ca[i], d, __builtin_elementwise_fma(cg[i], yy, cb[i]));
    o[i] = pack2bf(r.x, r.y);
  }
  return mk_u32x4(o[0], o[1], o[2], o[3]);
}
template <int V> struct IC { static constexpr int value = V; };
template <int N, int I = 0, typename Fn> PCS_DEV void sfor(Fn &&fn) {
  if constexpr (I < N) {
    fn(IC<I>{});
    sfor<N, I + 1>(fn);
  }
}

template <int COUT, int CIN, bool MASK>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(1, 1)))
void seg4_kernel(pcs_gemm_args a, float *__restrict__ wpart, int64_t rows_per_split) {
  typedef S4<COUT> F;
  constexpr int NBLK = CIN / CB;
  constexpr int ROWB = F::ROWB;
  constexpr int NST = F::NST;
  __shared__ __attribute__((aligned(16))) char lds[F::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = __builtin_amdgcn_readfirstlane(L / NBLK), n0 = __builtin_amdgcn_readfirstlane((L % NBLK) * CB);
  const int sps = a.chunks_per_scene;
  const int scene = __builtin_amdgcn_readfirstlane(chunk / sps), sis = __builtin_amdgcn_readfirstlane(chunk % sps);
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int64_t sbase = (int64_t)scene * N;
  const int rows = (int)(hi - lo);                    // >= 1 (no empty slices)
  const int nsteps = (rows + MS - 1) / MS;
  const char *dZg = reinterpret_cast<const char *>(a.A) + (sbase + lo) * ROWB;
  const char *Yg = reinterpret_cast<const char *>(a.A2) + (sbase + lo) * ROWB;
  const char *Ypg = reinterpret_cast<const char *>(a.Yp) + (sbase + lo) * (CIN * 2) + n0 * 2;
  const char *Mkg = MASK ? reinterpret_cast<const char *>(a.c_mask) + (sbase + lo) * (CIN / 8) + n0 / 8 : Ypg;
  constexpr int MKROW = MASK ? CIN / 8 : CIN * 2;
  const bf16_t *Wt = reinterpret_cast<const bf16_t *>(a.W);   // W^T [CIN][COUT]
  const float ks = MASK ? a.c_keep_scale : 1.f;
  const int l16 = lane & 15, g = lane >> 4;
  const int q = (lane >> 2) & 3, p = lane & 3, G = (lane >> 4) & 1, H = lane >> 5;   // transposed reads
  const int cw = 64 * wid;   // the wave's first column in the block

  // ---- DMA of step s into stage sidx: piece j = 4 i + wid (i < NPW) of 1 KB at stage offset
  // j KB -- dZ [0, NPD), Y [NPD, 2 NPD), Yp after -- then a dword piece of the dropout bits
  // (waves 0 / 1 its two halves, waves 2 / 3 the same bytes again).  Per-lane offsets within
  // a step carry the slot permutations; the step on the scalar offset; rows past the slice
  // fall outside the buffer ranges.
  const su32x4 rs_dz = rsrc_of(dZg, (uint32_t)rows * ROWB), rs_y = rsrc_of(Yg, (uint32_t)rows * ROWB);
  const su32x4 rs_yp = rsrc_of(Ypg, (uint32_t)rows * (CIN * 2)), rs_mk = rsrc_of(Mkg, (uint32_t)rows * MKROW);
  uint32_t voff[F::VM_STEP];
#pragma unroll
  for (int i = 0; i < F::NPW; ++i) {
    const int j = 4 * i + wid;
    if (j < 2 * F::NPD) {
      const int pj = j < F::NPD ? j : j - F::NPD;
      const int r = pj * (1024 / ROWB) + lane / F::CPR, sl = lane % F::CPR;
      voff[i] = (uint32_t)(r * ROWB + ((sl ^ fdz(r)) << 4));
    } else {
      const int r = 2 * (j - 2 * F::NPD) + (lane >> 5), sl = lane & 31;
      voff[i] = (uint32_t)(r * (CIN * 2) + ((sl ^ fyp(r)) << 4));
    }
  }
  voff[F::NPW] = (uint32_t)((8 * (wid & 1) + (lane >> 3)) * MKROW + (lane & 7) * 4);
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  auto dma_piece = [&](auto Ic, int s, int sidx) __attribute__((always_inline)) {
    constexpr int i = decltype(Ic)::value;
    const uint32_t mb = lds_m0 + sidx * F::STAGE + wid * 1024;
    if constexpr (i == F::NPW)
      blds4o<2 * F::DZB + F::YPB>(rs_mk, voff[i], (uint32_t)(s * MS * MKROW), lds_m0 + sidx * F::STAGE + (wid & 1) * 256);
    else if constexpr (4 * i < F::NPD)   // (NPD % 4 == 0: a round is one kind for every wave)
      blds16o<4096 * i>(rs_dz, voff[i], (uint32_t)(s * MS * ROWB), mb);
    else if constexpr (4 * i < 2 * F::NPD)
      blds16o<4096 * i>(rs_y, voff[i], (uint32_t)(s * MS * ROWB), mb);
    else
      blds16o<4096 * i>(rs_yp, voff[i], (uint32_t)(s * MS * CIN * 2), mb);
  };
  // the same piece in two parts: M0 (ahead of an MFMA group, whose instructions are the
  // SALU M0 write -> LDS-DMA wait state) and the load (after the group)
  auto dma_m0 = [&](auto Ic, int sidx) __attribute__((always_inline)) {
    constexpr int i = decltype(Ic)::value;
    if constexpr (i == F::NPW) set_m0<2 * F::DZB + F::YPB>(lds_m0 + sidx * F::STAGE + (wid & 1) * 256);
    else set_m0<4096 * i>(lds_m0 + sidx * F::STAGE + wid * 1024);
  };
  auto dma_load = [&](auto Ic, int s) __attribute__((always_inline)) {
    constexpr int i = decltype(Ic)::value;
    if constexpr (i == F::NPW) blds4_m0(rs_mk, voff[i], (uint32_t)(s * MS * MKROW));
    else if constexpr (4 * i < F::NPD) blds16_m0(rs_dz, voff[i], (uint32_t)(s * MS * ROWB));
    else if constexpr (4 * i < 2 * F::NPD) blds16_m0(rs_y, voff[i], (uint32_t)(s * MS * ROWB));
    else blds16_m0(rs_yp, voff[i], (uint32_t)(s * MS * CIN * 2));
  };

  // ---- coefficients in LDS: dy-transform alpha / beta / gamma (split); the first WLK k-steps
  // of the block's W^T rows (fdz-permuted 16-B chunks, as the dy rows)
  {
    float *cf = reinterpret_cast<float *>(lds + F::OFF_CF);
    for (int i = tid; i < COUT; i += THREADS) {
      const int j = split_idx(i, COUT);
      cf[j] = a.pa[i];
      cf[COUT + j] = a.pb[i];
      cf[2 * COUT + j] = a.pc[i];
    }
    if constexpr (F::WLK > 0) {
      constexpr int WCH = F::WLK * 4;   // 16-B chunks per staged W^T row
      for (int i = tid; i < CB * WCH; i += THREADS) {
        const int c = i / WCH, ch = i % WCH;
        *reinterpret_cast<u32x4 *>(lds + F::OFF_W + c * F::WROWB + ((ch ^ fdz(c & 15)) << 4)) =
            *reinterpret_cast<const u32x4 *>(Wt + (int64_t)(n0 + c) * COUT + 8 * ch);
      }
    }
  }
  // x = relu(es y + et) ks = relu((es ks) y + et ks) (ks > 0): the mask is x > 0; the lane's
  // column of each 16-column tile ct
  float esk[4], etk[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    esk[ct] = a.es[n0 + cw + 16 * ct + l16] * ks;
    etk[ct] = a.et[n0 + cw + 16 * ct + l16] * ks;
  }
  // the rest of the wave's W^T block in registers: k-steps WLK.., rows cw + 16 ct + l16,
  // k = 32 kk + 8 g .. + 7 (B of 16x16x32)
  constexpr int KR = F::KSD - F::WLK;
  bf16x8 wt[4][KR];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int kk = 0; kk < KR; ++kk)
      wt[ct][kk] = *reinterpret_cast<const bf16x8 *>(Wt + (int64_t)(n0 + cw + 16 * ct + l16) * COUT +
                                                    32 * (F::WLK + kk) + 8 * g);

  // ---- output rows through one buffer descriptor for the slice: stores past its rows are
  // dropped by the hardware, so every wave issues exactly two per step (the counted waits)
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char *>(a.C) + ((sbase + lo) * CIN + n0) * 2, 0,
      (int)(uint32_t)((uint32_t)(rows - 1) * (uint32_t)(CIN * 2) + CB * 2), 0x00020000);
  // store lanes: row l16, columns cw + 16 (g & 1) + 8 (g >> 1) + 32 h .. + 7 (h = 0, 1)
  const uint32_t o_st = (uint32_t)(l16 * (CIN * 2) + (cw + 16 * (g & 1) + 8 * (g >> 1)) * 2);
  auto store_rows = [&](uint32_t vo, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, rs_out, (int)vo, 0, 0); };

  // ---- per-lane LDS addresses as base + (constant ^ lane term): fdz(r) = 4 (r & 3) + tau and
  // chunk (4 k + c) ^ fdz(r) = 4 (k ^ (r & 3)) + (c ^ tau) for c < 4.  The lane terms are made
  // opaque once per step (pin below), so the addresses form at their use (one v_xad each)
  // instead of being hoisted out of the loop into dozens of registers.
  const int tau_l = fdz(l16) & 3;
  const int o_dg = l16 * ROWB + 16 * (g ^ tau_l);                        // dy A rows: + ((kk << 6) ^ dgx)
  const int o_wl = F::OFF_W + (cw + l16) * F::WROWB + 16 * (g ^ tau_l);  // staged W^T: + 16 ct rows + ((kk << 6) ^ dgx)
  const int dgx0 = (l16 & 3) << 6;
  // Yp by transposed reads: block (rows 4 g .. 4 g + 3, columns cw + 16 ct + 4 p ..): lane
  // 4 q + p gives row 4 g + q; chunk (cw >> 3) + 2 ct + (p >> 1) at slot chunk ^ fyp(row)
  const int ryp = 4 * g + q;
  const int o_yp = 2 * F::DZB + ryp * (CB * 2) + 8 * (p & 1) + ((((cw >> 3) + (p >> 1)) ^ fyp(ryp)) & ~6) * 16;
  const int ypx0 = ((((cw >> 3) + (p >> 1)) ^ fyp(ryp)) & 6) << 4;     // + ((ct << 5) ^ ypx)
  const int o_mk = 2 * F::DZB + F::YPB + 4 * g * (CB / 8) + cw / 8;      // bits of rows 4 g .. + 3
  char *xw = lds + F::OFF_X + wid * F::XWB;                             // x^T tile, v^T at + TILE
  // x^T / v^T tiles: element (c, row) at 32 c + 8 ((row >> 2) ^ tk(c)) + 2 (row & 3),
  // tk(c) = ((c >> 2) ^ (c >> 4)) & 3: the epilogue's 8-B writes (16 columns, one row quad per
  // lane group), the weight gradient's 8-B reads (32 columns x 2 row quads per half) and the
  // stores' transposed reads (8 columns x 4 row quads per half) are all conflict-free.
  // The lane's column 16 ct + l16, rows 4 g .. 4 g + 3: + ((520 ct) ^ twx)
  const int o_tw = l16 * 32;
  const int twx0 = 8 * ((g ^ (l16 >> 2)) & 3);
  // weight-gradient A (dy^T, transposed reads): rows r0 = 8 H + q, r1 = r0 + 4
  const int r0 = 8 * H + q, r1 = r0 + 4;
  const int cq = 2 * G + (p >> 1);
  const int o_t0 = r0 * ROWB + 16 * (cq ^ (fdz(r0) & 3)) + 8 * (p & 1);   // + ((o << 6) ^ trx)
  const int o_t1 = r1 * ROWB + 16 * (cq ^ (fdz(r1) & 3)) + 8 * (p & 1);
  const int trx0 = q << 6;
  // weight-gradient B (x^T rows c = 32 nb + (lane & 31), rows 8 H .. + 7: one ds_read_b128)
  const int cx = lane & 31;
  int o_xb[2][2];   // [nb][row quad 2 H + j]
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = 32 * nb + cx;
      o_xb[nb][j] = c * 32 + 8 * ((2 * H + j) ^ (((c >> 2) ^ (c >> 4)) & 3));
    }
  // the dz' stores: v^T rows c = 16 g + 4 s + q (s = 0..3), v rows 4 p ..: transposed reads
  // read s: rows c = 16 s + 4 g + q of v^T, v rows 4 p ..: + ((520 s) ^ vrx)
  const int o_vr = 128 * g + 32 * q;
  const int vrx0 = 8 * (p ^ g);
  // transform: logical chunk lc of rows trow + pass * (THREADS / CPR)
  const int lc = tid % F::CPR, trow = tid / F::CPR;
  int o_tr[F::TPASS];
#pragma unroll
  for (int ps = 0; ps < F::TPASS; ++ps) {
    const int r = trow + ps * (THREADS / F::CPR);
    o_tr[ps] = r * ROWB + ((lc ^ fdz(r)) << 4);
  }
  const char *cft = lds + F::OFF_CF + (lc * 16);   // split layout: elements 0-3 at + 16 lc, 4-7 at + COUT * 2 + 16 lc

  f32x16 acc[F::NO][2];
#pragma unroll
  for (int o = 0; o < F::NO; ++o)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc[o][nb] = f32x16{};
  // the lane's column of tile ct: S1 / S2 as packed pairs (rows 4 g + 2 j, 4 g + 2 j + 1), summed at the end
  f32x2 s1p[4] = {}, s2p[4] = {};

  // dy of step s (landed, barrier passed) in place over its dZ slab; rows past the slice -> 0
  f32x2 ca[4], cb[4], cg[4];   // the thread's transform coefficients (loop-invariant), read once below
  auto transform = [&](int s, int sidx) __attribute__((always_inline)) {
    char *st = lds + sidx * F::STAGE;
    const int rem = min(rows - s * MS, MS);
#pragma unroll
    for (int ps = 0; ps < F::TPASS; ++ps) {
      const int r = trow + ps * (THREADS / F::CPR);
      const int o = o_tr[ps];
      const u32x4 out = bnb_chunk(*reinterpret_cast<const u32x4 *>(st + o),
                                  *reinterpret_cast<const u32x4 *>(st + F::DZB + o), ca, cb, cg);
      // (MASK: rows past the slice need no zeroing -- their keep bits read as 0 from the range-
      // checked DMA, so their x, v and dW terms are 0 whatever dy holds)
      const bool in = MASK || r < rem;
      *reinterpret_cast<u32x4 *>(st + o) = mk_u32x4(in ? out.x : 0u, in ? out.y : 0u, in ? out.z : 0u, in ? out.w : 0u);
    }
  };

  // ---- prologue: steps 0 .. NST-2 in flight (each followed by two stores the range check
  // drops, as every loop step's DMA is followed by its two epilogue stores), step 0 landed
  // and transformed
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { dma_piece(Ic, s, s); });
    store_rows(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
    store_rows(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
  }
  wait_vm<2 + (NST - 2) * (F::VM_STEP + 2)>();
  barrier_lds();
  lds_pairs8(cft, COUT * 2, ca);
  lds_pairs8(cft + COUT * 4, COUT * 2, cb);
  lds_pairs8(cft + 2 * COUT * 4, COUT * 2, cg);
  transform(0, 0);

  int sc = 0, sn = 1, sd = NST - 1;   // stages of steps t, t+1 and t+NST-1 (= t-1's)
  uint32_t o_out = o_st;
  for (int t = 0; t < nsteps; ++t) {
    const int rem = min(rows - t * MS, MS);
    // one barrier per step: step t+1 landed (newer: the two stores of step t-NST+2 and the
    // DMA + stores of the NST-3 steps after it), dy of step t complete, every wave done with
    // step t-1's stage
    wait_vm<2 + (NST - 3) * (F::VM_STEP + 2)>();
    barrier_lds();
    const char *st = lds + sc * F::STAGE;
    int dgx = dgx0, ypx = ypx0, trx = trx0, twx = twx0, vrx = vrx0;
    asm volatile("" : "+v"(dgx), "+v"(ypx), "+v"(trx), "+v"(twx), "+v"(vrx));   // (pin: see above)
    const int sdma = t + NST - 1;

    // the epilogue's operands, read ahead of the input gradient: dropout bits of rows 4 g + r
    // (columns cw .. cw + 63), Yp[rows 4 g .. + 3][column cw + 16 ct + l16] (transposed reads:
    // element r = row 4 g + r)
    uint2 bb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bb[r] = MASK ? *reinterpret_cast<const uint2 *>(st + o_mk + r * (CB / 8)) : make_uint2(~0u, ~0u);
    u32x2 yv[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
      yv[ct] = __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(st + o_yp + ((ct << 5) ^ ypx))));

    // ---- input gradient of step t: dacc[ct] = D[row 4 g + r][column cw + 16 ct + l16]
    // (A = dy rows, B = W^T rows), operands read one k-step ahead, the DMA of step t+NST-1
    // between the MFMA groups
    f32x4 dacc[4] = {f32x4{}, f32x4{}, f32x4{}, f32x4{}};
    bf16x8 bq[2], wl[2][4];
    auto rd_k = [&](auto Kc) __attribute__((always_inline)) {
      constexpr int kk = decltype(Kc)::value;
      // ((kk << 6) ^ dgx) with dgx in bits 6-7: k-steps kk and kk + 4 differ by 256 B (an immediate)
      bq[kk & 1] = *reinterpret_cast<const bf16x8 *>(st + o_dg + (((kk & 3) << 6) ^ dgx) + 256 * (kk >> 2));
      if constexpr (kk < F::WLK) {
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
          wl[kk & 1][ct] = *reinterpret_cast<const bf16x8 *>(lds + o_wl + ct * 16 * F::WROWB + ((kk << 6) ^ dgx));
      }
    };
    rd_k(IC<0>{});
    sfor<F::KSD>([&](auto Kc) __attribute__((always_inline)) {
      constexpr int kk = decltype(Kc)::value;
      if constexpr (kk + 1 < F::KSD) rd_k(IC<kk + 1>{});
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (kk <= F::NPW) dma_m0(IC<kk>{}, sd);
      bf16x8 w[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if constexpr (kk < F::WLK) w[ct] = wl[kk & 1][ct];
        else w[ct] = wt[ct][kk - F::WLK];
      }
      if constexpr (F::DACC_V) {
        // (seg_conv2: dW's accumulators fill all 256 AGPRs; the builtin's AGPR-form D made hipcc
        // park 16 of them in VGPRs around every step -- 32 moves.  Here D is in VGPRs; the last
        // group's D gets 12 wait states before the epilogue reads it, an accumulate chain needs
        // none, and the A / B operands come from ds_reads (hipcc's s_waitcnt), never from a VALU
        // write in the 2 instructions before -- tests/test_asm_audit.py checks the compiled code)
#define PCS_MF(d, b, c) "v_mfma_f32_16x16x32_bf16 " d ", %4, " b ", " c "\n\t"
        if constexpr (kk == 0)
          asm volatile(PCS_MF("%0", "%5", "0") PCS_MF("%1", "%6", "0") PCS_MF("%2", "%7", "0")
                           PCS_MF("%3", "%8", "0")
                       : "=&v"(dacc[0]), "=&v"(dacc[1]), "=&v"(dacc[2]), "=&v"(dacc[3])
                       : "v"(bq[kk & 1]), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
        else if constexpr (kk + 1 < F::KSD)
          asm volatile(PCS_MF("%0", "%5", "%0") PCS_MF("%1", "%6", "%1") PCS_MF("%2", "%7", "%2")
                           PCS_MF("%3", "%8", "%3")
                       : "+v"(dacc[0]), "+v"(dacc[1]), "+v"(dacc[2]), "+v"(dacc[3])
                       : "v"(bq[kk & 1]), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
        else
          asm volatile(PCS_MF("%0", "%5", "%0") PCS_MF("%1", "%6", "%1") PCS_MF("%2", "%7", "%2")
                           PCS_MF("%3", "%8", "%3") "s_nop 7\n\ts_nop 3"
                       : "+v"(dacc[0]), "+v"(dacc[1]), "+v"(dacc[2]), "+v"(dacc[3])
                       : "v"(bq[kk & 1]), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
#undef PCS_MF
      } else {
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
          dacc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[kk & 1], w[ct], dacc[ct], 0, 0, 0);
      }
      if constexpr (kk <= F::NPW) dma_load(IC<kk>{}, sdma);
      __builtin_amdgcn_sched_barrier(0);
    });
    sfor<F::VM_STEP - (F::KSD < F::VM_STEP ? F::KSD : F::VM_STEP)>([&](auto Ic) __attribute__((always_inline)) {
      dma_piece(IC<F::KSD + decltype(Ic)::value>{}, sdma, sd);   // (seg_conv3: 4 k-steps, 5 pieces)
    });

    // ---- epilogue of step t: masks, S1 / S2, x^T and v^T into the wave's tiles
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      float xv[4], v[4];
#pragma unroll
      for (int j = 0; j < 2; ++j) {   // rows 2 j, 2 j + 1 in packed fp32 (v_pk_fma / mul / add)
        const f32x2 y2 = {bf_lo(yv[ct][j]), bf_hi(yv[ct][j])};
        const f32x2 z2 = __builtin_elementwise_fma(y2, f32x2{esk[ct], esk[ct]}, f32x2{etk[ct], etk[ct]});
        const f32x2 d2 = f32x2{dacc[ct][2 * j], dacc[ct][2 * j + 1]} * ks;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 2 * j + h;
          const uint32_t wb = ct < 2 ? bb[r].x : bb[r].y;
          // MASK: the keep bits of rows past the slice are 0 (range-checked DMA), no row test
          const int kb = __builtin_amdgcn_sbfe((int)wb, 16 * (ct & 1) + l16, 1);
          const int keep = (MASK || 4 * g + r < rem) ? kb : 0;
          xv[r] = __int_as_float(__float_as_int(relu(z2[h])) & keep);
          v[r] = xv[r] > 0.f ? d2[h] : 0.f;
        }
        const f32x2 v2 = {v[2 * j], v[2 * j + 1]};
        s1p[ct] += v2;
        s2p[ct] = __builtin_elementwise_fma(v2, y2, s2p[ct]);
      }
      *reinterpret_cast<uint2 *>(xw + o_tw + ((520 * ct) ^ twx)) = make_uint2(pack2bf(xv[0], xv[1]), pack2bf(xv[2], xv[3]));
      *reinterpret_cast<uint2 *>(xw + F::TILE + o_tw + ((520 * ct) ^ twx)) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- reads for the rest of the step, issued together (a wave's LDS operations complete
    // in order, so the tile reads see the writes above): the dz' rows from v^T, the weight
    // gradient's x^T operands and first three dy^T operands, and the transform's inputs of
    // step t+1
    u32x2 rd[4];
#pragma unroll
    for (int sq = 0; sq < 4; ++sq)
      rd[sq] = __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                              (lds_s16x4 *)(xw + F::TILE + o_vr + ((520 * sq) ^ vrx))));
    bf16x8 xf[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const uint2 lo2 = *reinterpret_cast<const uint2 *>(xw + o_xb[nb][0]);
      const uint2 hi2 = *reinterpret_cast<const uint2 *>(xw + o_xb[nb][1]);
      xf[nb] = __builtin_bit_cast(bf16x8, mk_u32x4(lo2.x, lo2.y, hi2.x, hi2.y));
    }
    auto rd_af = [&](int o) __attribute__((always_inline)) {   // ((o << 6) ^ trx), trx in bits 6-7
      const int x = ((o & 3) << 6) ^ trx;
      return tr_frag2(st + o_t0 + x + 256 * (o >> 2), st + o_t1 + x + 256 * (o >> 2));
    };
    bf16x8 afq[3];
    afq[0] = rd_af(0);
    afq[1] = rd_af(1);
    afq[2] = rd_af(2);
    char *stn = lds + sn * F::STAGE;
    const int remn = min(rows - (t + 1) * MS, MS);
    u32x4 tdz[F::TPASS], tyy[F::TPASS];
#pragma unroll
    for (int ps = 0; ps < F::TPASS; ++ps) {
      const int o = o_tr[ps];
      tdz[ps] = *reinterpret_cast<const u32x4 *>(stn + o);
      tyy[ps] = *reinterpret_cast<const u32x4 *>(stn + F::DZB + o);
    }
    __builtin_amdgcn_sched_barrier(0);

    // dz' stores: read s of v^T rows 16 s + 4 g + 0..3 (transposed: lane l16 gets row l16,
    // columns 16 s + 4 g ..); lane groups 2h / 2h+1 then trade reads (s, s + 1): each lane
    // holds 8 consecutive columns 16 (s + (g & 1)) + 8 (g >> 1) .. of row l16 -- two 16-B stores
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t w[4];
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto sw = __builtin_amdgcn_permlane16_swap(rd[2 * h][d], rd[2 * h + 1][d], false, false);
        w[d] = sw[0];
        w[2 + d] = sw[1];
      }
      store_rows(o_out + 64 * h, mk_u32x4(w[0], w[1], w[2], w[3]));
    }
    o_out += MS * CIN * 2;

    // ---- weight gradient of step t: acc[o][nb] = D[cout 32 o + m][cin cw + 32 nb + n] over
    // the 16 rows, dy^T operands three groups ahead; the transform of step t+1 (dy in place
    // over its dZ slab, zero past the slice) in the MFMA groups 1 and 2
    sfor<F::NO>([&](auto Oc) __attribute__((always_inline)) {
      constexpr int o = decltype(Oc)::value;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        acc[o][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afq[o % 3], xf[nb], acc[o][nb], 0, 0, 0);
      if constexpr (o + 3 < F::NO) afq[o % 3] = rd_af(o + 3);
      if constexpr (o >= 1 && o - 1 < F::TPASS) {
        constexpr int ps = o - 1;
        const int r = trow + ps * (THREADS / F::CPR);
        const u32x4 out = bnb_chunk(tdz[ps], tyy[ps], ca, cb, cg);
        // (past the last step: a stage nobody reads; MASK: rows past the slice need no zeroing,
        // as in transform() -- their keep bits are 0, so their x, v and dW terms are 0)
        const bool in = MASK || r < remn;
        *reinterpret_cast<u32x4 *>(stn + o_tr[ps]) =
            mk_u32x4(in ? out.x : 0u, in ? out.y : 0u, in ? out.z : 0u, in ? out.w : 0u);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    sd = sc;
    sc = sn;
    sn = sn + 1 == NST ? 0 : sn + 1;
  }
  wait_vm<0>();   // the clamped DMAs past the end

  // ---- dW partial (this slice's slab, columns n0 + cw ..): acc[o][nb] register e holds
  // row 32 o + (e & 3) + 8 (e >> 2) + 4 H, column cw + 32 nb + (lane & 31)
  float *out = wpart + (int64_t)chunk * COUT * CIN + n0 + cw + (lane & 31);
#pragma unroll
  for (int o = 0; o < F::NO; ++o)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        out[(int64_t)(32 * o + (e & 3) + 8 * (e >> 2) + 4 * H) * CIN + 32 * nb] = acc[o][nb][e];

  // ---- S1 / S2 over the four row groups g (lanes l16, l16 + 16, + 32, + 48)
  float s1[4], s2[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    s1[ct] = s1p[ct].x + s1p[ct].y;
    s2[ct] = s2p[ct].x + s2p[ct].y;
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int m = 16; m < 64; m <<= 1) {
      s1[ct] += __shfl_xor(s1[ct], m);
      s2[ct] += __shfl_xor(s2[ct], m);
    }
  if (g == 0) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int c = n0 + cw + 16 * ct + l16;
      *reinterpret_cast<float2 *>(a.stats + ((int64_t)chunk * CIN + c) * 2) =
          make_float2(s1[ct], a.erstd[c] * (s2[ct] - a.emean[c] * s1[ct]));
    }
  }
}

}  // namespace

// Shapes served: (Cout, Cin) = K x Ncols in {256 x 512 (seg_conv2), 128 x 256 (seg_conv3)}, bf16,
// PRO_BWD / EPI_DGRAD, no addend.
int64_t pcs_seg4_geometry(pcs_gemm_args *a);
bool pcs_seg4_applicable(const pcs_gemm_args &a) {
  if (!(a.dtype == PCS_BF16 && !(a.flags & PCS_FLAG_GENERIC) && !a.addend &&
        ((a.K == 256 && a.Ncols == 512) || (a.K == 128 && a.Ncols == 256))))
    return false;
  // the buffer-store range and the per-lane row offsets are 32-bit: a slice's rows (Ncols
  // bf16) below 2 GB
  pcs_gemm_args g = a;
  const int64_t rps = pcs_seg4_geometry(&g);
  return rps * (int64_t)a.Ncols * 2 < ((int64_t)1 << 31);
}

int64_t pcs_seg4_geometry(pcs_gemm_args *a) {
  const int nblk = a->Ncols / CB;
  int64_t sps = (256 + a->num_scenes * nblk - 1) / (a->num_scenes * nblk);   // one WG per CU
  const int64_t max_sps = (a->scene_rows + 8 * MS - 1) / (8 * MS);
  if (sps > max_sps) sps = max_sps;
  if (sps < 1) sps = 1;
  const int64_t rps = ((a->scene_rows + sps - 1) / sps + MS - 1) / MS * MS;
  a->chunks_per_scene = (int32_t)((a->scene_rows + rps - 1) / rps);   // no empty slices
  return rps;
}

int pcs_seg4_launch(const pcs_gemm_args &a, float *wpart, hipStream_t s) {
  pcs_gemm_args g = a;
  const int64_t rps = pcs_seg4_geometry(&g);
  if (g.chunks_per_scene != a.chunks_per_scene)
    return pcs_set_einval("pcs_dgrad_wgrad_bn", "chunks_per_scene must come from pcs_dgrad_wgrad_bn_workspace");
  const int nb = (int)(a.num_scenes * a.chunks_per_scene) * (a.Ncols / CB);
#define PCS_SEG4(CO, CI, MK) \
  hipLaunchKernelGGL((seg4_kernel<CO, CI, MK>), dim3(nb), dim3(THREADS), 0, s, a, wpart, rps)
  if (a.K == 256) {
    if (a.c_mask) PCS_SEG4(256, 512, true); else PCS_SEG4(256, 512, false);
  } else {
    if (a.c_mask) PCS_SEG4(128, 256, true); else PCS_SEG4(128, 256, false);
  }
#undef PCS_SEG4
  PCS_CHECK_LAUNCH();
  return 0;
}

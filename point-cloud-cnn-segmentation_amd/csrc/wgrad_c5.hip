// conv5's R = dz5^T a4 (a4 = relu(bn4(y4))) as one LDS-DMA stream: the alpha-term of conv5's
// weight gradient and, through pcs_bn_s2_from_r, bn5's S2 (autograd of P:110 at P:254).
//
// The register-staged pcs_wgrad kernel (gemm_tn.hip, 128 x 128 tiles, 64-row steps, a barrier
// and a register round trip per step) read dz5 and y4 at 4.5-4.9 TB/s (3.95-4.26 ms at cfg2).
// Here the fused seg backward's weight-gradient half (the r03 fused_seg.hip, now in git history) without its input gradient:
// * a workgroup (8 waves) owns NB = 256 dz5 columns and all 128 a4 channels of a scene-aligned
//   row slice: the [256 x 128] fp32 partial of R stays in registers (64 per lane), the slice's
//   partial goes out once, summed over the slices by pcs_reduce_partials (fixed order);
// * 32-row steps of dz5 (16 KB) and y4 (8 KB) through a 2-stage LDS ring by LDS-DMA, counted
//   waits; relu(bn4(y4)) formed once per element into a double-buffered x tile (the 4 column
//   blocks of a slice repeat this 128-wide transform, on one XCD, through L2);
// * MFMA operands by ds_read_b64_tr_b16 of the row-major dz5 and x tiles (k = rows), the
//   layouts (slot permutations, padded x rows) of the r03 fused_seg.hip, now in git history: bank-conflict free.
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int MS = 32;           // rows per step
constexpr int NB = 256;          // dz5 columns per workgroup
constexpr int CIN = 128;         // a4 channels
// two stages (66 KB of LDS) so that two workgroups share a CU (512 in the grid): 3.85 -> 3.64 ms
// in tools/bench_wc5.py against four stages at one workgroup per CU (three: 3.85)
#ifndef WC5_NST
#define WC5_NST 2
#endif
#ifndef WC5_TARGET
#define WC5_TARGET 512
#endif
constexpr int NST = WC5_NST;     // ring stages
constexpr int ROWB = NB * 2;     // 512-B dz5 rows in LDS
constexpr int SPR = ROWB / 16;   // 32 slots
constexpr int DZB = MS * ROWB;   // 16 KB
constexpr int YROW = CIN * 2;    // 256-B y4 rows
constexpr int YB = MS * YROW;    // 8 KB
constexpr int STAGE = DZB + YB;
constexpr int XR = CIN * 2 + 32;  // x row stride (32-B pad, prow rows)
constexpr int XB = MS * XR;
constexpr int OFF_X = NST * STAGE;
constexpr int BYTES = OFF_X + 2 * XB;
static_assert(BYTES <= 160 * 1024, "LDS budget");
constexpr int DZP = DZB / 1024 / 8;   // dz5 pieces per wave per step (2)
constexpr int LPS = DZP + 1;          // + one y4 piece
constexpr int OBW = NB / 128;         // 16-column output tiles of dz5 per wave (2)

typedef __attribute__((address_space(3))) void lds_void_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
template <int OFF> PCS_DEV void glds16o(const char *sbase, uint32_t voff, uint32_t m0base) {
  asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
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
// slot permutations (the r03 fused_seg.hip, now in git history): dz5 rows chunk c at c ^ ftr(r); y4 rows at c ^ (r & 15);
// x rows permuted (bits 2 <-> 3) and padded
PCS_DEV int ftr(int row) { return ((row & 3) << 1) | (row & 8); }
PCS_DEV int prow(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }
PCS_DEV bf16x8 tr_frag2(const char *p0, const char *p1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)p0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)p1);
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// S1: also the column sums of dz5 (pcs_wgrad_args.dy_colsum; the opt-in four-wave global_feat
// kernel's bn5 S1), a separate instantiation so that the default one keeps its registers
template <bool S1>
__global__ __launch_bounds__(THREADS) void wgrad_c5_kernel(pcs_wgrad_args a, int64_t rows_per_split) {
  __shared__ __attribute__((aligned(16))) char lds[BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Cout = a.Cout, ncb = Cout / NB;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = __builtin_amdgcn_readfirstlane(L / ncb), n0 = __builtin_amdgcn_readfirstlane((L % ncb) * NB);
  const int sps = a.splits_per_scene;
  const int scene = __builtin_amdgcn_readfirstlane(split / sps), sis = __builtin_amdgcn_readfirstlane(split % sps);
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int64_t sbase = (int64_t)scene * N;
  const int nsteps = (int)((hi - lo + MS - 1) / MS);   // >= 1 (no empty slices)
  const char *Dg = reinterpret_cast<const char *>(a.dZ) + n0 * 2;   // dz5 [M][Cout], this block's columns
  const char *Yg = reinterpret_cast<const char *>(a.X);             // y4 [M][128]
  const int64_t drow = (int64_t)Cout * 2;

  // transform: thread -> y4 row tid / 16, logical 16-B chunk tid % 16 (8 channels: bn4 scale /
  // shift in registers)
  const int xlc = tid & 15, xrr = tid >> 4;
  float xs[8], xt[8];
  load_vec<8>(a.s, 8 * xlc, xs);
  load_vec<8>(a.t, 8 * xlc, xt);
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(xs[e]), "v"(xt[e]));   // retired before the DMA
  __syncthreads();

  // ---- DMA of step s into stage sidx: dz5 pieces j = wid + 8 i (2 rows of 512 B each), the y4
  // piece wid (4 rows of 256 B); rows past the slice clamp to its last row (their x rows are
  // zeroed by the transform, so they add nothing)
  auto dz_off = [&](int i, int lastr) -> uint32_t {
    const int j = wid + 8 * i;
    const int r = j * 2 + lane / SPR, ps = lane % SPR;
    return (uint32_t)((int64_t)min(r, lastr) * drow + ((ps ^ ftr(r)) << 4));
  };
  auto y_off = [&](int lastr) -> uint32_t {
    const int r = wid * 4 + (lane >> 4);
    return (uint32_t)(min(r, lastr) * YROW + (((lane & 15) ^ (r & 15)) << 4));
  };
  uint32_t voff[LPS];
#pragma unroll
  for (int i = 0; i < DZP; ++i) voff[i] = dz_off(i, MS - 1);
  voff[DZP] = y_off(MS - 1);
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  auto dma_issue = [&](int sidx, int64_t m0, const uint32_t (&vo)[LPS]) {
    const uint32_t mb = lds_m0 + sidx * STAGE + wid * 1024;
    const char *bd = Dg + (sbase + m0) * drow;
    const char *by = Yg + (sbase + m0) * YROW;
    const uint32_t keep = m0_save();
    glds16o<0>(bd, vo[0], mb);
    glds16o<8192>(bd, vo[1], mb);
    glds16o<DZB>(by, vo[2], mb);
    m0_restore(keep);
  };
  static_assert(DZP == 2, "two dz5 pieces per wave per step");
  auto dma_step = [&](int s, int sidx) {
    const int64_t m0 = pcs_min64(lo + (int64_t)s * MS, hi - 1);
    const int lastr = (int)pcs_min64(hi - 1 - m0, MS - 1);
    if (lastr == MS - 1) {   // uniform: a full step
      dma_issue(sidx, m0, voff);
    } else {
      uint32_t vt[LPS];
#pragma unroll
      for (int i = 0; i < DZP; ++i) vt[i] = dz_off(i, lastr);
      vt[DZP] = y_off(lastr);
      dma_issue(sidx, m0, vt);
    }
  };

  constexpr bool do_s1 = S1;
  // x = relu(bn4(y4)) of step s into x buffer s & 1; rows past the slice -> 0
  const int o_yx = DZB + xrr * YROW + ((xlc ^ (xrr & 15)) << 4);
  const int o_xw = prow(xrr) * XR + xlc * 16;
  auto transform = [&](int s, int sidx) {
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)s * MS), MS);
    float v[8];
    unpack_chunk(*reinterpret_cast<const u32x4 *>(lds + sidx * STAGE + o_yx), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = relu(fmaf(v[e], xs[e], xt[e]));
    u32x4 out = pack_chunk(v);
    if (xrr >= rem) out = mk_u32x4(0, 0, 0, 0);
    *reinterpret_cast<u32x4 *>(lds + OFF_X + (s & 1) * XB + o_xw) = out;
    // S1 (dy_colsum): a 17th 16-channel block of ones in the row's pad, zero past the slice,
    // so that the same transposed read gives the ones fragment with R's row (k) order
    if constexpr (do_s1) if (xlc < 2) {
      const uint32_t one = xrr < rem ? 0x3f803f80u : 0u;
      *reinterpret_cast<u32x4 *>(lds + OFF_X + (s & 1) * XB + prow(xrr) * XR + CIN * 2 + xlc * 16) =
          mk_u32x4(one, one, one, one);
    }
  };

  // transposed-read offsets (the r03 fused_seg.hip, now in git history's weight-gradient half): dz5 columns 16 (2 wid + ob) +
  // 4 p of rows 8 g + q and 8 g + 4 + q; x columns 16 u + 4 p of the same rows
  const int g = lane >> 4, l16 = lane & 15, q = (lane >> 2) & 3, p = lane & 3;
  const int tr0 = 8 * g + q, tr1 = 8 * g + 4 + q;
  int o_td[OBW][2];
#pragma unroll
  for (int ob = 0; ob < OBW; ++ob) {
    const int s = 2 * (OBW * wid + ob) + (p >> 1);   // logical chunk of columns 16 (OBW wid + ob) + 4 p
    o_td[ob][0] = tr0 * ROWB + ((s ^ ftr(tr0)) << 4) + 8 * (p & 1);
    o_td[ob][1] = tr1 * ROWB + ((s ^ ftr(tr1)) << 4) + 8 * (p & 1);
  }
  const int o_tx0 = prow(tr0) * XR + 8 * p, o_tx1 = prow(tr1) * XR + 8 * p;   // + u 32 B

  f32x4 acc[OBW][8], acc1[OBW];   // acc1: S1 (every row of the 16 x 16 block is the column sum)
#pragma unroll
  for (int ob = 0; ob < OBW; ++ob) {
    acc1[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[ob][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // ---- prologue: steps 0 .. NST-2 in flight, step 0 landed and transformed
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) dma_step(s, s);
  wait_vm<(NST - 2) * LPS>();
  barrier_lds();
  transform(0, 0);
  barrier_lds();

  int sc = 0;
  for (int t = 0; t < nsteps; ++t) {
    const int sn = sc + 1 == NST ? 0 : sc + 1;
    dma_step(t + NST - 1, sc == 0 ? NST - 1 : sc - 1);   // into the stage of step t-1
    const char *st = lds + sc * STAGE;
    const char *xb = lds + OFF_X + (t & 1) * XB;
    bf16x8 dt[OBW], xf[2];
#pragma unroll
    for (int ob = 0; ob < OBW; ++ob) dt[ob] = tr_frag2(st + o_td[ob][0], st + o_td[ob][1]);
    xf[0] = tr_frag2(xb + o_tx0, xb + o_tx1);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u + 1 < 8) xf[(u + 1) & 1] = tr_frag2(xb + o_tx0 + (u + 1) * 32, xb + o_tx1 + (u + 1) * 32);
#pragma unroll
      for (int ob = 0; ob < OBW; ++ob)
        acc[ob][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[u & 1], dt[ob], acc[ob][u], 0, 0, 0);
    }
    if constexpr (do_s1) {
      const bf16x8 of = tr_frag2(xb + o_tx0 + 8 * 32, xb + o_tx1 + 8 * 32);
#pragma unroll
      for (int ob = 0; ob < OBW; ++ob) acc1[ob] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, dt[ob], acc1[ob], 0, 0, 0);
    }
    // step t+1 landed (newer: NST-2 steps' pieces)
    wait_vm<(NST - 2) * LPS>();
    barrier_lds();
    if (t + 1 < nsteps) transform(t + 1, sn);
    barrier_lds();
    sc = sn;
  }
  wait_vm<0>();   // the clamped DMAs past the end

  // ---- this slice's S1 partial (after all slices' R partials): lanes of row group g = 0
  if (do_s1 && g == 0) {
    const int64_t nsl = (int64_t)gridDim.x / ncb;
    float *o1 = a.partial + nsl * Cout * CIN + (int64_t)split * Cout + n0;
#pragma unroll
    for (int ob = 0; ob < OBW; ++ob) o1[16 * (OBW * wid + ob) + l16] = acc1[ob][0];
  }
  // ---- this slice's partial: R[n0 + 16 (OBW wid + ob) + l16][16 u + 4 g .. + 4]
  float *out = a.partial + ((int64_t)split * Cout + n0) * CIN;
#pragma unroll
  for (int ob = 0; ob < OBW; ++ob)
#pragma unroll
    for (int u = 0; u < 8; ++u)
      *reinterpret_cast<float4 *>(out + (int64_t)(16 * (OBW * wid + ob) + l16) * CIN + 16 * u + 4 * g) =
          make_float4(acc[ob][u][0], acc[ob][u][1], acc[ob][u][2], acc[ob][u][3]);
}

// ---------------------------------------------------------------------------------------
// The Gram of a4 = relu(bn4(y4)) (pcs_gram at C = 128: bn5's statistics from G = a4^T a4 and the
// column sums of a4, fwd_stats:conv5).  The generic tiled kernel reads y4 once per 64-wide tile
// column (3.2 TB/s, 0.66 ms at cfg2); here one workgroup owns all 128 x 128 of a row slice:
// * 64-row steps of y4 (16 KB) through an NST-stage LDS ring by LDS-DMA, rows in the transposed-
//   read layout (chunk c at c ^ ftr(r)); relu(bn4(.)) applied in place, rows past the slice zeroed;
// * both MFMA operands are transposed reads of that tile: wave w accumulates G[16 w + l16][all]
//   (8 blocks, 32 fp32 per lane); the fp32 column sums ride the transform.
constexpr int G_MS = 64;                  // rows per step
#ifndef GRAM_NST
#define GRAM_NST 4
#endif
#ifndef GRAM_TARGET
#define GRAM_TARGET 512
#endif
constexpr int G_NST = GRAM_NST;
constexpr int G_YB = G_MS * YROW;         // 16 KB
constexpr int G_LPS = G_YB / 1024 / 8;    // 1-KB DMA pieces per wave per step (2)
constexpr int G_BYTES = G_NST * G_YB;
static_assert(G_BYTES + 8 * CIN * 4 <= 160 * 1024, "LDS budget");

__global__ __launch_bounds__(THREADS) void gram128_kernel(pcs_wgrad_args a, int64_t rows_per_split) {
  __shared__ __attribute__((aligned(16))) char lds[G_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int split = xcd_remap(blockIdx.x, gridDim.x);
  const int sps = a.splits_per_scene;
  const int scene = __builtin_amdgcn_readfirstlane(split / sps), sis = __builtin_amdgcn_readfirstlane(split % sps);
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int64_t sbase = (int64_t)scene * N;
  // an empty trailing slice (splits x rounded rows past the scene) runs no step and writes zeros
  const int nsteps = hi > lo ? (int)((hi - lo + G_MS - 1) / G_MS) : 0;
  const char *Yg = reinterpret_cast<const char *>(a.Y);

  // transform: thread -> rows tid / 16 and 32 + tid / 16, logical chunk tid % 16 (8 channels)
  const int xlc = tid & 15, xrr = tid >> 4;
  float xs[8], xt[8], cs[8];
  load_vec<8>(a.s, 8 * xlc, xs);
  load_vec<8>(a.t, 8 * xlc, xt);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    asm volatile("" ::"v"(xs[e]), "v"(xt[e]));   // retired before the DMA
    cs[e] = 0.f;
  }
  __syncthreads();

  // DMA pieces j = wid + 8 i: 4 rows of 256 B each; rows past the slice clamp to its last row
  auto y_off = [&](int i, int lastr) -> uint32_t {
    const int r = (wid + 8 * i) * 4 + (lane >> 4), ps = lane & 15;
    return (uint32_t)(min(r, lastr) * YROW + ((ps ^ ftr(r)) << 4));
  };
  uint32_t voff[G_LPS];
#pragma unroll
  for (int i = 0; i < G_LPS; ++i) voff[i] = y_off(i, G_MS - 1);
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  static_assert(G_LPS == 2, "two y4 pieces per wave per step");
  auto dma_issue = [&](int sidx, int64_t m0, const uint32_t (&vo)[G_LPS]) {
    const uint32_t mb = lds_m0 + sidx * G_YB + wid * 1024;
    const char *by = Yg + (sbase + m0) * YROW;
    const uint32_t keep = m0_save();
    glds16o<0>(by, vo[0], mb);
    glds16o<8192>(by, vo[1], mb);
    m0_restore(keep);
  };
  auto dma_step = [&](int s) {
    const int64_t m0 = pcs_min64(lo + (int64_t)s * G_MS, hi - 1);
    const int lastr = (int)pcs_min64(hi - 1 - m0, G_MS - 1);
    const int sidx = s % G_NST;
    if (lastr == G_MS - 1) {   // uniform: a full step
      dma_issue(sidx, m0, voff);
    } else {
      uint32_t vt[G_LPS];
#pragma unroll
      for (int i = 0; i < G_LPS; ++i) vt[i] = y_off(i, lastr);
      dma_issue(sidx, m0, vt);
    }
  };
  // in place: a4 over y4 in the stage, rows past the slice -> 0
  auto transform = [&](int s) {
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)s * G_MS), G_MS);
    char *st = lds + (s % G_NST) * G_YB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = xrr + 32 * h;
      u32x4 *pc = reinterpret_cast<u32x4 *>(st + r * YROW + ((xlc ^ ftr(r)) << 4));
      float v[8];
      unpack_chunk(*pc, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = r < rem ? relu(fmaf(v[e], xs[e], xt[e])) : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += v[e];   // column sums in fp32 (as the tiled kernel)
      *pc = pack_chunk(v);
    }
  };

  // transposed reads: columns 16 u + 4 p of rows 32 kk + 8 g + q and 32 kk + 8 g + 4 + q
  const int g = lane >> 4, l16 = lane & 15, q = (lane >> 2) & 3, p = lane & 3;
  const int tr0 = 8 * g + q, tr1 = 8 * g + 4 + q;
  auto o_frag = [&](int u, int row) { return row * YROW + (((2 * u + (p >> 1)) ^ ftr(row)) << 4) + 8 * (p & 1); };
  // symmetric: wave w forms the 16-wide blocks (w, w + d mod 8), d = 0 .. 3 (and d = 4 for w < 4):
  // the 36 blocks of one triangle; the partial gets each block and its transpose
  constexpr int NU = 5;
  const int nu = wid < 4 ? 5 : 4;
  int o_u[NU][2];
#pragma unroll
  for (int d = 0; d < NU; ++d) {
    const int u = (wid + d) & 7;
    o_u[d][0] = o_frag(u, tr0);
    o_u[d][1] = o_frag(u, tr1);
  }
  const int o_w0 = o_frag(wid, tr0), o_w1 = o_frag(wid, tr1);

  f32x4 acc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < G_NST - 1; ++s) dma_step(s);
  for (int t = 0; t < nsteps; ++t) {
    wait_vm<(G_NST - 2) * G_LPS>();   // step t landed (t+1 .. t+NST-2 in flight)
    barrier_lds();                     // ... for every wave; all done with step t-1's stage
    dma_step(t + G_NST - 1);           // into step t-1's stage
    transform(t);
    barrier_lds();
    const char *st = lds + (t % G_NST) * G_YB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kb = kk * 32 * YROW;
      const bf16x8 w = tr_frag2(st + kb + o_w0, st + kb + o_w1);
      bf16x8 xf[2];
      xf[0] = tr_frag2(st + kb + o_u[0][0], st + kb + o_u[0][1]);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (u + 1 < NU) xf[(u + 1) & 1] = tr_frag2(st + kb + o_u[u + 1][0], st + kb + o_u[u + 1][1]);
        if (u < 4 || u < nu) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[u & 1], w, acc[u], 0, 0, 0);
      }
    }
  }
  wait_vm<0>();   // the clamped DMAs past the end

  // G partial: [16 wid + l16][16 u + 4 g .. + 4]
  float *out = a.partial + (int64_t)split * CIN * CIN;
#pragma unroll
  for (int d = 0; d < NU; ++d) {
    if (d >= nu) continue;
    const int u = (wid + d) & 7;
    *reinterpret_cast<float4 *>(out + (int64_t)(16 * wid + l16) * CIN + 16 * u + 4 * g) =
        make_float4(acc[d][0], acc[d][1], acc[d][2], acc[d][3]);
    if (d > 0) {   // the transposed block
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(16 * u + 4 * g + r) * CIN + 16 * wid + l16] = acc[d][r];
    }
  }
  // column sums: lanes l, l + 16, l + 32, l + 48 of a wave, then the 8 waves through LDS
  __syncthreads();
  float *red = reinterpret_cast<float *>(lds);   // [8 waves][128]
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float v = cs[e];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    cs[e] = v;
  }
  if (lane < 16) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wid * CIN + 8 * lane + e] = cs[e];
  }
  __syncthreads();
  if (tid < CIN) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[w * CIN + tid];
    const int64_t nsplit = a.num_scenes * (int64_t)sps;
    a.partial[nsplit * CIN * CIN + (int64_t)split * CIN + tid] = v;
  }
}

}  // namespace

bool pcs_gram128_class(const pcs_wgrad_args &a) {   // shapes / modes only (the split geometry)
  return a.dtype == PCS_BF16 && !(a.flags & PCS_FLAG_GENERIC) && a.dy_mode == PCS_PRO_BNRELU &&
         a.x_mode == PCS_PRO_BNRELU && a.Cin == CIN && a.Cout == CIN &&
         a.num_scenes * a.scene_rows < ((int64_t)1 << 31);
}
bool pcs_gram128_applicable(const pcs_wgrad_args &a) {
  return pcs_gram128_class(a) && a.Y && a.Y == a.X && a.s && a.t && !a.x_mask;
}
int pcs_gram128_splits(const pcs_wgrad_args &a) {
  int64_t sps = (GRAM_TARGET + a.num_scenes - 1) / a.num_scenes;
  const int64_t max_sps = (a.scene_rows + 4 * G_MS - 1) / (4 * G_MS);   // >= 4 steps per split
  if (sps > max_sps) sps = max_sps;
  if (sps < 1) sps = 1;
  return (int)sps;
}
int pcs_gram128_launch(const pcs_wgrad_args &a, hipStream_t s) {
  int64_t rps = (a.scene_rows + a.splits_per_scene - 1) / a.splits_per_scene;
  rps = (rps + G_MS - 1) / G_MS * G_MS;
  const int nb = (int)(a.num_scenes * a.splits_per_scene);
  hipLaunchKernelGGL(gram128_kernel, dim3(nb), dim3(THREADS), 0, s, a, rps);
  PCS_CHECK_LAUNCH();
  return 0;
}

// conv5's R: bf16, dy_mode RAW (dZ = dz5), x_mode BNRELU without dropout bits, Cin 128,
// Cout a multiple of 256
bool pcs_wgrad_c5_class(const pcs_wgrad_args &a) {   // shapes / modes only (the split geometry)
  return a.dtype == PCS_BF16 && !(a.flags & PCS_FLAG_GENERIC) && a.dy_mode == PCS_PRO_RAW &&
         a.x_mode == PCS_PRO_BNRELU && a.Cin == CIN && a.Cout % NB == 0 &&
         a.num_scenes * a.scene_rows < ((int64_t)1 << 31);
}
bool pcs_wgrad_c5_applicable(const pcs_wgrad_args &a) {
  return pcs_wgrad_c5_class(a) && !a.x_mask && a.dZ && a.X && a.s && a.t;
}

// two 512-thread workgroups per CU: splits per scene so that (Cout / 256) x B x splits ~ 512
int pcs_wgrad_c5_splits(const pcs_wgrad_args &a) {
  const int64_t ncb = a.Cout / NB;
  int64_t sps = (WC5_TARGET + a.num_scenes * ncb - 1) / (a.num_scenes * ncb);
  const int64_t max_sps = (a.scene_rows + 4 * MS - 1) / (4 * MS);   // >= 4 steps per split
  if (sps > max_sps) sps = max_sps;
  if (sps < 1) sps = 1;
  return (int)sps;
}

int pcs_wgrad_c5_launch(const pcs_wgrad_args &a, int64_t rows_per_split, hipStream_t s) {
  if (rows_per_split % MS) return pcs_set_einval("pcs_wgrad", "conv5 R: rows per split must be a multiple of 32");
  const int nb = (int)(a.num_scenes * a.splits_per_scene) * (a.Cout / NB);
  if (a.dy_colsum)
    hipLaunchKernelGGL(wgrad_c5_kernel<true>, dim3(nb), dim3(THREADS), 0, s, a, rows_per_split);
  else
    hipLaunchKernelGGL(wgrad_c5_kernel<false>, dim3(nb), dim3(THREADS), 0, s, a, rows_per_split);
  PCS_CHECK_LAUNCH();
  return 0;
}

// The two 1024-deep GEMMs of global_feat (P:113-114 forward, P:254 input gradient) on a
// four-wave, one-wave-per-SIMD LDS-DMA kernel with 32x32x16 bf16 MFMAs:
//   forward   y_g = a5 Wg^T            epilogue: max-pool partials on sign-folded W rows
//                                      (PCS_FLAG_POOL_SIGNED_W; the training path)
//   backward  dA5 = a5 H + c           epilogue: bn5's ReLU mask read from the operand itself,
//                                      bf16 store of dz5 (the max-pool rows are added after the
//                                      kernel by pcs_pool_rows_add; S1 comes from the consumer)
//
// Why a second structure beside gemm_glds.hip (8 waves of 128x64, two per SIMD): there the
// accumulators and fragments fill 246-256 VGPRs, so each tile's epilogue (a 128 KB dz5 store at
// the per-CU store rate, ~15k cycles) runs with no MFMA beside it: 3.1-3.5 of 17 ms.  Here
// * 4 waves as 2 (M) x 2 (N), each owning 128 x 128 outputs = 4 x 4 accumulators of
//   v_mfma_f32_32x32x16_bf16 (256 AGPRs); one wave per SIMD leaves 256 VGPRs for the rest;
// * the input gradient's tile is read out of the accumulators once (bf16-packed into 128
//   VGPRs) at the first k-step of the next tile, whose MFMAs start from the bias vector; the
//   ReLU mask is applied and the 32 stores per wave are issued during the next tile's K-tiles
//   1..4, so they drain under its MFMAs instead of ahead of them;
// * a wave reads 32 KB of fragments per K-tile (16 KB per operand, each fragment used by four
//   MFMAs) against 64 KB per SIMD in the 8-wave kernel.
//
// Pipeline: a K-tile (64 deep) of both operands is staged HBM -> LDS by global_load_lds_dwordx4
// as four 16 KB regions (A k 0..31 | A k 32..63 | W k 0..31 | W k 32..63, 256 rows x 64 B),
// double-buffered (128 KB).  Per K-tile four k-steps of 16 MFMAs; the next k-step's fragments
// are read during the current one.  Two raw barriers per K-tile: at k-step 1 (all waves done
// with the half-0 regions, which are then restaged for K-tile q+2 during k-steps 1 and 2; the
// half-1 regions of K-tile q have landed) and at k-step 3 (half-1 regions free, restaged during
// k-step 3 and the next k-step 0; half 0 of q+1 has landed).  Waits are counted: vmcnt(16)
// (loads, stores and LDS-DMA retire in order on that counter; a store issued between makes the
// wait longer, never short).
//
// Lane maps (32x32x16: lane l, r = l & 31, h = l >> 5):
// * a5 fragment of row block i, k-step t of a half: row 32 i + r, k = 16 t + 8 h + 0..7 (the
//   natural order), so the lane holds the a5 values of columns 8 h + e and 16 + 8 h + e of the
//   half's 32 -- the same columns it accumulates (below), which is what the mask needs;
// * W fragment of column block j: the lane loads W row c(r) with
//   c(m) = 16 (m >> 4) + 8 ((m >> 2) & 1) + (m & 3) + 4 ((m >> 3) & 1), so that accumulator
//   register q of lane (h, r) is output row 32 i + r, column 16 (q >> 3) + 8 h + (q & 7): each
//   lane owns two runs of 8 consecutive columns (two 16-B stores, 32 B per row per instruction);
// * LDS rows are 64 B, 16-B slot s of row x holds the logical chunk s ^ ((x >> 2) & 3): both
//   fragment patterns and the DMA pieces (16 rows x 64 B) are bank-conflict free.
#include "common.h"

#include <utility>

namespace {

constexpr int THREADS = 256;
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int REG = 256 * 64;               // one operand, half a K-tile: 256 rows x 64 B
constexpr int KBUF = 4 * REG;               // A-h0 | A-h1 | W-h0 | W-h1
constexpr int STAGE_BYTES = 2 * KBUF;       // 128 KB
constexpr int OFF_BIAS = STAGE_BYTES;       // [257][8] bf16: this block's bias (dgrad c / signed fwd bias)
                                            // split c = hi + mid + lo into elements 0..2 of a row
                                            // (an MFMA against a ones fragment starts every
                                            // accumulator from it exactly); row 256 = zeros
constexpr int OFF_SGN = OFF_BIAS + 257 * 16 + 16;  // FWD: [256] f32 +1 / -1 (the extremum the pool keeps)
constexpr int OFF_CUR = OFF_SGN + 1024;     // FWD: [2 wm][256] f32 running max of sgn * y
constexpr int OFF_POOL = OFF_CUR + 2048;    // FWD: [2 wm][256] float4 (max, argmax, min, argmin)
constexpr int OFF_RUNN = OFF_POOL + 8192;   // (unused pad)
constexpr int LDS_BYTES = OFF_RUNN + 16;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

enum { MODE_FWD = 0, MODE_DGRAD = 1 };
// W4_ABL (timing ablations, wrong results): 1 no tile readout, 2 no mask bits, 4 no deferred
// stores, 8 no chunk-end epilogue, 16 no DMA waits in the loop, 32 no loop barriers, 64 no DMA
// issue in the loop, 128 no fragment reads in the loop
#ifndef W4_ABL
#define W4_ABL 0
#endif

typedef __attribute__((address_space(3))) void lds_void_t;
typedef short s16x2 __attribute__((ext_vector_type(2)));

template <int V> struct IC { static constexpr int value = V; };
template <typename F, int... Is> PCS_DEV void sfor_impl(F &&f, std::integer_sequence<int, Is...>) { (f(IC<Is>{}), ...); }
template <int N, typename F> PCS_DEV void sfor(F &&f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
PCS_DEV void sbar() { __builtin_amdgcn_sched_barrier(0); }
// One LDS-DMA piece: 64 lanes x 16 B from sbase + voff (per lane) to the LDS address m0 + 16 lane
// (m0 = m0base + OFF, set per piece; the caller saves and restores m0 around a group).
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
PCS_DEV void barrier_raw() {
  sbar();
  asm volatile("s_barrier" ::: "memory");
  sbar();
}
template <int N> PCS_DEV void wait_vm() {
  sbar();
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  sbar();
}
PCS_DEV void wait_lgkm0() {
  sbar();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  sbar();
}
template <int CTRL> PCS_DEV float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL> PCS_DEV int dppi(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
// max / min over the 32 lanes of a wave half (two DPP rows: butterfly in the row, then the
// partner row through v_permlane16_swap)
PCS_DEV float half_max(float v) {
  v = fmaxf(v, dppf<0xB1>(v)); v = fmaxf(v, dppf<0x4E>(v)); v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}
PCS_DEV int half_mini(int v) {
  v = min(v, dppi<0xB1>(v)); v = min(v, dppi<0x4E>(v)); v = min(v, dppi<0x141>(v));
  v = min(v, dppi<0x140>(v));
  const auto sw = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
  return min((int)sw[0], (int)sw[1]);
}
// a VALU read of an accumulator element: the "a" constraint keeps every use of the loop-carried
// accumulators in AGPRs (MFMA C/D and this), so the register allocator never bounces them
// through VGPRs (the caller pads the MFMA -> read latency before the first read of a tile)
PCS_DEV float aread(float x) {
  float r;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(x));
  return r;
}
PCS_DEV float max3f(float a, float b, float c) {
  float r;
  asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
PCS_DEV float max2f(float a, float b) {
  float r;
  asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// 8 bits (element e -> bit e) of "bf16 x > 0" over one 8-element fragment: as int16, a bf16 is
// > 0 exactly when its bit pattern is a positive integer (-0 = 0x8000 and negatives are < 1).
// The four dwords are named, not indexed: hipcc (ROCm 7.2) folded x[d] in an unrolled loop over d
// to x[0] for every d here (tools/dbg_w4.py caught it).
PCS_DEV uint32_t pos2(uint32_t x) {
  s16x2 v = __builtin_bit_cast(s16x2, x);
  v = __builtin_elementwise_max(__builtin_elementwise_min(v, s16x2{1, 1}), s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, v);   // element 2d -> bit 0, 2d + 1 -> bit 16
}
PCS_DEV uint32_t pos_bits8(const bf16x8 &f) {
  const u32x4 x = __builtin_bit_cast(u32x4, f);
  const uint32_t t = pos2(x.x) | (pos2(x.y) << 2) | (pos2(x.z) << 4) | (pos2(x.w) << 6);
  return (t | (t >> 15)) & 0xffu;
}
// the W row a lane loads for MFMA row position m (see the lane maps above)
PCS_DEV int wrow_of(int m) { return 16 * (m >> 4) + 8 * ((m >> 2) & 1) + (m & 3) + 4 * ((m >> 3) & 1); }
PCS_DEV int swz64(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

template <int MODE>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm_w4_kernel(pcs_gemm_args a, int tiles_per_scene, int tiles_per_chunk, int ncb) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float *lbias = reinterpret_cast<float *>(lds + OFF_BIAS);
  float *lsgn = reinterpret_cast<float *>(lds + OFF_SGN);
  float *lcur = reinterpret_cast<float *>(lds + OFF_CUR);
  float4 *runp = reinterpret_cast<float4 *>(lds + OFF_POOL);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int L = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  const int chunk = L / ncb, cb = L % ncb;
  const int cps = a.chunks_per_scene;
  const int scene = chunk / cps, cis = chunk % cps;
  const int n0 = cb * BN;
  const int K = a.K, Ncols = a.Ncols;
  const int64_t N = a.scene_rows;
  const int t_begin = cis * tiles_per_chunk;
  const int t_end = min(t_begin + tiles_per_chunk, tiles_per_scene);
  if (t_begin >= t_end) return;   // uniform across the workgroup
  const int nks = K / BK;
  const int total = (t_end - t_begin) * nks;
  // FWD: row tiles visited in the order t -> (t * P) mod n (gemm_glds.hip: spatially ordered
  // clouds make a column's running maximum grow tile after tile; a strided order settles it early)
  const int ntl = t_end - t_begin;
  int P = 1;
  if (MODE == MODE_FWD && ntl > 8) {
    constexpr int primes[6] = {97, 89, 83, 79, 73, 71};
#pragma unroll
    for (int i = 5; i >= 0; --i)
      if (primes[i] < ntl && ntl % primes[i] != 0) P = primes[i];
    P = __builtin_amdgcn_readfirstlane(P);
  }
  auto pnext = [&](int pt) __attribute__((always_inline)) { return pt + P >= ntl ? pt + P - ntl : pt + P; };
  const int64_t row0 = (int64_t)scene * N + (int64_t)t_begin * BM;
  const int64_t scene_end = (int64_t)(scene + 1) * N;
  const char *Ab = reinterpret_cast<const char *>(a.A);
  const char *Wb = reinterpret_cast<const char *>(a.W) + (int64_t)n0 * K * 2;
  const uint32_t rowbytes = (uint32_t)K * 2u;
  const char *Arow0 = Ab + row0 * rowbytes;
  const uint32_t tile_bytes = (uint32_t)BM * rowbytes;
  const int rows_left = (int)pcs_min64(scene_end - row0, (int64_t)ntl * BM);

  // ---- per-workgroup constants -> LDS (ordinary loads, all retired before the first DMA)
  if (tid < BN) {
    const float c = a.bias ? a.bias[n0 + tid] : 0.f;
    const uint32_t hi = pack2bf(c, 0.f) & 0xffffu;
    const float r1 = c - bf2f(hi);
    const uint32_t mid = pack2bf(r1, 0.f) & 0xffffu;
    const uint32_t lo = pack2bf(r1 - bf2f(mid), 0.f) & 0xffffu;
    *reinterpret_cast<u32x4 *>(lbias + 4 * tid) = mk_u32x4(hi | (mid << 16), lo, 0u, 0u);
    if (tid == 0) *reinterpret_cast<u32x4 *>(lbias + 4 * BN) = mk_u32x4(0u, 0u, 0u, 0u);
    if constexpr (MODE == MODE_FWD) {
      lsgn[tid] = (a.es && a.es[n0 + tid] < 0.f) ? -1.f : 1.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        runp[h * BN + tid] = make_float4(-__builtin_huge_valf(), __int_as_float(0x7fffffff),
                                         __builtin_huge_valf(), __int_as_float(0x7fffffff));
        lcur[h * BN + tid] = -__builtin_huge_valf();
      }
    }
  }
  __syncthreads();

  // ---- DMA: wave w stages pieces p = 4 w + q (q = 0..3) of every region, rows 16 p + lane / 4,
  // slot lane % 4 holding logical chunk lc = (lane & 3) ^ ((lane >> 4) & 3)
  const uint32_t lc16 = (uint32_t)(((lane & 3) ^ ((lane >> 4) & 3)) << 4);
  const int prow = 64 * wid + (lane >> 2);   // + 16 q
  uint32_t vW[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) vW[q] = (uint32_t)(prow + 16 * q) * rowbytes + lc16;
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  const uint32_t m0_wave = __builtin_amdgcn_readfirstlane(lds_m0 + wid * 4096);
  const int cw = wrow_of(lr);
  // (qseq, tile in visiting order, kt, half hh, group g): pieces q = 2g, 2g+1 of A-hh and W-hh
  auto issue = [&](int qseq, int ptl, int kt, int hh, int g) __attribute__((always_inline)) {
    if (qseq >= total) return;   // nothing left: the waits below shrink to match
    const uint32_t mA = __builtin_amdgcn_readfirstlane(lds_m0 + (qseq & 1) * KBUF + hh * REG + wid * 4096);
    const uint32_t mW = mA + 2 * REG;
    const int64_t rb = row0 + (int64_t)ptl * BM;
    const int valid = (int)pcs_min64(BM, scene_end - rb);
    const char *sa = Ab + rb * rowbytes + kt * 128 + hh * 64;
    const char *sw = Wb + kt * 128 + hh * 64;
    uint32_t va0 = (uint32_t)(prow + 32 * g) * rowbytes + lc16;
    uint32_t va1 = va0 + 16 * rowbytes;
    if (valid < BM) {   // uniform: a scene's last tile; rows past it re-read its last row
      va0 = (uint32_t)min(prow + 32 * g, valid - 1) * rowbytes + lc16;
      va1 = (uint32_t)min(prow + 32 * g + 16, valid - 1) * rowbytes + lc16;
    }
    const uint32_t keep = m0_save();
    if (g == 0) {
      glds16o<0>(sa, va0, mA);
      glds16o<1024>(sa, va1, mA);
      glds16o<0>(sw, vW[0], mW);
      glds16o<1024>(sw, vW[1], mW);
    } else {
      glds16o<2048>(sa, va0, mA);
      glds16o<3072>(sa, va1, mA);
      glds16o<2048>(sw, vW[2], mW);
      glds16o<3072>(sw, vW[3], mW);
    }
    m0_restore(keep);
  };

  // ---- fragment reads: a5 rows wm*128 + 32 i + lr, W rows wn*128 + 32 j + wrow_of(lr)
    int oA[2], oW[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    oA[t] = (wm * 128 + lr) * 64 + 16 * swz64(lr, 2 * t + lh);
    oW[t] = 2 * REG + (wn * 128 + cw) * 64 + 16 * swz64(cw, 2 * t + lh);
  }
  bf16x8 af[2][4], wf[2][4];   // [k-step parity][block]
  auto read_frags = [&](int set, int buf, int hh, int t) __attribute__((always_inline)) {
    const char *base = lds + buf * KBUF + hh * REG;
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[set][j] = *reinterpret_cast<const bf16x8 *>(base + oW[t] + j * 32 * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[set][i] = *reinterpret_cast<const bf16x8 *>(base + oA[t] + i * 32 * 64);
  };

  f32x16 acc[4][4];
  // One k-step as a hand-placed stream: the 16 MFMAs of fragment set SET, each followed by one
  // piece of the next k-step's work -- slots 0-3 the next W fragments, 4-7 the next a5
  // fragments (both from buffer nbuf, half NHH, k-step NT), 8-11 the DMA pieces of group G of half
  // HH of K-tile qseq -- with scheduling barriers between slots, so that the fragment reads and
  // the DMA issue run in the MFMAs' shadow instead of ahead of them.  The DMA is branch-free: a
  // K-tile past the chunk re-reads the chunk's first rows into the (free) region it would use,
  // so every wave issues the same pieces every k-step and one count serves every wait.
  auto kstep = [&](auto SETc, auto NHHc, auto NTc, auto HHc, auto Gc, int nbuf, int qseq, int ptl, int ktl,
                   auto &&ex) __attribute__((always_inline)) {
    constexpr int SET = decltype(SETc)::value, NSET = SET ^ 1, NHH = decltype(NHHc)::value;
    constexpr int NT = decltype(NTc)::value, HH = decltype(HHc)::value, G = decltype(Gc)::value;
    // 32-bit offsets from the chunk's first row (a chunk spans < 2^31 rows and < 2^32 bytes of
    // row tiles: pcs_gemm_w4_applicable), so the per-k-step address work stays a few SALU ops
    const bool live = qseq < total;
    const int pt = live ? ptl : 0, kk = live ? ktl : 0;
    const int valid = min(BM, rows_left - pt * BM);
    const char *sa = Arow0 + ((uint32_t)pt * tile_bytes + (uint32_t)(kk * 128 + HH * 64));
    const char *sw = Wb + (kk * 128 + HH * 64);
    const uint32_t va0 = (uint32_t)min(prow + 32 * G, valid - 1) * rowbytes + lc16;
    const uint32_t va1 = (uint32_t)min(prow + 32 * G + 16, valid - 1) * rowbytes + lc16;
    const uint32_t mA = m0_wave + (uint32_t)(qseq & 1) * KBUF + HH * REG;
    const uint32_t mW = mA + 2 * REG;
    const char *rbase = lds + nbuf * KBUF + NHH * REG;
    sbar();
    const uint32_t keep = m0_save();
    sfor<16>([&](auto Sc) __attribute__((always_inline)) {
      constexpr int S = decltype(Sc)::value, I = S >> 2, J = S & 3;
      acc[I][J] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[SET][J], af[SET][I], acc[I][J], 0, 0, 0);
      if constexpr (S < 4) { if (!(W4_ABL & 128)) wf[NSET][S] = *reinterpret_cast<const bf16x8 *>(rbase + oW[NT] + S * 32 * 64); }
      else if constexpr (S < 8) { if (!(W4_ABL & 128)) af[NSET][S - 4] = *reinterpret_cast<const bf16x8 *>(rbase + oA[NT] + (S - 4) * 32 * 64); }
      else if constexpr (W4_ABL & 64) {}
      else if constexpr (S == 8) glds16o<2048 * G>(sa, va0, mA);
      else if constexpr (S == 9) glds16o<2048 * G + 1024>(sa, va1, mA);
      else if constexpr (S == 10) glds16o<2048 * G>(sw, vW[2 * G], mW);
      else if constexpr (S == 11) glds16o<2048 * G + 1024>(sw, vW[2 * G + 1], mW);
      ex(Sc);   // the caller's work for this slot (epilogue pieces)
      sbar();
    });
    m0_restore(keep);
  };
  // bias as an MFMA: A' = the split bias of the lane's W row at k = 0..2 (lane half 0; half 1
  // reads the zero row), B' = ones at k = 0..2, so mfma(A', B', 0) = c[column] exactly
  const int obias = lh ? 16 * BN : 16 * (wn * 128 + cw);
  auto bias_frag = [&](int j) __attribute__((always_inline)) {
    return *reinterpret_cast<const bf16x8 *>(reinterpret_cast<const char *>(lbias) + obias + (lh ? 0 : 16 * 32 * j));
  };
  const u32x4 ones_u = lh ? mk_u32x4(0u, 0u, 0u, 0u) : mk_u32x4(0x3f803f80u, 0x3f80u, 0u, 0u);
  const bf16x8 ones_f = __builtin_bit_cast(bf16x8, ones_u);
  const f32x16 zero16 = {};

  // DGRAD state: the previous tile, bf16-packed, waiting for its mask and stores
  uint32_t pk[4][4][8];
  uint32_t mcur[4][2], mprev[4][2];   // mask bits [i][j >> 1]: bit 16 (j & 1) + q <-> register q
  // the previous tile's output rows through a buffer descriptor whose range ends at its last
  // valid row: a store past it is dropped by the hardware, so every lane issues both stores of
  // every block -- the counted waits below then see a fixed number of stores per k-step
  bf16_t *Cg = reinterpret_cast<bf16_t *>(a.C);
  auto tile_rsrc = [&](int64_t rb, int valid) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char *>(Cg + rb * (int64_t)Ncols), 0,
                                             (int)((uint32_t)valid * (uint32_t)Ncols * 2u), 0x00020000);
  };
  __amdgpu_buffer_rsrc_t rs_prev = tile_rsrc(0, 0);
  const int kqa0 = (n0 + 128 * wn) / BK;   // K-tiles holding this wave's mask columns: kqa0, +1
  const uint32_t o_st = (uint32_t)(((wm * 128 + lr) * Ncols + n0 + wn * 128 + 8 * lh) * 2);
  // mask + store of half H (columns 16 H + 8 lh + 0..7) of block (I, J) of a finished tile
  auto flush_half = [&](auto Ic, auto Jc, auto Hc, const uint32_t (&mw)[4][2], __amdgpu_buffer_rsrc_t rs) __attribute__((always_inline)) {
    constexpr int I = decltype(Ic)::value, J = decltype(Jc)::value, H = decltype(Hc)::value;
    const uint32_t w = mw[I][J >> 1] >> (16 * (J & 1) + 8 * H);
    uint32_t v[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)w, 2 * d, 1);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)w, 2 * d + 1, 1);
      v[d] = pk[I][J][4 * H + d] & ((lo & 0xffffu) | (hi << 16));
    }
    // one lane offset for every block: the block's row step on the scalar offset, its column
    // step in the instruction's immediate
    const int so = __builtin_amdgcn_readfirstlane(I * 32 * Ncols * 2);
    __builtin_amdgcn_raw_buffer_store_b128(mk_u32x4(v[0], v[1], v[2], v[3]), rs, (int)o_st + 64 * J + 32 * H, so, 0);
  };
  // read out accumulator block (I, J) into pk (DGRAD)
  auto pack_block = [&](auto Ic, auto Jc) __attribute__((always_inline)) {
    constexpr int I = decltype(Ic)::value, J = decltype(Jc)::value;
    sbar();
#pragma unroll
    for (int d = 0; d < 8; ++d) pk[I][J][d] = pack2bf(aread(acc[I][J][2 * d]), aread(acc[I][J][2 * d + 1]));
    sbar();
  };

  // FWD: the max-pool update of column block j from the accumulators of the finished tile
  // (rows rb + wm*128 + 32 i + lr; valid rows only)
  auto pool_block = [&](auto Jc, int64_t rb, int valid) __attribute__((always_inline)) {
    constexpr int J = decltype(Jc)::value;
    sbar();
    // per-call opaque base (no loop-invariant hoisting of 16 x 3 LDS addresses per column block)
    int cbase = wn * 128 + 8 * lh;
    asm volatile("" : "+v"(cbase));
    const float *cur = lcur + wm * BN + cbase + 32 * J;
    const float4 c0 = *reinterpret_cast<const float4 *>(cur), c1 = *reinterpret_cast<const float4 *>(cur + 4);
    const float4 c2 = *reinterpret_cast<const float4 *>(cur + 16), c3 = *reinterpret_cast<const float4 *>(cur + 20);
    const float cc[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
    const bool full = valid == BM;
    uint32_t okr = 0;   // bit i: row wm*128 + 32 i + lr of the tile is in the scene
#pragma unroll
    for (int i = 0; i < 4; ++i) okr |= (uint32_t)(wm * 128 + 32 * i + lr < valid) << i;
    float vx[16];
    bool beat = false;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (full) {
        vx[q] = max2f(max3f(aread(acc[0][J][q]), aread(acc[1][J][q]), aread(acc[2][J][q])), aread(acc[3][J][q]));
      } else {
        float m = -__builtin_huge_valf();
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if ((okr >> i) & 1u) m = fmaxf(m, aread(acc[i][J][q]));
        vx[q] = m;
      }
      beat |= vx[q] >= cc[q];   // >=: an equal value may sit on an earlier row
    }
    sbar();
    if (__builtin_amdgcn_ballot_w64(beat) == 0) return;   // uniform: the fast path
    // slow path: per register q, the column's tile maximum over the half's 32 lanes and its
    // first row; lane lr == q of each half then merges it into the running (max, row)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float m = half_max(vx[q]);
      if (__builtin_amdgcn_ballot_w64(m >= cc[q]) == 0) continue;
      int ix = 0x7fffffff;
#pragma unroll
      for (int i = 3; i >= 0; --i)
        if (((okr >> i) & 1u) && aread(acc[i][J][q]) == m) ix = (int)(rb + wm * 128 + 32 * i + lr);
      ix = half_mini(ix);
      if (lr == q && m >= cc[q]) {
        const int col = cbase + 32 * J + 16 * (q >> 3) + (q & 7);
        const int cme = wm * BN + col;
        const float4 old = runp[cme];
        const float sgl = lsgn[col];
        const float curv = sgl > 0.f ? old.x : -old.z;
        const int curix = __float_as_int(sgl > 0.f ? old.y : old.w);
        if (m > curv || ix < curix) {
          float4 u = old;
          if (sgl > 0.f) { u.x = m; u.y = __int_as_float(ix); }
          else { u.z = -m; u.w = __int_as_float(ix); }
          runp[cme] = u;
          lcur[cme] = m;
        }
      }
    }
  };

  // ---- prologue: the steady state at k-step 0 of K-tile 0 (both halves of 0, half 0 of 1 and
  // group 0 of half 1 of 1 issued), K-tile 0's half 0 landed, F(0,0) read
  const int tl1 = nks == 1 ? pnext(0) : 0, kt1 = nks == 1 ? 0 : 1;
  issue(0, 0, 0, 0, 0); issue(0, 0, 0, 0, 1); issue(0, 0, 0, 1, 0); issue(0, 0, 0, 1, 1);
  issue(1, tl1, kt1, 0, 0); issue(1, tl1, kt1, 0, 1); issue(1, tl1, kt1, 1, 0);
  wait_vm<0>();
  barrier_raw();
  read_frags(0, 0, 0, 0);
  wait_lgkm0();

  // DGRAD work placed in the MFMA slots of k-step KS (fragment set SET): the mask bits of the
  // a5 fragments in the wave's two mask K-tiles (slots 1, 3, 5, 7: i = 0..3; mcur[i][u] collects
  // k-steps 0..3 of K-tile kqa0 + u), and block (kt - 1, KS) of the previous tile in K-tiles
  // 1..4 (slots 12, 14: its two halves).  Both words of mcur go through selects: an if / else
  // on u lets LLVM index mcur by u, and the array then lives in memory.
  auto mask_piece = [&](auto SETc, auto KSc, auto Ic, int u) __attribute__((always_inline)) {
    constexpr int SET = decltype(SETc)::value, KS = decltype(KSc)::value, i = decltype(Ic)::value;
    const bool u0 = u == 0;
    const uint32_t b = pos_bits8(af[SET][i]) << (8 * KS);
    const uint32_t m0 = KS == 0 ? 0u : mcur[i][0], m1 = KS == 0 ? 0u : mcur[i][1];
    mcur[i][0] = u0 ? (m0 | b) : mcur[i][0];
    mcur[i][1] = u0 ? mcur[i][1] : (m1 | b);
  };
  auto slot_work = [&](auto SETc, auto KSc, bool do_mask, int u, bool do_defer, int kt) __attribute__((always_inline)) {
    return [&, SETc, KSc, do_mask, u, do_defer, kt](auto Sc) __attribute__((always_inline)) {
      constexpr int S = decltype(Sc)::value;
      if constexpr (MODE != MODE_DGRAD) {
        (void)SETc; (void)KSc; (void)do_mask; (void)u; (void)do_defer; (void)kt;
      } else {
        if constexpr ((S & 1) && S < 8) {
          if (!(W4_ABL & 2) && do_mask) mask_piece(SETc, KSc, IC<(S >> 1)>{}, u);
        } else if constexpr (S == 12 || S == 14) {
          if (!(W4_ABL & 4) && do_defer) {
            constexpr int H = S == 14;
            switch (kt) {
              case 1: flush_half(IC<0>{}, KSc, IC<H>{}, mprev, rs_prev); break;
              case 2: flush_half(IC<1>{}, KSc, IC<H>{}, mprev, rs_prev); break;
              case 3: flush_half(IC<2>{}, KSc, IC<H>{}, mprev, rs_prev); break;
              default: flush_half(IC<3>{}, KSc, IC<H>{}, mprev, rs_prev); break;
            }
          }
        }
      }
    };
  };

  // The counted waits at barriers X and Y: 16 DMA pieces are newer than the ones awaited, plus
  // (DGRAD) the deferred stores issued since -- vector memory operations retire in order, so a
  // count that left them out would wait for the stores too.  Two stores per k-step of K-tiles
  // 1..4 (none in a chunk's first tile, K >= 6 * 64 so none in a tile's last K-tile):
  //   X (awaits K-tile kt-1's k-step 0 DMA): + 8 [kt-1 in 1..4] + 2 [kt in 1..4]
  //   Y (awaits K-tile kt-1's k-step 2 DMA): + 4 [kt-1 in 1..4] + 6 [kt in 1..4]
  auto wait_x = [&](int dn) __attribute__((always_inline)) {
    switch (dn) {
      case 1: wait_vm<18>(); break;
      case 2: case 3: case 4: wait_vm<26>(); break;
      case 5: wait_vm<24>(); break;
      default: wait_vm<16>(); break;
    }
  };
  auto wait_y = [&](int dn) __attribute__((always_inline)) {
    switch (dn) {
      case 1: wait_vm<22>(); break;
      case 2: case 3: case 4: wait_vm<26>(); break;
      case 5: wait_vm<20>(); break;
      default: wait_vm<16>(); break;
    }
  };
  // (row tile, K-tile) of qs+1 and qs+2 as loop counters (no divisions); p*: visiting order
  int ka = 0, pa = 0;
  int qs = 0;
  int pcur = 0;
  int64_t rb_cur = row0;
  int valid_cur = 0;
  for (int tcur = 0; tcur < ntl; ++tcur) {
    rb_cur = row0 + (int64_t)pcur * BM;
    valid_cur = (int)pcs_min64(BM, scene_end - rb_cur);
    // every accumulator starts from the bias (exact: hi + mid + lo against ones)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bf16x8 bfj = bias_frag(j);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfj, ones_f, zero16, 0, 0, 0);
    }
    for (int kt = 0; kt < nks; ++kt, ++qs) {
      const int buf = qs & 1;
      const bool w1 = kt + 1 == nks;
      pa = w1 ? pnext(pcur) : pcur;
      ka = w1 ? 0 : kt + 1;
      const bool w2 = ka + 1 == nks;
      const int kb = w2 ? 0 : ka + 1;
      const int pb = w2 ? pnext(pa) : pa;
      const int u = kt - kqa0;                         // DGRAD: 0 / 1 in this wave's mask K-tiles
      const bool do_mask = MODE == MODE_DGRAD && (unsigned)u < 2u;
      const bool do_defer = MODE == MODE_DGRAD && tcur > 0 && kt >= 1 && kt <= 4;
      const int dn = MODE == MODE_DGRAD && tcur > 0 ? kt : 0;   // the barriers' store counts

      // ======== k-step 0: F(qs,0) in set 0; read F(qs,1); DMA group 1 of half 1 of qs+1
      kstep(IC<0>{}, IC<0>{}, IC<1>{}, IC<1>{}, IC<1>{}, buf, qs + 1, pa, ka,
            slot_work(IC<0>{}, IC<0>{}, do_mask, u, do_defer, kt));
      wait_lgkm0();
      // barrier X: half 0 of buf is free (every wave retired its reads before arriving); half 1
      // of qs landed (newer: both halves of qs+1, 16 pieces)
      if (!(W4_ABL & 16)) wait_x(dn);
      if (!(W4_ABL & 32)) barrier_raw();

      // ======== k-step 1: F(qs,1) in set 1; read F(qs,2); DMA group 0 of half 0 of qs+2
      kstep(IC<1>{}, IC<1>{}, IC<0>{}, IC<0>{}, IC<0>{}, buf, qs + 2, pb, kb,
            slot_work(IC<1>{}, IC<1>{}, do_mask, u, do_defer, kt));
      wait_lgkm0();

      // ======== k-step 2: F(qs,2) in set 0; read F(qs,3); DMA group 1 of half 0 of qs+2
      kstep(IC<0>{}, IC<1>{}, IC<1>{}, IC<0>{}, IC<1>{}, buf, qs + 2, pb, kb,
            slot_work(IC<0>{}, IC<2>{}, do_mask, u, do_defer, kt));
      wait_lgkm0();
      // barrier Y: half 1 of buf is free; half 0 of qs+1 landed (newer: half 1 of qs+1, half 0
      // of qs+2)
      if (!(W4_ABL & 16)) wait_y(dn);
      if (!(W4_ABL & 32)) barrier_raw();

      // ======== k-step 3: F(qs,3) in set 1; read F(qs+1,0); DMA group 0 of half 1 of qs+2
      kstep(IC<1>{}, IC<0>{}, IC<0>{}, IC<1>{}, IC<0>{}, buf ^ 1, qs + 2, pb, kb,
            slot_work(IC<1>{}, IC<3>{}, do_mask, u, do_defer, kt));
      wait_lgkm0();
    }
    pcur = pa;
    if (tcur + 1 == ntl) break;   // the last tile's epilogue runs after the loop
    // the finished tile out of the accumulators: DGRAD bf16-packed for the next tile's K-tiles
    // 1..4 (mask + stores); FWD max-pool
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");   // MFMA results before VALU reads
    if constexpr (MODE == MODE_DGRAD) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { mprev[i][0] = mcur[i][0]; mprev[i][1] = mcur[i][1]; }
      rs_prev = tile_rsrc(rb_cur, valid_cur);
      if (!(W4_ABL & 1)) sfor<4>([&](auto Ic) __attribute__((always_inline)) { sfor<4>([&](auto Jc) __attribute__((always_inline)) { pack_block(Ic, Jc); }); });
    } else {
      if (!(W4_ABL & 1)) sfor<4>([&](auto Jc) __attribute__((always_inline)) { pool_block(Jc, rb_cur, valid_cur); });
    }
  }
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  wait_vm<0>();   // the re-read DMAs past the chunk

  // ---- chunk end: the last tile
  if (W4_ABL & 8) return;
  if constexpr (MODE == MODE_DGRAD) {
    const __amdgpu_buffer_rsrc_t rs_last = tile_rsrc(rb_cur, valid_cur);
    sfor<4>([&](auto Ic) __attribute__((always_inline)) { sfor<4>([&](auto Jc) __attribute__((always_inline)) { pack_block(Ic, Jc); }); });
    sfor<4>([&](auto Ic) __attribute__((always_inline)) { sfor<4>([&](auto Jc) __attribute__((always_inline)) { flush_half(Ic, Jc, IC<0>{}, mcur, rs_last); flush_half(Ic, Jc, IC<1>{}, mcur, rs_last); }); });
  } else {
    sfor<4>([&](auto Jc) __attribute__((always_inline)) { pool_block(Jc, rb_cur, valid_cur); });
    __syncthreads();
    if (tid < BN && a.pool) {
      const int64_t o = (int64_t)chunk * Ncols + n0 + tid;
      float4 p = runp[tid];
      const float4 q = runp[BN + tid];
      const int pi = __float_as_int(p.y), qi = __float_as_int(q.y);
      const int pj = __float_as_int(p.w), qj = __float_as_int(q.w);
      if (q.x > p.x || (q.x == p.x && qi < pi)) { p.x = q.x; p.y = q.y; }
      if (q.z < p.z || (q.z == p.z && qj < pj)) { p.z = q.z; p.w = q.w; }
      *reinterpret_cast<float4 *>(a.pool + o * 4) = p;
    }
  }
}

}  // namespace

// forward: max-pool on sign-folded W rows only (no statistics, no C); input gradient: folded
// form with bias, mask from the operand, no statistics / addend / sparse rows (those run
// elsewhere); bf16, K % 128 == 0, Ncols % 256 == 0
bool pcs_gemm_w4_applicable(const pcs_gemm_args &a) {
  if (a.dtype != PCS_BF16 || !(a.flags & PCS_FLAG_W4) || (a.flags & (PCS_FLAG_GENERIC | PCS_FLAG_NO_GLDS | PCS_FLAG_AW_FP8)))
    return false;
  if (a.prologue != PCS_PRO_RAW || a.K % (2 * BK) != 0 || a.Ncols % BN != 0 || a.stats) return false;
  // a chunk's row tiles addressed by 32-bit offsets (after pcs_gemm_geometry)
  if (a.chunks_per_scene <= 0) return false;
  const int64_t tps = (a.scene_rows + BM - 1) / BM, tpc = (tps + a.chunks_per_scene - 1) / a.chunks_per_scene;
  if (tpc * BM * a.K * 2 > 0xffffffffLL) return false;
  if (a.epilogue == PCS_EPI_FWD)
    return a.C == nullptr && a.scene_bias == nullptr && a.pool && a.es && (a.flags & PCS_FLAG_POOL_SIGNED_W);
  if (a.epilogue == PCS_EPI_DGRAD)   // the deferred stores use K-tiles 1..4 (not the last): K >= 6 * 64
    return a.K >= 6 * BK && a.Yp == a.A && a.K == a.Ncols && !a.es && !a.et && !a.erstd && !a.addend && !a.c_mask && !a.pool_w;
  return false;
}

int pcs_gemm_w4_launch(const pcs_gemm_args &g, int tps, int tpc, hipStream_t s) {
  const int ncb = g.Ncols / BN;
  const int nb = ncb * (int)(g.num_scenes * g.chunks_per_scene);
  if (g.epilogue == PCS_EPI_FWD)
    hipLaunchKernelGGL((gemm_w4_kernel<MODE_FWD>), dim3(nb), dim3(THREADS), 0, s, g, tps, tpc, ncb);
  else
    hipLaunchKernelGGL((gemm_w4_kernel<MODE_DGRAD>), dim3(nb), dim3(THREADS), 0, s, g, tps, tpc, ncb);
  PCS_CHECK_LAUNCH();
  return 0;
}

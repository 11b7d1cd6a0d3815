// Streaming forward pass of a narrow-K 1x1 Conv1d with the previous layer's BN + ReLU (+ dropout)
// applied to its input (P:106-110, P:123-128):
//
//   x   = relu(Yp * s + t) [* keep * ks]          (PCS_PRO_BNRELU, per input channel)
//   y   = x W^T (+ bias | + scene bias)            stored bf16; per-chunk (mean, M2) of the stored
//                                                   values (PCS_EPI_FWD)
//   or  a = relu(y * es + et)                       stored bf16; per-chunk column sums of the stored
//                                                   values (PCS_EPI_BNRELU: conv5 -> a5)
//
// The register-staged kernels (gemm_nt.hip 128x128, gemm_big.hip 256x256) ran these at
// 2.8-3.6 TB/s: their prologue transforms every operand fragment once per column wave, their
// epilogue stages the tile through LDS, and each k-step is a barrier.  Here:
// * a workgroup (8 waves) owns NB output columns of a scene-aligned row slice; each wave keeps its
//   WC columns of W for the whole slice in registers as MFMA A operands (W rows = output
//   channels), so only the activations stream;
// * MS-row steps of Yp (and its dropout bits) come through an NST-stage LDS ring by LDS-DMA
//   (global_load_lds_dwordx4), counted waits (loads and stores retire in issue order on vmcnt;
//   every wave issues the same loads and stores per step, clamped or range-dropped past the
//   slice end), two steps in flight while one computes;
// * the BN + ReLU (+ dropout through an LDS table of AND masks) is applied once per element, in
//   place in LDS, one step ahead of the MFMAs;
// * the epilogue works on the accumulators in registers: lane = 4 consecutive channels of one
//   row; bias, rounding to bf16, statistics of the rounded values (per-lane shifted sums, merged
//   with Chan's formula at the slice end), 16-B stores widened with v_permlane16_swap through a
//   buffer descriptor whose range ends at the slice's last row.
// The 16-B slots of an LDS row hold the source chunks XOR-permuted by the row (put on the DMA
// source address, since the DMA writes LDS linearly), so the B-fragment reads (16 rows, one
// chunk) are bank-conflict free.
#include "common.h"

namespace {

constexpr int THREADS = 512;

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

// Shapes (K = input channels, NCOLS = output channels) and their tiling:
//   NB output columns per workgroup, WCN wave columns (8 / WCN wave rows), MS rows per step,
//   NST ring stages.
template <int K, int NCOLS> struct FsCfg;
// TARGET: workgroups in the grid (256 = one per CU; the small 64-wide layers, whose workgroups
// fit several to a CU, take more)
template <> struct FsCfg<64, 512> {   // seg_conv1 (local half)
  static constexpr int NB = 512, WCN = 8, MS = 64, NST = 4, TARGET = 256;
};
template <> struct FsCfg<512, 256> {   // seg_conv2
  static constexpr int NB = 256, WCN = 8, MS = 32, NST = 4, TARGET = 256;
};
template <> struct FsCfg<256, 128> {   // seg_conv3
  static constexpr int NB = 128, WCN = 4, MS = 64, NST = 4, TARGET = 256;
};
template <> struct FsCfg<128, 1024> {  // conv5 (BN5 + ReLU on the way out: a5)
  static constexpr int NB = 512, WCN = 8, MS = 64, NST = 4, TARGET = 256;
};
#ifndef FS_SMALL_TARGET
#define FS_SMALL_TARGET 1024
#endif
template <> struct FsCfg<64, 128> {    // conv4
  static constexpr int NB = 128, WCN = 4, MS = 64, NST = 4, TARGET = FS_SMALL_TARGET;
};
template <> struct FsCfg<64, 64> {     // conv2, conv3
  static constexpr int NB = 64, WCN = 2, MS = 64, NST = 4, TARGET = FS_SMALL_TARGET;
};

#ifndef FS_STG
#define FS_STG 1
#endif
#ifndef FS_ILV
#define FS_ILV 1
#endif
#ifndef FS_CPOL
#define FS_CPOL 2   // cache policy bits of the staged (STG) output stores: 2 = nt
#endif

template <int K, int NCOLS, bool MASK, bool C8 = false> struct FsGeo {
  typedef FsCfg<K, NCOLS> C;
  static constexpr int NB = C::NB, WCN = C::WCN, MS = C::MS, NST = C::NST;
  static constexpr int WRN = 8 / WCN;          // wave rows
  static constexpr int WC = NB / WCN;          // columns per wave
  // 128-B wave rows (WC = 64): the output goes through a per-wave LDS tile and leaves as 8 rows x
  // 128 B per store instruction (16 rows x 64 B straight from the MFMA layout otherwise)
  // FS_STG 2: the whole step's [MS][NB] tile is staged and each store instruction writes one
  // NB * 2 = 1 KB row, after the step's first barrier (all waves' parts of the tile written)
  // C8 (the fp8 e4m3 a5 of cfg5): 64-B wave rows, staged, 16 rows x 64 B per store
  static constexpr int STG = C8 ? 1 : (FS_STG && WC == 64) ? ((FS_STG == 2 && NB == 512 && WRN == 1) ? 2 : 1) : 0;
  static constexpr int ESZ = C8 ? 1 : 2;                  // output element bytes
  // the transform of step t+1 between the MFMA k-step groups of step t (its DMA waited for
  // before them) instead of after the epilogue; not with STG 2 (stores after the first barrier).
  // Measured (profiles/ab_r03_fwd_stream.md): seg_conv1 1.98 -> 1.89 ms, but seg_conv2 2.96 ->
  // 3.03, seg_conv3 1.33 -> 1.35, conv5 3.68 -> 3.71 (the earlier wait costs them prefetch depth)
  static constexpr bool ILV = FS_ILV && STG != 2 && K == 64;
  static constexpr int SROW = WC * ESZ;                   // staged wave-row bytes (128 or 64)
  static constexpr int CT = WC / 16;           // 16-column MFMA tiles per wave
  static constexpr int RW = MS / WRN;          // rows per wave per step
  static constexpr int RT = RW / 16;           // 16-row MFMA tiles per wave
  static constexpr int KS = K / 32;            // MFMA k-steps
  static constexpr int ROWB = K * 2;           // bytes per LDS row
  static constexpr int SPR = K / 8;            // 16-B slots per row
  static constexpr int XB = MS * ROWB;         // Yp slab per stage
  static constexpr int MKB = MASK ? MS * K / 8 : 0;   // dropout bits per stage
  static constexpr int STAGE = XB + MKB;
  static constexpr int PPW = XB / 1024 / 8;    // 1-KB DMA pieces per wave per step
  static constexpr int MPW = MKB / 256 / 8;    // 256-B (dword) DMA pieces per wave per step
  static constexpr int OFF_LUT = NST * STAGE;  // dropout byte -> 4 AND masks of packed bf16
  static constexpr int OFF_RED = OFF_LUT + (MASK ? 256 * 16 : 0);   // chunk-end merge [WRN][NB] float4
  static constexpr int OFF_STG = OFF_RED + WRN * NB * 16;             // [8 waves][RW][WC] bf16 (STG)
  static constexpr int BYTES = OFF_STG + (STG ? 8 * RW * SROW : 0);   // (STG 2: MS * NB * 2, the same)
  static constexpr int LPS = PPW + MPW;        // vector-memory loads per wave per step
  static constexpr int SPS = STG == 2 ? MS / 8 : STG ? RW * SROW / 1024 : (CT / 2) * RT;   // stores per wave per step
  // vector-memory operations newer than step t+1's DMA at the loop's wait (STG 2 stores step t
  // only after it)
  static constexpr int WAIT_N = (NST - 2) * (LPS + SPS) + (STG == 2 ? 0 : SPS);
  static constexpr int TPASS = MS * SPR / THREADS;   // transform passes (slots per thread)
  static_assert(NCOLS % NB == 0 && NB % WCN == 0 && WC % 32 == 0, "column tiling (CT even)");
  static_assert(MS % (16 * WRN) == 0 && XB % 8192 == 0 && PPW >= 1, "row tiling / DMA pieces");
  static_assert(!MASK || (MKB % 2048 == 0 && MPW >= 1), "dropout-bit pieces");
  static_assert(K % 32 == 0 && ROWB <= 1024 && (MS * SPR) % THREADS == 0, "K");
  static_assert(BYTES <= 160 * 1024, "LDS budget");
  static_assert(!C8 || (WC == 64 && RW % 16 == 0), "fp8 output staging");
};

// physical 16-B slot of logical slot c in LDS row r: c ^ f(r), f distinct over the 16 rows a
// ds_read_b128 lane group touches at one logical slot (128-B rows hold two rows per bank row)
template <int K> PCS_DEV int fsw(int r) { return K == 64 ? ((r >> 1) & 7) : (r & 15); }

// GRAM (conv3: K = NCOLS = 64, one workgroup per chunk): the chunk's x^T x and column sums of
// the transformed operand x = relu(bn2(y2)) = a2, from the stage the MFMAs read (transposed
// ds_read_b64_tr_b16 fragments, k = rows; rows past the slice are zeroed by the transform).
// Wave w accumulates the 16 x 16 blocks (w / 2, 2 (w % 2)) and (w / 2, 2 (w % 2) + 1) of the
// full 64 x 64 product; the column sums come from the transform (each thread's 8 channels,
// summed over its rows, then over the threads of those channels at the chunk end).
template <int K, int NCOLS, int EPI, bool MASK, bool SBIAS, bool C8 = false, bool GRAM = false>
__global__ __launch_bounds__(THREADS) void fwd_stream_kernel(pcs_gemm_args a, int64_t rows_per_chunk) {
  typedef FsGeo<K, NCOLS, MASK, C8> F;
  static_assert(!C8 || EPI == PCS_EPI_BNRELU, "fp8 output: the BN+ReLU epilogue (a5)");
  static_assert(!GRAM || (K == 64 && NCOLS == 64 && EPI == PCS_EPI_FWD && !MASK && !SBIAS && !C8 && F::ILV),
                "Gram of the operand: conv3 only");
  constexpr int NB = F::NB, MS = F::MS, NST = F::NST, CT = F::CT, RT = F::RT, KS = F::KS;
  constexpr int ROWB = F::ROWB, SPR = F::SPR;
  constexpr int NCB = NCOLS / NB;
  __shared__ __attribute__((aligned(16))) char lds[F::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid % F::WCN, wr = wid / F::WCN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = __builtin_amdgcn_readfirstlane(L / NCB), n0 = __builtin_amdgcn_readfirstlane((L % NCB) * NB);
  const int cps = a.chunks_per_scene;
  const int scene = __builtin_amdgcn_readfirstlane(chunk / cps), cis = __builtin_amdgcn_readfirstlane(chunk % cps);
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)cis * rows_per_chunk;
  const int64_t hi = pcs_min64(lo + rows_per_chunk, N);
  const int64_t sbase = (int64_t)scene * N;
  const int nsteps = (int)((hi - lo + MS - 1) / MS);   // >= 1 (no empty chunks)
  const char *Xg = reinterpret_cast<const char *>(a.A);
  const char *Mg = MASK ? reinterpret_cast<const char *>(a.a_mask) : nullptr;
  const bf16_t *Wg = reinterpret_cast<const bf16_t *>(a.W);

  const int l16 = lane & 15, g = lane >> 4;
  const int col0 = n0 + wc * F::WC;   // this wave's first output column
  // ---- W fragments (A operand: lane = output channel col0 + 16 ct + l16, k chunk 4 kk + g) and
  // the per-lane epilogue constants of its channels c = col0 + 16 ct + 4 g + r
  u32x4 wfr[CT][KS];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
      wfr[ct][kk] = *reinterpret_cast<const u32x4 *>(Wg + (int64_t)(col0 + 16 * ct + l16) * K + (4 * kk + g) * 8);
  float eb[CT][4], es[CT][4];   // FWD: bias; BNRELU: shift (et + bias es) and scale
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = col0 + 16 * ct + 4 * g + r;
      const float b = SBIAS ? a.scene_bias[(int64_t)scene * NCOLS + c] : (a.bias ? a.bias[c] : 0.f);
      if constexpr (EPI == PCS_EPI_BNRELU) {
        es[ct][r] = a.es[c];
        eb[ct][r] = a.et[c] + b * a.es[c];
      } else {
        es[ct][r] = 0.f;
        eb[ct][r] = b;
      }
    }
  // transform: thread -> logical slot tc (fixed: its 8 input channels' BN coefficients in
  // registers) of rows trow + p * (THREADS / SPR)
  const int tc = tid % SPR, trow = tid / SPR;
  float ts[8], tt[8];
  {
    const float4 s0 = *reinterpret_cast<const float4 *>(a.pa + 8 * tc);
    const float4 s1 = *reinterpret_cast<const float4 *>(a.pa + 8 * tc + 4);
    const float4 t0 = *reinterpret_cast<const float4 *>(a.pb + 8 * tc);
    const float4 t1 = *reinterpret_cast<const float4 *>(a.pb + 8 * tc + 4);
    // with dropout the kept values are relu(y s + t) ks = relu(y (s ks) + t ks) (ks = 1 / (1 - p) > 0),
    // then ANDed with the keep masks: the keep scale is folded into the coefficients
    const float ks = MASK ? a.a_keep_scale : 1.f;
    ts[0] = s0.x; ts[1] = s0.y; ts[2] = s0.z; ts[3] = s0.w; ts[4] = s1.x; ts[5] = s1.y; ts[6] = s1.z; ts[7] = s1.w;
    tt[0] = t0.x; tt[1] = t0.y; tt[2] = t0.z; tt[3] = t0.w; tt[4] = t1.x; tt[5] = t1.y; tt[6] = t1.z; tt[7] = t1.w;
#pragma unroll
    for (int e = 0; e < 8; ++e) { ts[e] *= ks; tt[e] *= ks; }
  }
  if constexpr (MASK) {   // dropout byte -> the AND masks of 8 packed bf16 values
    if (tid < 256) {
      uint32_t *lut = reinterpret_cast<uint32_t *>(lds + F::OFF_LUT) + tid * 4;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        lut[d] = (((tid >> (2 * d)) & 1) ? 0x0000FFFFu : 0u) | (((tid >> (2 * d + 1)) & 1) ? 0xFFFF0000u : 0u);
    }
  }
  // Every ordinary load above retires here, before the first DMA: the empty asm uses make hipcc
  // place its own wait for them now (its wait counting does not see the inline-asm DMAs, so a
  // wait it placed later would drain the DMA pipeline).  From here on no ordinary global load.
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) asm volatile("" ::"v"(wfr[ct][kk]));
#pragma unroll
    for (int r = 0; r < 4; ++r) asm volatile("" ::"v"(eb[ct][r]), "v"(es[ct][r]));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(ts[e]), "v"(tt[e]));
  __syncthreads();

  // ---- DMA of step s into stage sidx.  Piece j = wid + 8 i (1 KB): rows j * (1024 / ROWB) +
  // lane / SPR, physical slot lane % SPR holding logical slot (lane % SPR) ^ f(row); dropout
  // bits: dword piece wid + 8 i of the step's contiguous MS * K / 8 bytes.  Rows past the slice
  // clamp to its last row (their outputs are dropped, their statistics skipped).
  auto piece_off = [&](int i, int lastr) -> uint32_t {
    const int j = wid + 8 * i;
    const int r = j * (1024 / ROWB) + lane / SPR, ps = lane % SPR;
    const int rc = min(r, lastr);
    return (uint32_t)(rc * ROWB + ((ps ^ fsw<K>(r)) << 4));
  };
  auto mask_off = [&](int i, int lastr) -> uint32_t {
    const int byte = (wid + 8 * i) * 256 + lane * 4;
    const int r = byte / (K / 8);
    return (uint32_t)(min(r, lastr) * (K / 8) + byte % (K / 8));
  };
  uint32_t voff[F::PPW + F::MPW];
#pragma unroll
  for (int i = 0; i < F::PPW; ++i) voff[i] = piece_off(i, MS - 1);
#pragma unroll
  for (int i = 0; i < F::MPW; ++i) voff[F::PPW + i] = mask_off(i, MS - 1);
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  auto dma_issue = [&](int sidx, int64_t m0, const uint32_t (&vo)[F::PPW + F::MPW]) {
    const uint32_t mb = lds_m0 + sidx * F::STAGE + wid * 1024;
    const char *bx = Xg + (sbase + m0) * ROWB;
    const uint32_t keep = m0_save();
    glds16o<0>(bx, vo[0], mb);
    if constexpr (F::PPW > 1) glds16o<8192>(bx, vo[1], mb);
    if constexpr (F::PPW > 2) glds16o<16384>(bx, vo[2], mb);
    if constexpr (F::PPW > 3) glds16o<24576>(bx, vo[3], mb);
    static_assert(F::PPW <= 4, "pieces per wave");
    if constexpr (MASK) {
      static_assert(F::MPW == 1, "one dword piece of dropout bits per wave");
      const char *bm = Mg + (sbase + m0) * (K / 8);
      glds4o<F::XB>(bm, vo[F::PPW], lds_m0 + sidx * F::STAGE + wid * 256);
    }
    m0_restore(keep);
  };
  auto dma_step = [&](int s, int sidx) {
    const int64_t m0 = pcs_min64(lo + (int64_t)s * MS, hi - 1);
    const int lastr = (int)pcs_min64(hi - 1 - m0, MS - 1);
    if (lastr == MS - 1) {   // uniform: a full step
      dma_issue(sidx, m0, voff);
    } else {
      uint32_t vt[F::PPW + F::MPW];
#pragma unroll
      for (int i = 0; i < F::PPW; ++i) vt[i] = piece_off(i, lastr);
#pragma unroll
      for (int i = 0; i < F::MPW; ++i) vt[F::PPW + i] = mask_off(i, lastr);
      dma_issue(sidx, m0, vt);
    }
  };

  float gsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // GRAM: column sums of channels 8 tc ..
  // ---- in-place BN + ReLU (+ dropout) of a landed stage: each element once
  auto transform_pass = [&](int sidx, int p, int rem) {
    char *st = lds + sidx * F::STAGE;
    {
      const int r = trow + p * (THREADS / SPR);
      u32x4 *q = reinterpret_cast<u32x4 *>(st + r * ROWB + ((tc ^ fsw<K>(r)) << 4));
      float v[8];
      unpack_chunk(*q, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = relu(fmaf(v[e], ts[e], tt[e]));
      u32x4 out = pack_chunk(v);
      if constexpr (MASK) {
        const uint32_t byte = (uint8_t)st[F::XB + r * (K / 8) + tc];
        const u32x4 m = *reinterpret_cast<const u32x4 *>(lds + F::OFF_LUT + byte * 16);
        out = mk_u32x4(out[0] & m[0], out[1] & m[1], out[2] & m[2], out[3] & m[3]);
      }
      if constexpr (GRAM) {   // rows past the slice (clamped copies of its last row) out of the Gram
        if (r >= rem) out = mk_u32x4(0, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gsum[2 * e] += bf2f(out[e] & 0xffffu);
          gsum[2 * e + 1] += bf2f(out[e] >> 16);
        }
      }
      *q = out;
    }
  };
  auto step_rem = [&](int s) { return (int)pcs_min64(hi - (lo + (int64_t)s * MS), MS); };
  auto transform = [&](int sidx, int rem) {
#pragma unroll
    for (int p = 0; p < F::TPASS; ++p) transform_pass(sidx, p, rem);
  };

  // ---- output through one buffer descriptor for the slice's rows (columns n0 .. of the block):
  // rows past the slice fall outside its range and are dropped by the hardware, so every wave
  // issues the same stores each step; the prologue's placeholder stores lie wholly out of range
  constexpr int ESZ = F::ESZ;
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char *>(a.C) + ((sbase + lo) * NCOLS + n0) * ESZ, 0,
      (int)(uint32_t)((hi - lo - 1) * NCOLS * ESZ + NB * ESZ), 0x00020000);
  const int rbase = wr * F::RW;   // this wave's first row of a step
  // lane (l16, g) after the swaps: row l16 of a row tile, columns 16 (2 q + (g & 1)) + 8 (g >> 1)
  const uint32_t o_st = (uint32_t)((rbase + l16) * (NCOLS * 2) + (wc * F::WC + 16 * (g & 1) + 8 * (g >> 1)) * 2);
  // (nt measured faster for the staged 128-B row stores -- conv5 3.74 -> 3.65 ms, seg_conv1 2.02 ->
  // 1.98 -- and slower for the 16 x 64 B ones of seg_conv2 / seg_conv3, 3.06 -> 3.12 ms)
  auto store16 = [&](uint32_t vo, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, rs_out, (int)vo, 0, F::STG ? FS_CPOL : 0);
  };
  // STG 1: lane = row rbase + lane / 8 (+ 8 i), columns wc WC + 8 (lane % 8) .. + 8;
  // STG 2: lane = row wid (+ 8 i), columns 64 (lane / 8) + 8 (lane % 8) .. + 8
  // C8: lane = row rbase + lane / 4 (+ 16 i), columns wc WC + 16 (lane % 4) .. + 16
  uint32_t o_stg = C8 ? (uint32_t)((rbase + (lane >> 2)) * NCOLS + wc * F::WC + 16 * (lane & 3))
                 : F::STG == 2 ? (uint32_t)(wid * (NCOLS * 2) + (64 * (lane >> 3) + 8 * (lane & 7)) * 2)
                               : (uint32_t)((rbase + (lane >> 3)) * (NCOLS * 2) + (wc * F::WC + 8 * (lane & 7)) * 2);

  // B-fragment LDS offsets: row rbase + 16 rt + l16 (f(row) = f(l16) for both swizzles, as
  // rbase + 16 rt is a multiple of 16), logical slot 4 kk + g
  int xo[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) xo[kk] = (rbase + l16) * ROWB + (((4 * kk + g) ^ fsw<K>(l16)) << 4);

  // statistics of the stored values: FWD per-lane sums shifted by the lane's first value (merged
  // with Chan's formula at the end); BNRELU plain column sums
  float sh[CT][4], s1[CT][4], s2[CT][4];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) { sh[ct][r] = 0.f; s1[ct][r] = 0.f; s2[ct][r] = 0.f; }
  float nrow = 0.f;   // rows this lane has counted

  // ---- prologue: steps 0 .. NST-2 in flight (each followed by SPS placeholder stores, as every
  // loop step's DMA is followed by its stores), step 0 landed and transformed
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    dma_step(s, s);
    // (distinct out-of-range offsets: hipcc merges identical stores, which would break the count)
#pragma unroll
    for (int q = 0; q < F::SPS; ++q) store16(0xFFF00000u + (uint32_t)(s * F::SPS + q) * 4096u, mk_u32x4(0, 0, 0, 0));
  }
  // step 0 landed: newer are the SPS stores after it and NST-2 (DMA, stores) groups
  wait_vm<F::SPS + (NST - 2) * (F::LPS + F::SPS)>();
  barrier_lds();
  transform(0, step_rem(0));
  barrier_lds();

  // GRAM: fragment offsets (within a stage) of k-step ks, row quad h: lane 4 q + p of group g
  // reads row 32 ks + 8 g + 4 h + q, columns 16 blk + 4 p .. + 3 (8 B at logical slot
  // 2 blk + p / 2, half p % 2, of the permuted 128-B row)
  auto gfrag = [&](const char *st, int ks, int blk) __attribute__((always_inline)) {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int r0 = 32 * ks + 8 * g + q, r1 = r0 + 4;
    const int sl = 2 * blk + (p >> 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4 *)(st + r0 * ROWB + ((sl ^ fsw<K>(r0)) << 4) + 8 * (p & 1)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4 *)(st + r1 * ROWB + ((sl ^ fsw<K>(r1)) << 4) + 8 * (p & 1)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  const int gbi = wid >> 1, gbj = 2 * (wid & 1);
  f32x4 gacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};

  int sc = 0;
  uint32_t o_out = o_st;
  for (int t = 0; t < nsteps; ++t) {
    // DMA of step t + NST - 1 into the stage of step t - 1 (its MFMAs are behind the last
    // barrier of every wave)
    dma_step(t + NST - 1, sc == 0 ? NST - 1 : sc - 1);
    const char *st = lds + sc * F::STAGE;
    const int sn = sc + 1 == NST ? 0 : sc + 1;   // stage of step t+1
    const bool more = t + 1 < nsteps;
    if constexpr (F::ILV) {
      // step t+1 landed (newer: NST-2 (DMA, stores) groups), so its transform can run between
      // this step's MFMA groups
      wait_vm<(NST - 2) * (F::LPS + F::SPS)>();
      barrier_lds();
    }
    f32x4 acc[CT][RT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[ct][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      bf16x8 xf[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) xf[rt] = *reinterpret_cast<const bf16x8 *>(st + xo[kk] + rt * 16 * ROWB);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          acc[ct][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wfr[ct][kk]), xf[rt],
                                                               acc[ct][rt], 0, 0, 0);
        }
      if constexpr (F::ILV) {
        constexpr int PER = KS / F::TPASS;   // MFMA k-steps per transform pass
        if ((kk + 1) % PER == 0 && more) {
          __builtin_amdgcn_sched_barrier(0);
          transform_pass(sn, kk / PER, step_rem(t + 1));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if constexpr (GRAM) {
#pragma unroll
      for (int ks = 0; ks < MS / 32; ++ks) {
        const bf16x8 fa = gfrag(st, ks, gbi);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x8 fb = gfrag(st, ks, gbj + j);
          gacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, gacc[j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);   // (one pair of fragments live at a time)
        }
      }
    }
    // ---- epilogue of step t: lane holds y[row rbase + 16 rt + l16][col0 + 16 ct + 4 g + r]
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)t * MS), MS);
    const bool full = rem == MS;   // uniform
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const bool live = full || rbase + 16 * rt + l16 < rem;
      const float livef = live ? 1.f : 0.f;   // BNRELU: the column sums add d * livef by v_fma
                                              // (exact: d or +0), no per-element select
      uint32_t pk[CT][2];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (EPI == PCS_EPI_BNRELU) v[r] = relu(fmaf(acc[ct][rt][r], es[ct][r], eb[ct][r]));
          else v[r] = acc[ct][rt][r] + eb[ct][r];
        }
        float d[4];   // the stored values
        if constexpr (C8) {
          pk[ct][0] = pack4fp8(v[0], v[1], v[2], v[3]);
          pk[ct][1] = 0u;
          const f32x2 d0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)pk[ct][0], false);
          const f32x2 d1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)pk[ct][0], true);
          d[0] = d0[0]; d[1] = d0[1]; d[2] = d1[0]; d[3] = d1[1];
        } else {
          pk[ct][0] = pack2bf(v[0], v[1]);
          pk[ct][1] = pack2bf(v[2], v[3]);
          d[0] = bf2f(pk[ct][0] & 0xffffu); d[1] = bf2f(pk[ct][0] >> 16);
          d[2] = bf2f(pk[ct][1] & 0xffffu); d[3] = bf2f(pk[ct][1] >> 16);
        }
        if constexpr (EPI == PCS_EPI_BNRELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) s1[ct][r] = fmaf(d[r], livef, s1[ct][r]);
        } else {
          if (t == 0 && rt == 0) {   // uniform: the lane's first value shifts its sums
#pragma unroll
            for (int r = 0; r < 4; ++r) sh[ct][r] = d[r];
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dd = live ? d[r] - sh[ct][r] : 0.f;
            s1[ct][r] += dd;
            s2[ct][r] = fmaf(dd, dd, s2[ct][r]);
          }
        }
      }
      nrow += livef;
      if constexpr (F::STG) {
        // 8-B granule 4 ct + g of the wave's row 16 rt + l16, at granule (4 ct + g) ^ (row & 15):
        // the 16 rows a lane group writes at one granule hit 16 distinct granules of the bank row
        if constexpr (C8) {   // 4-B granules of 64-B rows, the same (row & 15) permutation
          char *sw = lds + F::OFF_STG + wid * (F::RW * 64) + (16 * rt + l16) * 64;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) *reinterpret_cast<uint32_t *>(sw + (((4 * ct + g) ^ l16) << 2)) = pk[ct][0];
          continue;
        }
        char *sw = F::STG == 2 ? lds + F::OFF_STG + (16 * rt + l16) * (NB * 2) + wc * 128
                               : lds + F::OFF_STG + wid * (F::RW * 128) + (16 * rt + l16) * 128;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          *reinterpret_cast<uint2 *>(sw + (((4 * ct + g) ^ l16) << 3)) = make_uint2(pk[ct][0], pk[ct][1]);
        continue;
      }
#pragma unroll
      for (int q = 0; q < CT / 2; ++q) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto sw = __builtin_amdgcn_permlane16_swap(pk[2 * q][h], pk[2 * q + 1][h], false, false);
          pk[2 * q][h] = sw[0];
          pk[2 * q + 1][h] = sw[1];
        }
        store16(o_out + (uint32_t)(rt * 16 * NCOLS * 2 + q * 64), mk_u32x4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0],
                                                                         pk[2 * q + 1][1]));
      }
    }
    if constexpr (C8) {
      // rows back: lane = row 16 i + lane / 4, logical granules 4c .. 4c+3 (c = lane % 4), granule
      // G of a row at physical granule G ^ (row & 15): four 4-B reads at lane-constant offsets
      // (row & 15 = lane / 4 for every i), no per-lane selects
      const int c = lane & 3;
#pragma unroll
      for (int i = 0; i < F::RW / 16; ++i) {
        const int row = 16 * i + (lane >> 2);
        const char *rp = lds + F::OFF_STG + wid * (F::RW * 64) + row * 64;
        u32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = *reinterpret_cast<const uint32_t *>(rp + (((4 * c + e) ^ (row & 15)) << 2));
        store16(o_stg + (uint32_t)(i * 16 * NCOLS), w);
      }
      o_stg += MS * NCOLS;
    } else if constexpr (F::STG == 1) {
      // rows back from the wave's tile: lane = row 8 i + lane / 8, logical 8-B granules 2c, 2c+1
      // (c = lane % 8) at physical granules G ^ (row & 15): two 8-B reads at lane offsets that
      // depend on i only through its parity, no per-lane selects
      const uint32_t gl = (uint32_t)((2 * (lane & 7)) ^ (lane >> 3)) << 3;   // granule 2c, even i
#pragma unroll
      for (int i = 0; i < F::RW / 8; ++i) {
        const int row = 8 * i + (lane >> 3);
        const char *rp = lds + F::OFF_STG + wid * (F::RW * 128) + row * 128;
        const uint32_t go = (i & 1) ? gl ^ 64u : gl;   // row & 15 = lane / 8 + 8 (i & 1)
        const uint2 lo8 = *reinterpret_cast<const uint2 *>(rp + go);
        const uint2 hi8 = *reinterpret_cast<const uint2 *>(rp + (go ^ 8u));
        store16(o_stg + (uint32_t)(i * 8 * NCOLS * 2), mk_u32x4(lo8.x, lo8.y, hi8.x, hi8.y));
      }
      o_stg += MS * NCOLS * 2;
    }
    o_out += MS * NCOLS * 2;
    // step t+1 landed: newer are NST-2 (DMA, stores) groups and (unless STG 2) this step's stores
    if constexpr (!F::ILV) {
      wait_vm<F::WAIT_N>();
      barrier_lds();
    }
    if constexpr (F::STG == 2) {
      // whole rows of the step's tile: wave w stores rows w + 8 i, lane = 16-B chunk lane % 8 of
      // the 128-B column block lane / 8 (granule swizzle as written, halves swapped on odd rows)
      const int c = lane & 7, b = lane >> 3;
#pragma unroll
      for (int i = 0; i < MS / 8; ++i) {
        const int row = wid + 8 * i;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(lds + F::OFF_STG + row * (NB * 2) + b * 128 +
                                                         ((c ^ ((row >> 1) & 7)) << 4));
        const u32x4 w = (row & 1) ? mk_u32x4(v[2], v[3], v[0], v[1]) : v;
        store16(o_stg + (uint32_t)(i * 8 * NCOLS * 2), w);
      }
      o_stg += MS * NCOLS * 2;
    }
    if constexpr (!F::ILV) {
      if (more) transform(sn, step_rem(t + 1));
    }
    barrier_lds();
    sc = sc + 1 == NST ? 0 : sc + 1;
  }
  wait_vm<0>();   // the clamped DMAs past the end

  // ---- chunk end: merge the lanes of each column (and the wave rows) and write the partials
  float4 *red = reinterpret_cast<float4 *>(lds + F::OFF_RED);
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (EPI == PCS_EPI_BNRELU) {
        float s = s1[ct][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o);
        if (l16 == 0) red[wr * NB + wc * F::WC + 16 * ct + 4 * g + r] = make_float4(s, 0.f, 0.f, 0.f);
      } else {
        float n = nrow, mean = 0.f, m2 = 0.f;
        if (n > 0.f) {
          const float d1 = s1[ct][r] / n;
          mean = sh[ct][r] + d1;
          m2 = relu(s2[ct][r] - s1[ct][r] * d1);
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const float nb = __shfl_xor(n, o), mb = __shfl_xor(mean, o), qb = __shfl_xor(m2, o);
          chan_merge(n, mean, m2, nb, mb, qb);
        }
        if (l16 == 0) red[wr * NB + wc * F::WC + 16 * ct + 4 * g + r] = make_float4(n, mean, m2, 0.f);
      }
    }
  __syncthreads();
  if (a.stats) {
    for (int c = tid; c < NB; c += THREADS) {
      float4 p = red[c];
#pragma unroll
      for (int w = 1; w < F::WRN; ++w) {
        const float4 q = red[w * NB + c];
        if constexpr (EPI == PCS_EPI_BNRELU) p.x += q.x;
        else chan_merge(p.x, p.y, p.z, q.x, q.y, q.z);
      }
      const int64_t o = (int64_t)chunk * NCOLS + n0 + c;
      *reinterpret_cast<float2 *>(a.stats + o * 2) =
          EPI == PCS_EPI_BNRELU ? make_float2(p.x, 0.f) : make_float2(p.y, p.z);
    }
  }
  if constexpr (GRAM) {   // the chunk's [64 x 64 | 64] record: G[16 bi + 4 g + r][16 bj + l16]
    float *gr = a.gram + (int64_t)chunk * (K * K + K);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) gr[(16 * gbi + 4 * g + r) * K + 16 * (gbj + j) + l16] = gacc[j][r];
    // column sums: the 8 lanes of a wave that share tc (lane % 8), then the 8 waves via LDS
    // (the statistics merge above is done with the red area)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) gsum[e] += __shfl_xor(gsum[e], o);
    float *gs = reinterpret_cast<float *>(lds + F::OFF_RED);
    __syncthreads();
    if (lane < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) gs[wid * 64 + 8 * lane + e] = gsum[e];
    }
    __syncthreads();
    if (tid < K) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += gs[w * 64 + tid];
      gr[K * K + tid] = v;
    }
  }
}

template <int K, int NC> struct FsShape {
  static bool is(const pcs_gemm_args &a) { return a.K == K && a.Ncols == NC; }
};

}  // namespace

// Class (geometry, shapes only) and applicability (operands) of the streaming forward kernel.
// bf16, PRO_BNRELU; EPI_FWD on (K, Ncols) = (64, 512) seg_conv1, (512, 256) seg_conv2, (256, 128)
// seg_conv3, (64, 128) conv4, (64, 64) conv2 / conv3; EPI_BNRELU with a bf16 store on (128, 1024) conv5.
template <int K, int NC> int fs_nb(int *target) {
  if (target) *target = FsCfg<K, NC>::TARGET;
  return FsCfg<K, NC>::NB;
}
int pcs_fwd_stream_nb(const pcs_gemm_args &a, int *target) {
  if (a.dtype != PCS_BF16 || (a.flags & (PCS_FLAG_GENERIC | PCS_FLAG_AW_FP8)) || a.prologue != PCS_PRO_BNRELU)
    return 0;
  if (a.epilogue == PCS_EPI_FWD) {
    if (FsShape<64, 512>::is(a)) return fs_nb<64, 512>(target);
    if (FsShape<512, 256>::is(a)) return fs_nb<512, 256>(target);
    if (FsShape<256, 128>::is(a)) return fs_nb<256, 128>(target);
    if (FsShape<64, 128>::is(a)) return fs_nb<64, 128>(target);
    if (FsShape<64, 64>::is(a)) return fs_nb<64, 64>(target);
  } else if (a.epilogue == PCS_EPI_BNRELU) {
    if (FsShape<128, 1024>::is(a)) return fs_nb<128, 1024>(target);
  }
  return 0;
}

bool pcs_fwd_stream_applicable(const pcs_gemm_args &a) {
  if (!pcs_fwd_stream_nb(a, nullptr) || !a.C || !a.pa || !a.pb || a.pool) return false;
  if ((a.flags & PCS_FLAG_C_FP8) && a.epilogue != PCS_EPI_BNRELU) return false;
  if (a.scene_rows * a.num_scenes >= ((int64_t)1 << 31)) return false;
  // 32-bit store ranges / row offsets: a chunk of the widest rows must stay below 2 GB
  const int64_t rpc = a.chunks_per_scene > 0 ? (a.scene_rows + a.chunks_per_scene - 1) / a.chunks_per_scene
                                             : a.scene_rows;
  if (rpc * (int64_t)(a.K > a.Ncols ? a.K : a.Ncols) * 2 >= ((int64_t)1 << 31)) return false;
  if (a.epilogue == PCS_EPI_BNRELU) return a.es && a.et && !a.a_mask && !a.scene_bias;
  // dropout bits only where the layer has them (seg_conv2 / seg_conv3 inputs)
  if (a.a_mask && !(FsShape<512, 256>::is(a) || FsShape<256, 128>::is(a))) return false;
  if (a.scene_bias && !FsShape<64, 512>::is(a)) return false;
  return true;
}

int pcs_fwd_stream_launch(const pcs_gemm_args &a, int64_t rows_per_chunk, hipStream_t s) {
  const int nb_cols = pcs_fwd_stream_nb(a, nullptr);
  const int nb = (int)(a.num_scenes * a.chunks_per_scene) * (a.Ncols / nb_cols);
#define PCS_FS(K, NC, EPI, MK, SB) \
  hipLaunchKernelGGL((fwd_stream_kernel<K, NC, EPI, MK, SB>), dim3(nb), dim3(THREADS), 0, s, a, rows_per_chunk)
  const bool mk = a.a_mask != nullptr;
  if (a.epilogue == PCS_EPI_BNRELU) {
    if (a.flags & PCS_FLAG_C_FP8)
      hipLaunchKernelGGL((fwd_stream_kernel<128, 1024, PCS_EPI_BNRELU, false, false, true>), dim3(nb), dim3(THREADS), 0,
                         s, a, rows_per_chunk);
    else
      PCS_FS(128, 1024, PCS_EPI_BNRELU, false, false);
  } else if (FsShape<64, 512>::is(a)) {
    if (a.scene_bias) PCS_FS(64, 512, PCS_EPI_FWD, false, true); else PCS_FS(64, 512, PCS_EPI_FWD, false, false);
  } else if (FsShape<512, 256>::is(a)) {
    if (mk) PCS_FS(512, 256, PCS_EPI_FWD, true, false); else PCS_FS(512, 256, PCS_EPI_FWD, false, false);
  } else if (FsShape<256, 128>::is(a)) {
    if (mk) PCS_FS(256, 128, PCS_EPI_FWD, true, false); else PCS_FS(256, 128, PCS_EPI_FWD, false, false);
  } else if (FsShape<64, 128>::is(a)) {
    PCS_FS(64, 128, PCS_EPI_FWD, false, false);
  } else if (FsShape<64, 64>::is(a)) {
    if (a.gram)
      hipLaunchKernelGGL((fwd_stream_kernel<64, 64, PCS_EPI_FWD, false, false, false, true>), dim3(nb), dim3(THREADS), 0,
                         s, a, rows_per_chunk);
    else
      PCS_FS(64, 64, PCS_EPI_FWD, false, false);
  } else {
    return pcs_set_einval("pcs_gemm", "streaming forward: unsupported shape");
  }
#undef PCS_FS
  PCS_CHECK_LAUNCH();
  return 0;
}

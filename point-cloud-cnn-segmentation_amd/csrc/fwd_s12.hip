// seg_conv1's local half and seg_conv2 in one streaming pass (the training step's forward,
// P:117-125), so that seg_conv1's 512-wide output is written once and never read back here:
//
//   a2  = relu(y2 * s2 + t2)                       (bn2 + ReLU of conv2's stored output, bf16)
//   Y1  = a2 W1^T + sbias[b]                       stored bf16: seg_conv1's pre-BN output, kept
//                                                  for the backward (fused_seg4.hip reads it)
//   x   = relu(Y1 * s1 + t1) * keep * ks           (bn_seg1 + ReLU + dropout, P:123-124)
//   Y2  = x W2^T                                   stored bf16 with per-chunk (mean, M2) of the
//                                                  stored values (bn_seg2's statistics)
//
// bn_seg1's batch statistics are needed before Y1 exists; they come from the Gram of a2
// (pcs_bn_stats_gram_sbias below), as bn5's come from the Gram of a4.  Against the two streaming
// passes this replaces (fwd_stream.hip <64, 512> and <512, 256>) the 8.6 GB re-read of Y1 at
// cfg2 and the 512-wide statistics epilogue go away.
//
// A workgroup (8 waves) owns a scene-aligned row slice.  Per 32-row step:
// * LDS-DMA (dword pieces, counted waits) brings y2 (4 KB) and the step's keep bits (2 KB)
//   through a 3-stage ring (NST); bn2 + ReLU is applied once per element, in place;
// * stage 1: wave w computes Y1 columns 64 w .. 64 w + 63 (W1 rows from LDS, 16 MFMAs), its
//   epilogue adds the scene bias, rounds, stores Y1 (16-B stores after v_permlane16_swap) and
//   writes x = bn_seg1 / ReLU / dropout of the ROUNDED values (the backward recomputes x from the
//   stored Y1) into a [32 x 512] LDS tile;
// * stage 2: wave w computes Y2 columns 32 w .. 32 w + 31 over K = 512 (its W2 rows in registers,
//   64 MFMAs), then rounding, statistics and stores as in fwd_stream.hip.
// The 16-B slots of an LDS row hold the logical slots XOR-permuted by the row (y2 / a2 and W1
// rows of 128 B: (row >> 1) & 7; x rows of 1 KB: row & 15), so the fragment reads are
// bank-conflict free.
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int MS = 32, NST = 3;
constexpr int K1 = 64, N1 = 512, K2 = 512, N2 = 256;
constexpr int ROW1 = K1 * 2;                  // 128-B y2 / a2 / W1 rows
constexpr int XB1 = MS * ROW1;                // 4 KB of y2 per stage
constexpr int MROW = K2 / 8;                  // 64 B of keep bits per row
constexpr int MKB = MS * MROW;                // 2 KB per stage
constexpr int STAGE = XB1 + MKB;
constexpr int XROW = K2 * 2;                  // 1-KB x rows
constexpr int OFF_X = NST * STAGE;            // x tiles [2][MS][1 KB] (steps of either parity)
constexpr int XT = MS * XROW;
constexpr int OFF_W1 = OFF_X + 2 * XT;        // W1 [512][128 B]
constexpr int OFF_SB = OFF_W1 + N1 * ROW1;    // scene bias [512]
constexpr int OFF_S1 = OFF_SB + N1 * 4;       // bn_seg1 scale * ks [512]
constexpr int OFF_T1 = OFF_S1 + N1 * 4;       // bn_seg1 shift * ks [512]
constexpr int OFF_S2 = OFF_T1 + N1 * 4;       // bn2 scale [64]
constexpr int OFF_T2 = OFF_S2 + K1 * 4;       // bn2 shift [64]
constexpr int OFF_LUT = OFF_T2 + K1 * 4;      // keep byte -> AND masks of 8 packed bf16 [256][4]
constexpr int OFF_SH = OFF_LUT + 256 * 16;    // Y2 statistics: per-column shift (row 0 of the chunk),
constexpr int OFF_SS = OFF_SH + N2 * 4;       //   sum and sum of squares of the shifted values [256]
constexpr int OFF_SQ = OFF_SS + N2 * 4;
constexpr int BYTES = OFF_SQ + N2 * 4;
static_assert(BYTES <= 160 * 1024, "LDS budget");
constexpr int KS2 = K2 / 32;                  // stage-2 k-steps
// Ring of three stages: in iteration t, step t + 1's stage feeds stage 1, step t + 2's (DMA'd in
// iteration t - 1) gets bn2 + ReLU for the next iteration, and step t's (consumed in iteration
// t - 1) takes the DMA of step t + 3; so one barrier per step.  Vector-memory operations per wave
// per iteration, in issue order: 3 DMA pieces, 4 Y1 stores (step t + 1), 2 Y2 stores (step t);
// the wait at the top of iteration t retires the DMA of step t + 2, issued one iteration
// earlier: newer are that iteration's 6 stores
static_assert(NST == 3, "the ring's roles assume three stages");
constexpr int VM_WAIT = 6;

typedef __attribute__((address_space(3))) void lds_void_t;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
template <int N> PCS_DEV float row_ror(float v) {   // rotate within the 16 lanes of a DPP row
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x120 + N, 0xf, 0xf, true));
}
PCS_DEV int f64s(int r) { return (r >> 1) & 7; }   // slot permutation of 128-B rows

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

template <bool MASK>
__global__ __launch_bounds__(THREADS) void fwd_s12_kernel(pcs_seg12_args a, int64_t rows_per_chunk) {
  __shared__ __attribute__((aligned(16))) char lds[BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int chunk = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  const int cps = a.chunks_per_scene;
  const int scene = __builtin_amdgcn_readfirstlane(chunk / cps), cis = __builtin_amdgcn_readfirstlane(chunk % cps);
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)cis * rows_per_chunk;
  const int64_t hi = pcs_min64(lo + rows_per_chunk, N);
  const int64_t sbase = (int64_t)scene * N;
  const int nsteps = (int)((hi - lo + MS - 1) / MS);   // >= 1 (no empty chunks)
  const char *Yg = reinterpret_cast<const char *>(a.y2);
  const char *Mg = MASK ? reinterpret_cast<const char *>(a.keep1) : nullptr;
  const int l16 = lane & 15, g = lane >> 4;

  // ---- per-workgroup constants: W1 rows (permuted slots) and the coefficient vectors -> LDS;
  // this wave's W2 rows (A operand: lane = output channel 32 w + 16 ct + l16, k chunk 4 kk + g)
  {
    const bf16_t *W1g = reinterpret_cast<const bf16_t *>(a.W1);
    for (int i = tid; i < N1 * 8; i += THREADS) {
      const int r = i >> 3, ls = i & 7;
      *reinterpret_cast<u32x4 *>(lds + OFF_W1 + r * ROW1 + ((ls ^ f64s(r)) << 4)) =
          *reinterpret_cast<const u32x4 *>(W1g + (int64_t)r * K1 + ls * 8);
    }
    const float ks = MASK ? a.keep_scale : 1.f;   // relu(v s + t) ks = relu(v (s ks) + t ks), ks > 0
    float *cf = reinterpret_cast<float *>(lds + OFF_SB);
    for (int c = tid; c < N1; c += THREADS) {
      cf[c] = a.sbias[(int64_t)scene * N1 + c];
      cf[N1 + c] = a.s1[c] * ks;
      cf[2 * N1 + c] = a.t1[c] * ks;
    }
    if (tid < K1) {
      reinterpret_cast<float *>(lds + OFF_S2)[tid] = a.s2[tid];
      reinterpret_cast<float *>(lds + OFF_T2)[tid] = a.t2[tid];
    }
    if (tid < N2) {
      reinterpret_cast<float *>(lds + OFF_SS)[tid] = 0.f;
      reinterpret_cast<float *>(lds + OFF_SQ)[tid] = 0.f;
    }
    if (tid < 256) {   // keep byte -> the AND masks of 8 packed bf16 values (bit i = column i)
      uint32_t *lut = reinterpret_cast<uint32_t *>(lds + OFF_LUT) + tid * 4;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        lut[d] = (((tid >> (2 * d)) & 1) ? 0x0000FFFFu : 0u) | (((tid >> (2 * d + 1)) & 1) ? 0xFFFF0000u : 0u);
    }
  }
  const bf16_t *W2g = reinterpret_cast<const bf16_t *>(a.W2);
  u32x4 wfr[2][KS2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int kk = 0; kk < KS2; ++kk)
      wfr[ct][kk] = *reinterpret_cast<const u32x4 *>(W2g + (int64_t)(32 * w + 16 * ct + l16) * K2 + (4 * kk + g) * 8);
  // every ordinary load retires here, before the first DMA (hipcc's own waits do not count the
  // inline-asm DMAs; one placed later would drain them)
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int kk = 0; kk < KS2; ++kk) asm volatile("" ::"v"(wfr[ct][kk]));
  __syncthreads();

  // ---- DMA of step s into stage sidx: dword pieces of 256 B.  y2: pieces p = w, w + 8 (rows 2p,
  // 2p + 1; lane -> row 2p + lane / 32, physical slot (lane % 32) / 4, dword lane % 4, holding
  // logical slot ps ^ f(row) of the source row); keep bits: piece w (rows 4 w .. 4 w + 3, 64 B
  // each), dword d of row r holding logical dword d ^ (r & 15), so the 16 rows the epilogue reads
  // at one logical byte fall in 16 banks instead of 2 (8-way).  Rows past the slice clamp to its
  // last row.
  auto y_off = [&](int p, int lastr) -> uint32_t {
    const int r = 2 * p + (lane >> 5), ps = (lane & 31) >> 2;
    return (uint32_t)(min(r, lastr) * ROW1 + ((ps ^ f64s(r)) << 4) + 4 * (lane & 3));
  };
  auto m_off = [&](int lastr) -> uint32_t {
    const int r = 4 * w + (lane >> 4);
    return (uint32_t)(min(r, lastr) * MROW + 4 * ((lane & 15) ^ (r & 15)));
  };
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  auto dma_step = [&](int s, int sidx) {
    const int64_t m0 = pcs_min64(lo + (int64_t)s * MS, hi - 1);
    const int lastr = (int)pcs_min64(hi - 1 - m0, MS - 1);
    const char *by = Yg + (sbase + m0) * ROW1;
    const uint32_t mb = lds_m0 + sidx * STAGE;
    const uint32_t keep = m0_save();
    glds4o<0>(by, y_off(w, lastr), mb + w * 256);
    glds4o<0>(by, y_off(w + 8, lastr), mb + (w + 8) * 256);
    if constexpr (MASK) glds4o<XB1>(Mg + (sbase + m0) * MROW, m_off(lastr), mb + w * 256);
    else glds4o<XB1>(by, y_off(w, lastr), mb + w * 256);   // (no bits: a placeholder of the count)
    m0_restore(keep);
  };

  // ---- bn2 + ReLU in place, each element once (thread: row tid / 16, logical slot (tid / 2) % 8,
  // its half tid % 2: 4 elements)
  auto transform = [&](int sidx) {
    const int r = tid >> 4, ls = (tid >> 1) & 7, hf = tid & 1;
    uint2 *q = reinterpret_cast<uint2 *>(lds + sidx * STAGE + r * ROW1 + ((ls ^ f64s(r)) << 4) + 8 * hf);
    const f32x4 s2 = *reinterpret_cast<const f32x4 *>(lds + OFF_S2 + (8 * ls + 4 * hf) * 4);
    const f32x4 t2 = *reinterpret_cast<const f32x4 *>(lds + OFF_T2 + (8 * ls + 4 * hf) * 4);
    const uint2 u = *q;
    const f32x2 v01 = __builtin_elementwise_fma(f32x2{bf2f(u.x & 0xffffu), bf2f(u.x >> 16)}, f32x2{s2[0], s2[1]},
                                                f32x2{t2[0], t2[1]});
    const f32x2 v23 = __builtin_elementwise_fma(f32x2{bf2f(u.y & 0xffffu), bf2f(u.y >> 16)}, f32x2{s2[2], s2[3]},
                                                f32x2{t2[2], t2[3]});
    *q = make_uint2(pack2bf(relu(v01.x), relu(v01.y)), pack2bf(relu(v23.x), relu(v23.y)));
  };

  // ---- outputs through buffer descriptors over the slice's rows (stores past them are dropped)
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char *>(a.Y1) + (sbase + lo) * (N1 * 2), 0, (int)(uint32_t)((hi - lo) * (N1 * 2)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char *>(a.Y2) + (sbase + lo) * (N2 * 2), 0, (int)(uint32_t)((hi - lo) * (N2 * 2)), 0x00020000);
  // after the swaps lane (l16, g) holds 8 consecutive columns 16 (g & 1) + 8 (g >> 1) of a 32-column pair
  const uint32_t o1 = (uint32_t)(l16 * (N1 * 2) + (64 * w + 16 * (g & 1) + 8 * (g >> 1)) * 2);
  const uint32_t o2 = (uint32_t)(l16 * (N2 * 2) + (32 * w + 16 * (g & 1) + 8 * (g >> 1)) * 2);
  const int fa = f64s(l16);   // (16 rt + l16) >> 1 & 7 and (64 w + 16 ct + l16) >> 1 & 7 alike
  // keep byte 8 w + 2 ct + (g >> 1) of row 16 rt + l16 (permuted dwords, see the DMA): at
  // 1024 rt + 2 (ct & 1) + (lkb ^ 4 (2 w + (ct >> 1))), one v_xor with a uniform per read
  const int lkb = 68 * l16 + (g >> 1);

  // ---- stage 1 of a step, one 16-column tile ct at a time: Y1[row 16 rt + l16][64 w + 16 ct + 4 g + r]
  auto stage1 = [&](const char *st, int ct, f32x4 (&acc1)[2]) __attribute__((always_inline)) {
    acc1[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc1[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 af = *reinterpret_cast<const bf16x8 *>(lds + OFF_W1 + (64 * w + 16 * ct + l16) * ROW1 +
                                                          (((4 * kk + g) ^ fa) << 4));
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const bf16x8 bf = *reinterpret_cast<const bf16x8 *>(st + (16 * rt + l16) * ROW1 + (((4 * kk + g) ^ fa) << 4));
        acc1[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc1[rt], 0, 0, 0);
      }
    }
  };
  // its epilogue: scene bias, round into pk (packed bf16 of Y1), x of the ROUNDED values (the
  // backward recomputes x from the stored Y1) into x tile xb: relu(d s1 ks + t1 ks) as packed
  // bf16, ANDed with the keep masks
  auto epi1 = [&](const char *st, char *xb, int ct, const f32x4 (&acc1)[2], uint32_t (&pk)[2][2]) __attribute__((always_inline)) {
    const int c0 = 64 * w + 16 * ct + 4 * g;
    const f32x4 sb = *reinterpret_cast<const f32x4 *>(lds + OFF_SB + c0 * 4);
    const f32x4 sc1 = *reinterpret_cast<const f32x4 *>(lds + OFF_S1 + c0 * 4);
    const f32x4 tc1 = *reinterpret_cast<const f32x4 *>(lds + OFF_T1 + c0 * 4);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int R = 16 * rt + l16;
      // (column pairs in packed fp32: v_pk_add_f32 / v_pk_fma_f32, the same roundings)
      const f32x2 y01 = f32x2{acc1[rt][0], acc1[rt][1]} + f32x2{sb[0], sb[1]};
      const f32x2 y23 = f32x2{acc1[rt][2], acc1[rt][3]} + f32x2{sb[2], sb[3]};
      pk[rt][0] = pack2bf(y01.x, y01.y);
      pk[rt][1] = pack2bf(y23.x, y23.y);
      const f32x2 z01 = __builtin_elementwise_fma(f32x2{bf2f(pk[rt][0] & 0xffffu), bf2f(pk[rt][0] >> 16)},
                                                  f32x2{sc1[0], sc1[1]}, f32x2{tc1[0], tc1[1]});
      const f32x2 z23 = __builtin_elementwise_fma(f32x2{bf2f(pk[rt][1] & 0xffffu), bf2f(pk[rt][1] >> 16)},
                                                  f32x2{sc1[2], sc1[3]}, f32x2{tc1[2], tc1[3]});
      uint2 xo = make_uint2(pack2bf(relu(z01.x), relu(z01.y)), pack2bf(relu(z23.x), relu(z23.y)));
      if constexpr (MASK) {   // columns c0 .. c0 + 3: keep byte c0 / 8 of row R, bits 4 (g % 2) ..
        const uint32_t byte = *reinterpret_cast<const uint8_t *>(st + XB1 + 1024 * rt + 2 * (ct & 1) +
                                                                 (lkb ^ (4 * (2 * w + (ct >> 1)))));
        const uint2 m = *reinterpret_cast<const uint2 *>(lds + OFF_LUT + byte * 16 + 8 * (g & 1));
        xo.x &= m.x;
        xo.y &= m.y;
      }
      *reinterpret_cast<uint2 *>(xb + R * XROW + (((8 * w + 2 * ct + (g >> 1)) ^ l16) << 4) + 8 * (g & 1)) = xo;
    }
  };
  // the 32 columns of tiles 2 hq, 2 hq + 1 of Y1: one 16-B store per row tile after the swap
  auto store1 = [&](uint32_t (&pa)[2][2], uint32_t (&pb)[2][2], int hq, uint32_t out) __attribute__((always_inline)) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto sw = __builtin_amdgcn_permlane16_swap(pa[rt][h], pb[rt][h], false, false);
        pa[rt][h] = sw[0];
        pb[rt][h] = sw[1];
      }
      __builtin_amdgcn_raw_buffer_store_b128(mk_u32x4(pa[rt][0], pa[rt][1], pb[rt][0], pb[rt][1]), rs1,
                                             (int)(out + (uint32_t)(rt * 16 * N1 * 2 + hq * 64)), 0, 0);
    }
  };
  // stage 2, k-steps k0 .. k0 + n - 1: Y2[row 16 rt + l16][32 w + 16 ct + 4 g + r]
  auto stage2 = [&](const char *xb, int k0, int n, f32x4 (&acc2)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int kq = 0; kq < n; ++kq) {
      const int kk = k0 + kq;
      bf16x8 xf[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        xf[rt] = *reinterpret_cast<const bf16x8 *>(xb + (16 * rt + l16) * XROW + (((4 * kk + g) ^ l16) << 4));
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          acc2[ct][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wfr[ct][kk]), xf[rt],
                                                                acc2[ct][rt], 0, 0, 0);
    }
  };

  // ---- prologue: the DMAs of steps 0, 1, 2 (each followed by 6 stores, as in the loop:
  // placeholders at distinct out-of-range offsets -- hipcc merges identical stores -- except the
  // last group, which holds step 0's Y1 stores), steps 0 and 1 transformed, step 0 through stage
  // 1 into x tile 0
  auto pad_stores = [&](int s, int n1, int n2) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < n1)
        __builtin_amdgcn_raw_buffer_store_b128(mk_u32x4(0, 0, 0, 0), rs1, (int)(0xFFF00000u + (uint32_t)(s * 8 + q) * 4096u), 0, 0);
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (q < n2)
        __builtin_amdgcn_raw_buffer_store_b128(mk_u32x4(0, 0, 0, 0), rs2, (int)(0xFFF00000u + (uint32_t)(s * 8 + 4 + q) * 4096u), 0, 0);
  };
  dma_step(0, 0);
  pad_stores(0, 4, 2);
  dma_step(1, 1);
  pad_stores(1, 4, 2);
  wait_vm<6>();   // steps 0 and 1 landed
  barrier_lds();
  transform(0);
  transform(1);
  barrier_lds();
  dma_step(2, 2);
  {
    f32x4 acc1[2];
    uint32_t pa[2][2], pb[2][2];
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      stage1(lds, 2 * hq, acc1);
      epi1(lds, lds + OFF_X, 2 * hq, acc1, pa);
      stage1(lds, 2 * hq + 1, acc1);
      epi1(lds, lds + OFF_X, 2 * hq + 1, acc1, pb);
      store1(pa, pb, hq, o1);
    }
  }
  pad_stores(2, 0, 2);

  uint32_t out1 = o1 + MS * N1 * 2, out2 = o2;
  for (int t = 0; t < nsteps; ++t) {
    const int s1i = (t + 1) % NST;   // stage of step t + 1 (transformed in iteration t - 1)
    // step t + 2 landed; every wave is past iteration t - 1, so x tile t & 1 and step t + 1's
    // transform are complete and the stage of step t is free
    wait_vm<VM_WAIT>();
    barrier_lds();
    dma_step(t + 3, t % NST);
    transform((t + 2) % NST);
    const char *st1 = lds + s1i * STAGE;
    const char *xr = lds + OFF_X + (t & 1) * XT;
    char *xw = lds + OFF_X + ((t + 1) & 1) * XT;
    // stage 2 of step t interleaved with stage 1 (+ its epilogue) of step t + 1
    f32x4 acc2[2][2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) acc2[ct][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      f32x4 acc1[2];
      uint32_t pa[2][2], pb[2][2];
      stage2(xr, 0, 3, acc2);
      stage1(st1, 0, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 3, 3, acc2);
      epi1(st1, xw, 0, acc1, pa);
      stage1(st1, 1, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 6, 3, acc2);
      epi1(st1, xw, 1, acc1, pb);
      store1(pa, pb, 0, out1);
      stage1(st1, 2, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 9, 3, acc2);
      epi1(st1, xw, 2, acc1, pa);
      stage1(st1, 3, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 12, 4, acc2);
      epi1(st1, xw, 3, acc1, pb);
      store1(pa, pb, 1, out1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue 2 of step t: round, statistics of the stored values, store Y2.  Statistics:
    // per column the 32 rows' sum and sum of squares, shifted by the chunk's row-0 value, reduced
    // over the 16 lanes of a DPP row and accumulated in LDS by lane 0 of the row (each wave owns
    // its 32 columns)
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)t * MS), MS);
    uint32_t pk[2][2][2];   // [rt][ct][h]
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        pk[rt][ct][0] = pack2bf(acc2[ct][rt][0], acc2[ct][rt][1]);
        pk[rt][ct][1] = pack2bf(acc2[ct][rt][2], acc2[ct][rt][3]);
      }
    {
      float *shp = reinterpret_cast<float *>(lds + OFF_SH) + 32 * w + 4 * g;
      float *ssp = reinterpret_cast<float *>(lds + OFF_SS) + 32 * w + 4 * g;
      float *sqp = reinterpret_cast<float *>(lds + OFF_SQ) + 32 * w + 4 * g;
      // the shift: row 0 of the chunk (always live), from lane 0 of the row at step 0 (a shuffle:
      // the lanes of a wave do not see each other's LDS writes without a barrier in the language's
      // model, and hipcc forwards a lane's own store), from LDS after
      f32x4 shv[2];
      if (t == 0) {   // uniform
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            shv[ct][r] = __shfl(bf2f(r & 1 ? pk[0][ct][r >> 1] >> 16 : pk[0][ct][r >> 1] & 0xffffu), lane & 48);
        if (l16 == 0) {
#pragma unroll
          for (int ct = 0; ct < 2; ++ct) *reinterpret_cast<f32x4 *>(shp + 16 * ct) = shv[ct];
        }
      } else {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) shv[ct] = *reinterpret_cast<const f32x4 *>(shp + 16 * ct);
      }
      const bool live0 = l16 < rem, live1 = 16 + l16 < rem;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const f32x4 sh = shv[ct];
        f32x4 sv, qv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d0 = bf2f(r & 1 ? pk[0][ct][r >> 1] >> 16 : pk[0][ct][r >> 1] & 0xffffu);
          const float d1 = bf2f(r & 1 ? pk[1][ct][r >> 1] >> 16 : pk[1][ct][r >> 1] & 0xffffu);
          const float e0 = live0 ? d0 - sh[r] : 0.f, e1 = live1 ? d1 - sh[r] : 0.f;
          float sr = e0 + e1, qr = fmaf(e0, e0, e1 * e1);
          sr += row_ror<8>(sr);   // every lane of the row ends with the total
          qr += row_ror<8>(qr);
          sr += row_ror<4>(sr);
          qr += row_ror<4>(qr);
          sr += row_ror<2>(sr);
          qr += row_ror<2>(qr);
          sr += row_ror<1>(sr);
          qr += row_ror<1>(qr);
          sv[r] = sr;
          qv[r] = qr;
        }
        if (l16 == 0) {
          *reinterpret_cast<f32x4 *>(ssp + 16 * ct) += sv;
          *reinterpret_cast<f32x4 *>(sqp + 16 * ct) += qv;
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto sw = __builtin_amdgcn_permlane16_swap(pk[rt][0][h], pk[rt][1][h], false, false);
        pk[rt][0][h] = sw[0];
        pk[rt][1][h] = sw[1];
      }
      __builtin_amdgcn_raw_buffer_store_b128(mk_u32x4(pk[rt][0][0], pk[rt][0][1], pk[rt][1][0], pk[rt][1][1]), rs2,
                                             (int)(out2 + (uint32_t)(rt * 16 * N2 * 2)), 0, 0);
    }
    out1 += MS * N1 * 2;
    out2 += MS * N2 * 2;
  }
  wait_vm<0>();   // the clamped DMAs past the end

  // ---- chunk end: (mean, M2) of each column of the slice
  __syncthreads();
  if (a.stats && tid < N2) {
    const float n = (float)(hi - lo);
    const float S = reinterpret_cast<const float *>(lds + OFF_SS)[tid];
    const float Q = reinterpret_cast<const float *>(lds + OFF_SQ)[tid];
    const float d1 = S / n;
    *reinterpret_cast<float2 *>(a.stats + ((int64_t)chunk * N2 + tid) * 2) =
        make_float2(reinterpret_cast<const float *>(lds + OFF_SH)[tid] + d1, relu(Q - S * d1));
  }
}

// bn_seg1's batch statistics from the Gram of a2 (16 output channels per workgroup; each of the
// C / 16 workgroups rebuilds the 64 x 64 fp64 Cw, a few microseconds, below): the
// centred within-scene Gram Cw = G - sum_b S_b S_b^T / N (fp64, in LDS), then per channel
// M2w = w Cw w^T and the per-scene means S_b w / N + sbias[b]; written as per-scene partials
// (mean_b, M2w / B) whose Chan merge in pcs_bn_fwd_finalize adds the between-scene term
__global__ __launch_bounds__(256) void bn_stats_gram_sbias_kernel(const float *__restrict__ G, const float *__restrict__ Sb,
                                                                  int64_t B, int64_t N, const float *__restrict__ W,
                                                                  int64_t ldw, int Cin, int C,
                                                                  const float *__restrict__ sbias, float *__restrict__ stats) {
  // a workgroup: 16 channels x 16 threads; thread e of a channel takes rows p = e, e + 16, ..
  // of Cw w and of S_b . w, and the 16 partial sums meet by shuffles
  __shared__ double cw[64 * 64];
  __shared__ double wl[16][64];
  const int tid = threadIdx.x;
  for (int i = tid; i < Cin * Cin; i += 256) {
    const int p = i / Cin, q = i % Cin;
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += (double)Sb[b * Cin + p] * (double)Sb[b * Cin + q];
    cw[i] = (double)G[(int64_t)p * Cin + q] - s / (double)N;
  }
  const int cl = tid >> 4, e = tid & 15;
  const int c = blockIdx.x * 16 + cl;
  for (int q = e; q < 64; q += 16) wl[cl][q] = (c < C && q < Cin) ? (double)W[(int64_t)c * ldw + q] : 0.0;
  __syncthreads();
  double m2 = 0.0;
  for (int p = e; p < Cin; p += 16) {
    double u = 0.0;
    for (int q = 0; q < Cin; ++q) u += cw[p * Cin + q] * wl[cl][q];
    m2 += wl[cl][p] * u;
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) m2 += __shfl_xor(m2, o);
  if (m2 < 0.0) m2 = 0.0;
  for (int b = 0; b < B; ++b) {
    double sw = 0.0;
    for (int p = e; p < Cin; p += 16) sw += (double)Sb[b * Cin + p] * wl[cl][p];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sw += __shfl_xor(sw, o);
    if (e == 0 && c < C) {
      const double mean = sw / (double)N + (sbias ? (double)sbias[b * C + c] : 0.0);
      *reinterpret_cast<float2 *>(stats + ((int64_t)b * C + c) * 2) = make_float2((float)mean, (float)(m2 / (double)B));
    }
  }
}

}  // namespace

extern "C" int64_t pcs_fwd_seg12_geometry(pcs_seg12_args *a) {
  if (!a || a->num_scenes <= 0 || a->scene_rows <= 0) return pcs_set_einval("pcs_fwd_seg12_geometry", "empty geometry");
  pcs_gemm_args g{};
  g.num_scenes = a->num_scenes;
  g.scene_rows = a->scene_rows;
  g.chunks_per_scene = a->chunks_per_scene;
  const int64_t rpc = pcs_fill_geometry(&g, MS, 256, 1);   // one workgroup per CU
  a->chunks_per_scene = g.chunks_per_scene;
  return rpc;
}

extern "C" int pcs_fwd_seg12(const pcs_seg12_args *ap, pcs_stream_t stream) {
  if (!ap) return pcs_set_einval("pcs_fwd_seg12", "null args");
  pcs_seg12_args a = *ap;
  if (!a.y2 || !a.s2 || !a.t2 || !a.W1 || !a.sbias || !a.Y1 || !a.s1 || !a.t1 || !a.W2 || !a.Y2)
    return pcs_set_einval("pcs_fwd_seg12", "missing operand");
  if (a.num_scenes * a.scene_rows >= ((int64_t)1 << 31)) return pcs_set_einval("pcs_fwd_seg12", "M must be < 2^31 rows");
  const int32_t cps_in = a.chunks_per_scene;
  const int64_t rpc = pcs_fwd_seg12_geometry(&a);
  if (rpc < 0) return (int)rpc;
  if (cps_in > 0 && cps_in != a.chunks_per_scene) return pcs_set_einval("pcs_fwd_seg12", "chunks_per_scene mismatch");
  // 32-bit buffer ranges: a slice of Y1 rows below 2 GB
  if (rpc * N1 * 2 >= ((int64_t)1 << 31)) return pcs_set_einval("pcs_fwd_seg12", "row slice too large");
  const int nb = (int)(a.num_scenes * a.chunks_per_scene);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a.keep1) hipLaunchKernelGGL(fwd_s12_kernel<true>, dim3(nb), dim3(THREADS), 0, s, a, rpc);
  else hipLaunchKernelGGL(fwd_s12_kernel<false>, dim3(nb), dim3(THREADS), 0, s, a, rpc);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_bn_stats_gram_sbias(const float *G, const float *Sb, int64_t num_scenes, int64_t scene_rows,
                                       const float *W, int64_t ldw, int32_t Cin, int32_t C, const float *sbias,
                                       float *stats, pcs_stream_t stream) {
  if (!G || !Sb || !W || !stats || num_scenes <= 0 || scene_rows <= 0 || Cin <= 0 || Cin > 64 || C <= 0 || ldw < Cin)
    return pcs_set_einval("pcs_bn_stats_gram_sbias", "bad arguments (1 <= Cin <= 64, ldw >= Cin)");
  hipLaunchKernelGGL(bn_stats_gram_sbias_kernel, dim3((C + 15) / 16), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     G, Sb, num_scenes, scene_rows, W, ldw, Cin, C, sbias, stats);
  PCS_CHECK_LAUNCH();
  return 0;
}

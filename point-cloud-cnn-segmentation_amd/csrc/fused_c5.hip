// conv5's folded input gradient (autograd of P:110 at P:254) as one LDS-DMA stream:
//
//   g    = dz5 Ws^T + relu(bn4(y4)) H4^T + c5     (Ws = diag(alpha5) W5 as [128][1024], H4 =
//          W5^T diag(gamma5) W5 [128][128], c5 = W5^T beta5: pcs_bn_fold; the PCS_PRO_CAT call)
//   dA4  = relu'(bn4(y4)) * g                      (stored bf16; S1 = sum dA4, S2 = sum dA4 xhat4)
//
// The generic register-staged kernel ran this at 3.9-4.0 TB/s (5.4 ms at cfg2): 32-element
// k-steps, a barrier each, for a K of 1152.  Here:
// * a workgroup owns all 128 output columns of a scene-aligned row slice, so dz5 (17 GB at cfg2,
//   the whole cost) is read exactly once;
// * each of the 8 waves keeps its 16 columns of Ws^T and H4^T in registers for the whole slice
//   (36 x 16 B per lane), so only dz5 and y4 stream: 32-row steps (64 KB of dz5 + 8 KB of y4)
//   through a 2-stage LDS ring by LDS-DMA, counted waits, the next step's loads in flight while
//   this step's 72 MFMAs per wave run;
// * relu(bn4(y4)) is formed once per element, in LDS, one step ahead; the epilogue reads the raw
//   y4 of the step for bn4's ReLU mask and S2.
// dz5 rows carry the chunk permutation ftr of the r03 fused_seg.hip, now in git history (conflict-free fragment reads), y4
// rows the (row & 15) permutation (conflict-free epilogue reads), both put on the DMA source.
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int MS = 32;                      // rows per step
constexpr int K1 = 1024, K2 = 128, NC = 128;
constexpr int DZROW = K1 * 2;               // 2 KB dz5 row
constexpr int YROW = K2 * 2;                // 256 B y4 row
constexpr int DZB = MS * DZROW;             // 64 KB
constexpr int YB = MS * YROW;               // 8 KB
constexpr int STAGE = DZB + YB;
constexpr int NST = 2;
constexpr int OFF_A = NST * STAGE;          // relu(bn4(y4)) of the next step [MS][256 B]
constexpr int OFF_CF = OFF_A + YB;          // pa | pb (split layout) [2][128], then bias | es | et | em | er [5][128]
constexpr int BYTES = OFF_CF + 7 * NC * 4;
static_assert(BYTES <= 160 * 1024, "LDS budget");
constexpr int KS1 = K1 / 32, KS2 = K2 / 32;  // MFMA k-steps
constexpr int DZP = DZB / 1024;             // 64 pieces: 8 per wave

typedef __attribute__((address_space(3))) void lds_void_t;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
PCS_DEV int ftr(int row) { return ((row & 3) << 1) | (row & 8); }
PCS_DEV int fyp(int row) { return row & 15; }

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
PCS_DEV float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
PCS_DEV float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
PCS_DEV int split_idx(int i, int n) { return ((i & 7) >> 2) * (n / 2) + (i >> 3) * 4 + (i & 3); }
PCS_DEV void lds_vec8(const char *p, int half_bytes, float (&v)[8]) {
  const u32x4 x = *reinterpret_cast<const u32x4 *>(p);
  const u32x4 y = *reinterpret_cast<const u32x4 *>(p + half_bytes);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = __uint_as_float(x[e]);
    v[4 + e] = __uint_as_float(y[e]);
  }
}

__global__ __launch_bounds__(THREADS) void c5_dgrad_kernel(pcs_gemm_args a, int64_t rows_per_chunk) {
  __shared__ __attribute__((aligned(16))) char lds[BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int chunk = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  const int cps = a.chunks_per_scene;
  const int scene = __builtin_amdgcn_readfirstlane(chunk / cps), cis = __builtin_amdgcn_readfirstlane(chunk % cps);
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)cis * rows_per_chunk;
  const int64_t hi = pcs_min64(lo + rows_per_chunk, N);
  const int64_t sbase = (int64_t)scene * N;
  const int nsteps = (int)((hi - lo + MS - 1) / MS);   // >= 1 (no empty chunks)
  const char *dZg = reinterpret_cast<const char *>(a.A);    // dz5 [M][1024]
  const char *Yg = reinterpret_cast<const char *>(a.A2);    // y4  [M][128]
  const bf16_t *Ws = reinterpret_cast<const bf16_t *>(a.W);    // [128][1024]
  const bf16_t *H4 = reinterpret_cast<const bf16_t *>(a.W2);   // [128][128]

  // ---- constants into LDS: bn4's (scale, shift) in the split layout of the transform, and the
  // epilogue's per-column bias | es | et | emean | erstd
  {
    float *cf = reinterpret_cast<float *>(lds + OFF_CF);
    if (tid < NC) {
      const int j = split_idx(tid, NC);
      cf[j] = a.pa[tid];
      cf[NC + j] = a.pb[tid];
      cf[2 * NC + tid] = a.bias ? a.bias[tid] : 0.f;
      cf[3 * NC + tid] = a.es ? a.es[tid] : 1.f;
      cf[4 * NC + tid] = a.et ? a.et[tid] : 0.f;
      cf[5 * NC + tid] = a.emean ? a.emean[tid] : 0.f;
      cf[6 * NC + tid] = a.erstd ? a.erstd[tid] : 0.f;
    }
  }

  // ---- DMA: dz5 piece j = wid + 8 i (row j / 2, half j & 1), y4 piece wid (rows 4 wid ..)
  auto dz_off = [&](int i, int lastr) -> uint32_t {
    const int j = wid + 8 * i, r = j >> 1;
    const int logical = ((j & 1) * 64 + lane) ^ ftr(r);
    return (uint32_t)(min(r, lastr) * DZROW + (logical << 4));
  };
  auto y_off = [&](int lastr) -> uint32_t {
    const int r = 4 * wid + (lane >> 4);
    return (uint32_t)(min(r, lastr) * YROW + (((lane & 15) ^ fyp(r)) << 4));
  };
  uint32_t voff[DZP / 8 + 1];
#pragma unroll
  for (int i = 0; i < DZP / 8; ++i) voff[i] = dz_off(i, MS - 1);
  voff[DZP / 8] = y_off(MS - 1);
  const uint32_t lds_m0 = (uint32_t)(uintptr_t)(lds_void_t *)lds;
  auto dma_issue = [&](int sidx, int64_t m0, const uint32_t (&vo)[DZP / 8 + 1]) {
    const uint32_t mb = lds_m0 + sidx * STAGE + wid * 1024;
    const char *bdz = dZg + (sbase + m0) * DZROW;
    const char *by = Yg + (sbase + m0) * YROW;
    const uint32_t keep = m0_save();
    glds16o<0>(bdz, vo[0], mb);
    glds16o<8192>(bdz, vo[1], mb);
    glds16o<16384>(bdz, vo[2], mb);
    glds16o<24576>(bdz, vo[3], mb);
    glds16o<32768>(bdz, vo[4], mb);
    glds16o<40960>(bdz, vo[5], mb);
    glds16o<49152>(bdz, vo[6], mb);
    glds16o<57344>(bdz, vo[7], mb);
    glds16o<DZB>(by, vo[8], mb);
    m0_restore(keep);
  };
  static_assert(DZP / 8 == 8, "eight dz5 pieces per wave per step");
  auto dma_step = [&](int s, int sidx) {
    const int64_t m0 = pcs_min64(lo + (int64_t)s * MS, hi - 1);
    const int lastr = (int)pcs_min64(hi - 1 - m0, MS - 1);
    if (lastr == MS - 1) {   // uniform: a full step
      dma_issue(sidx, m0, voff);
    } else {
      uint32_t vt[DZP / 8 + 1];
#pragma unroll
      for (int i = 0; i < DZP / 8; ++i) vt[i] = dz_off(i, lastr);
      vt[DZP / 8] = y_off(lastr);
      dma_issue(sidx, m0, vt);
    }
  };

  // ---- this wave's 16 output columns of Ws^T / H4^T as MFMA operands (lane: column 16 ct + l16,
  // k chunk 4 kk + g)
  const int l16 = lane & 15, g = lane >> 4, ct = wid;
  u32x4 wfr[KS1], wh[KS2];
#pragma unroll
  for (int kk = 0; kk < KS1; ++kk)
    wfr[kk] = *reinterpret_cast<const u32x4 *>(Ws + (int64_t)(16 * ct + l16) * K1 + (4 * kk + g) * 8);
#pragma unroll
  for (int kk = 0; kk < KS2; ++kk)
    wh[kk] = *reinterpret_cast<const u32x4 *>(H4 + (int64_t)(16 * ct + l16) * K2 + (4 * kk + g) * 8);

  // loop-invariant LDS offsets: fragment chunk 4 kk + g of row 16 u + l16 sits at chunk
  // 16 (kk >> 2) + ((4 (kk & 3) + g) ^ ftr(l16))
  int xb[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) xb[b] = ((4 * b + g) ^ ftr(l16)) << 4;
  const int cc = 16 * ct + 4 * g;   // the lane's 4 output columns (epilogue)
  const int o_ye = DZB + l16 * YROW + ((((cc >> 3) ^ l16) << 4) | ((cc & 7) << 1));   // + u 16 rows
  const int trow = tid >> 4, tpc = tid & 15, tlc = tpc ^ fyp(trow);   // transform: one chunk per thread
  const int o_ty = DZB + trow * YROW + tpc * 16;
  const int o_ta = OFF_A + trow * YROW + ((tlc ^ ftr(trow)) << 4);
  const char *cft = lds + OFF_CF + tlc * 16;

  f32x4 accd[2];
  float s1[4], s2[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { s1[r] = 0.f; s2[r] = 0.f; }

  // relu(bn4(y4)) of step s (landed in stage sidx) into the A buffer; zeros past the slice
  auto transform = [&](int s, int sidx) {
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)s * MS), MS);
    float sc[8], sh[8], v[8];
    lds_vec8(cft, NC * 2, sc);
    lds_vec8(cft + NC * 4, NC * 2, sh);
    unpack_chunk(*reinterpret_cast<const u32x4 *>(lds + sidx * STAGE + o_ty), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = relu(fmaf(v[e], sc[e], sh[e]));
    u32x4 out = pack_chunk(v);
    if (rem < MS && trow >= rem) out = mk_u32x4(0, 0, 0, 0);
    *reinterpret_cast<u32x4 *>(lds + o_ta) = out;
  };

  // output rows through one buffer descriptor for the slice (rows past it dropped by the range
  // check, so every wave issues one store per step; the placeholder stores lie out of range)
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char *>(reinterpret_cast<bf16_t *>(a.C) + (sbase + lo) * NC), 0,
      (int)(uint32_t)((hi - lo) * NC * 2), 0x00020000);
  uint32_t o_out = (uint32_t)((16 * (g & 1) + l16) * (NC * 2) + (16 * ct + 8 * (g >> 1)) * 2);

  // ---- prologue: step 0 in flight (+ a dropped store: each step is loads then one store),
  // landed, transformed
  dma_step(0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(mk_u32x4(0, 0, 0, 0), rs_out, (int)0xFFFFFF00u, 0, 0);
  wait_vm<1>();
  barrier_lds();
  transform(0, 0);
  barrier_lds();

  int sc_ = 0;
  for (int t = 0; t < nsteps; ++t) {
    const int rem = (int)pcs_min64(hi - (lo + (int64_t)t * MS), MS);
    dma_step(t + 1, sc_ ^ 1);   // into the stage step t-1 used (free since the last barrier)
    const char *st = lds + sc_ * STAGE;
    accd[0] = accd[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    {   // g = dz5 Ws^T over 32 k-steps (operand reads PD ahead), then relu(bn4(y4)) H4^T
      constexpr int PD = 2;
      bf16x8 yf[PD + 1][2];
      auto rd = [&](int kk, bf16x8 (&d)[2]) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
          d[u] = *reinterpret_cast<const bf16x8 *>(st + (16 * u + l16) * DZROW + (kk >> 2) * 256 + xb[kk & 3]);
      };
#pragma unroll
      for (int kk = 0; kk < PD; ++kk) rd(kk, yf[kk]);
#pragma unroll
      for (int kk = 0; kk < KS1; ++kk) {
        if (kk + PD < KS1) rd(kk + PD, yf[(kk + PD) % (PD + 1)]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2; ++u)
          accd[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wfr[kk]), yf[kk % (PD + 1)][u],
                                                           accd[u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int kk = 0; kk < KS2; ++kk)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16x8 af = *reinterpret_cast<const bf16x8 *>(lds + OFF_A + (16 * u + l16) * YROW + xb[kk]);
          accd[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wh[kk]), af, accd[u], 0, 0, 0);
        }
    }
    // epilogue: + c5, bn4's ReLU mask, S1 / S2, 16-B stores (lane groups trade row tiles)
    {
      const float *cf = reinterpret_cast<const float *>(lds + OFF_CF);
      const float4 bb = *reinterpret_cast<const float4 *>(cf + 2 * NC + cc);
      const float4 es = *reinterpret_cast<const float4 *>(cf + 3 * NC + cc);
      const float4 et = *reinterpret_cast<const float4 *>(cf + 4 * NC + cc);
      const float4 em = *reinterpret_cast<const float4 *>(cf + 5 * NC + cc);
      const float4 er = *reinterpret_cast<const float4 *>(cf + 6 * NC + cc);
      const float b4[4] = {bb.x, bb.y, bb.z, bb.w}, es4[4] = {es.x, es.y, es.z, es.w};
      const float et4[4] = {et.x, et.y, et.z, et.w}, em4[4] = {em.x, em.y, em.z, em.w}, er4[4] = {er.x, er.y, er.z, er.w};
      uint32_t pk[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint2 yp = *reinterpret_cast<const uint2 *>(st + o_ye + u * 16 * YROW);
        const float y[4] = {bf_lo(yp.x), bf_hi(yp.x), bf_lo(yp.y), bf_hi(yp.y)};
        const bool live = 16 * u + l16 < rem;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = fmaf(y[r], es4[r], et4[r]);
          v[r] = (live & (z > 0.f)) ? accd[u][r] + b4[r] : 0.f;
          s1[r] += v[r];
          s2[r] = fmaf(v[r], (y[r] - em4[r]) * er4[r], s2[r]);
        }
        pk[u][0] = pack2bf(v[0], v[1]);
        pk[u][1] = pack2bf(v[2], v[3]);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][h], pk[1][h], false, false);
        pk[0][h] = sw[0];
        pk[1][h] = sw[1];
      }
      __builtin_amdgcn_raw_buffer_store_b128(mk_u32x4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]), rs_out, (int)o_out, 0, 0);
      o_out += MS * NC * 2;
    }
    // step t+1 landed (only this step's store is newer)
    wait_vm<1>();
    barrier_lds();
    if (t + 1 < nsteps) transform(t + 1, sc_ ^ 1);
    barrier_lds();
    sc_ ^= 1;
  }
  wait_vm<0>();

  // ---- S1 / S2 of this chunk: over the 16 lanes (rows) of each column
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s1[r] += __shfl_xor(s1[r], o);
      s2[r] += __shfl_xor(s2[r], o);
    }
  if (a.stats && l16 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<float2 *>(a.stats + ((int64_t)chunk * NC + cc + r) * 2) = make_float2(s1[r], s2[r]);
  }
}

}  // namespace

// conv5's folded input gradient: bf16, PCS_PRO_CAT with K1 = 1024, K - K1 = 128, 128 output
// columns, EPI_DGRAD without dropout bits, addend or sparse pool rows.
bool pcs_c5_dgrad_class(const pcs_gemm_args &a) {
  return a.dtype == PCS_BF16 && !(a.flags & PCS_FLAG_GENERIC) && a.prologue == PCS_PRO_CAT &&
         a.epilogue == PCS_EPI_DGRAD && a.K1 == K1 && a.K == K1 + K2 && a.Ncols == NC;
}

bool pcs_c5_dgrad_applicable(const pcs_gemm_args &a) {
  return pcs_c5_dgrad_class(a) && !a.c_mask && !a.addend && !a.pool_w && a.A2 && a.W2 && a.pa && a.pb && a.C &&
         a.Yp == a.A2 && (!a.erstd || a.emean);
}

int pcs_c5_dgrad_launch(const pcs_gemm_args &a, int64_t rows_per_chunk, hipStream_t s) {
  if (rows_per_chunk % MS != 0) return pcs_set_einval("pcs_gemm", "c5 dgrad: rows per chunk must be a multiple of 32");
  const int nb = (int)(a.num_scenes * a.chunks_per_scene);
  hipLaunchKernelGGL(c5_dgrad_kernel, dim3(nb), dim3(THREADS), 0, s, a, rows_per_chunk);
  PCS_CHECK_LAUNCH();
  return 0;
}

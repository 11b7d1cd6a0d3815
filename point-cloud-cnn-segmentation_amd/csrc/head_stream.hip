// The segmentation head's training pass as a stream (pcs_head, PCS_HEAD_CE, C <= 4 classes, bf16,
// no logits out): seg_conv4 (P:128) on relu(bn_seg3(y)), the weighted CE (P:216, P:251) and its
// gradient, dz_s3 = relu'(.) (dlogits W), bn_seg3's S1 / S2, dW / db of seg_conv4.
//
// The register-resident head_small_kernel (small.hip) holds its batch of rows in VGPRs: at 234
// VGPRs (2 waves / SIMD) its loads in flight (~32 KB per CU) leave it at 3.3 TB/s.  Here the rows
// come in by LDS-DMA, so the bytes in flight no longer cost registers:
// * every wave streams its own 8 rows of each 64-row step (2 KB of y, 64 B of labels) through a
//   wave-private NST-stage LDS ring and computes exactly those rows: no barrier in the loop, only
//   the wave's counted vmcnt waits (its DMAs and its two output stores per step, in order);
// * 4 stages and at most 128 VGPRs (S2 kept as sum dz y, centred by the mean at the end), so two
//   workgroups share a CU; 1024 in the grid: 1.05 -> 0.98 ms against 8 stages at one per CU;
// * 16 lanes per row (one 16-B chunk of 8 channels each), logits all-reduced by shuffles, as the
//   register kernel; class weights in registers (no gathers in the loop);
// * dz rows go out through a buffer descriptor limited to the chunk's rows (the hardware drops
//   rows past it), so every wave issues the same stores every step.
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int CIN = 128;
constexpr int ROWB = CIN * 2;          // 256-B y rows
constexpr int MS = 64;                 // rows per step (8 per wave)
constexpr int WR = 8;                  // rows per wave per step
constexpr int YW = WR * ROWB;          // 2 KB of y per wave per step
constexpr int WAVEB = YW + WR * 8;     // + 64 B of labels
#ifndef HS_NST
#define HS_NST 4
#endif
#ifndef HS_WPS
#define HS_WPS 4   // waves per SIMD requested for C <= 2: two workgroups per CU, at most 128 VGPRs
                   // (no spills; C = 3, 4 would spill 60-70 registers there and keep one per CU)
#endif
constexpr int NST = HS_NST;
constexpr int BYTES = 8 * NST * WAVEB;
static_assert(BYTES <= 160 * 1024, "LDS budget");
constexpr int LPS = 3;                 // DMAs per wave per step: two y pieces, one label piece
constexpr int SPS = 2;                 // output stores per wave per step
static_assert((NST - 1) * (LPS + SPS) < 64, "vmcnt range");

typedef __attribute__((address_space(3))) void lds_void_t;

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

template <int C>
__global__ __launch_bounds__(THREADS, (C <= 2 ? HS_WPS : 1)) void head_stream_kernel(pcs_head_args a, int64_t rows_per_chunk) {
  __shared__ __attribute__((aligned(16))) char lds[BYTES];
  __shared__ float red[THREADS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane & 15, rq = lane >> 4, ch0 = sub * 8;
  const int cps = a.chunks_per_scene;
  const int scene = blockIdx.x / cps, cis = blockIdx.x % cps;
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)cis * rows_per_chunk, hi = pcs_min64(lo + rows_per_chunk, N);
  const int64_t sbase = (int64_t)scene * N;
  const int nsteps = hi > lo ? (int)((hi - lo + MS - 1) / MS) : 0;

  float s[8], t[8], w[C][8], bias[C], cw[C];
  load_vec<8>(a.s, ch0, s);
  load_vec<8>(a.t, ch0, t);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    load_vec<8>(a.W + c * CIN, ch0, w[c]);
    bias[c] = a.bias[c];
    cw[c] = a.class_weight[c];
  }
  const float gsc = a.wsum ? 1.f / *a.wsum : 1.f;
  // the ordinary loads above retire before the first DMA (the counted waits see only the ring)
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(s[e]), "v"(t[e]));
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(w[c][e]));
    asm volatile("" ::"v"(bias[c]), "v"(cw[c]));
  }
  asm volatile("" ::"v"(gsc));
  __syncthreads();

  // ---- DMA of step st into this wave's stage st % NST: y rows 8 wid + 4 i + rq (i = 0, 1), label
  // words of rows 8 wid + lane / 2 (lanes 0..15); rows past the chunk clamp to its last row
  const char *Yg = reinterpret_cast<const char *>(a.Y);
  const char *Lg = reinterpret_cast<const char *>(a.labels);
  const uint32_t lds_w = (uint32_t)(uintptr_t)(lds_void_t *)lds + wid * NST * WAVEB;
  auto dma_step = [&](int st) {
    const int64_t m0 = pcs_min64(lo + (int64_t)st * MS, hi - 1);
    const int lastr = (int)pcs_min64(hi - 1 - m0, MS - 1);
    const uint32_t mb = lds_w + (st % NST) * WAVEB;
    const char *by = Yg + (sbase + m0) * ROWB;
    const char *bl = Lg + (sbase + m0) * 8;
    const uint32_t v0 = (uint32_t)(min(WR * wid + rq, lastr) * ROWB + sub * 16);
    const uint32_t v1 = (uint32_t)(min(WR * wid + 4 + rq, lastr) * ROWB + sub * 16);
    const uint32_t vl = (uint32_t)(min(WR * wid + (lane >> 1), lastr) * 8 + 4 * (lane & 1));
    const uint32_t keep = m0_save();
    glds16o<0>(by, v0, mb);
    glds16o<1024>(by, v1, mb);
    if (lane < 16) glds4o<YW>(bl, vl, mb);
    m0_restore(keep);
  };

  // ---- dz rows through a descriptor limited to the chunk's rows
  char *dZc = reinterpret_cast<char *>(a.dZ) + (sbase + lo) * ROWB;
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
      dZc, 0, (int)(uint32_t)(hi > lo ? (hi - lo) * ROWB : 0), 0x00020000);
  auto store_row = [&](uint32_t vo, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, rs_out, (int)vo, 0, 2); };

  float s1[8], s2[8], dw[C][8], db[C], lsum = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    db[c] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) dw[c][e] = 0.f;
  }

  // prologue: steps 0 .. NST-2 in flight, each followed by two stores the range check drops (as
  // every loop step's DMA is followed by its two row stores)
#pragma unroll
  for (int st = 0; st < NST - 1; ++st) {
    dma_step(st);
    store_row(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
    store_row(0xFFFFFE00u, mk_u32x4(0, 0, 0, 0));
  }

  for (int it = 0; it < nsteps; ++it) {
    dma_step(it + NST - 1);
    wait_vm<(NST - 1) * (LPS + SPS)>();   // step it landed (this wave's part)
    const char *stg = lds + wid * NST * WAVEB + (it % NST) * WAVEB;
    const int64_t rbase = (int64_t)it * MS + WR * wid;   // chunk-relative row of the wave's first
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rr = 4 * h + rq;
      const int64_t rrel = rbase + rr;
      const bool ok = lo + rrel < hi;
      const u32x4 yv = *reinterpret_cast<const u32x4 *>(stg + rr * ROWB + sub * 16);
      const uint2 lb = *reinterpret_cast<const uint2 *>(stg + YW + rr * 8);
      float y[8], av[8];
      unpack_chunk(yv, y);
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = relu(fmaf(y[e], s[e], t[e]));
      float lg[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float p = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) p = fmaf(av[e], w[c][e], p);
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) p += __shfl_xor(p, o);
        lg[c] = p + bias[c];
      }
      float mx = lg[0];
#pragma unroll
      for (int c = 1; c < C; ++c) mx = fmaxf(mx, lg[c]);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) se += expf(lg[c] - mx);
      const float lse = mx + logf(se);
      // int64 label: valid iff 0 <= l < C (high word 0, low word < C); -1 and the rest ignored
      const bool valid = ok && lb.y == 0u && lb.x < (uint32_t)C;
      const int l = (int)lb.x;
      float wt = 0.f, zl = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c)
        if (c == l) { wt = cw[c]; zl = lg[c]; }
      wt = valid ? wt : 0.f;
      float dl[C];
#pragma unroll
      for (int c = 0; c < C; ++c) dl[c] = wt * gsc * (expf(lg[c] - lse) - (c == l ? 1.f : 0.f));
      if (valid && sub == 0) lsum += wt * (lse - zl);
      float dz[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) d = fmaf(dl[c], w[c][e], d);
        dz[e] = av[e] > 0.f ? d : 0.f;
        s1[e] += dz[e];
        s2[e] = fmaf(dz[e], y[e], s2[e]);   // sum dz y; S2 = rstd (sum dz y - mean S1) at the end
#pragma unroll
        for (int c = 0; c < C; ++c) dw[c][e] = fmaf(dl[c], av[e], dw[c][e]);
      }
#pragma unroll
      for (int c = 0; c < C; ++c) db[c] += dl[c];
      // rows past the chunk: dz = 0 (wt = 0) and the store is dropped by the range check
      store_row((uint32_t)(rrel * ROWB + sub * 16), pack_chunk(dz));
    }
  }
  wait_vm<0>();   // the clamped DMAs past the end, the last stores

  // ---- reduce over the 32 row slots sharing a channel chunk (same `sub`), one value at a time
  const int r0 = tid / 16;
  const int64_t chunk = blockIdx.x;
  auto reduce_store = [&](float v, float *dst) {
    red[tid] = v;
    __syncthreads();
    if (r0 == 0 && dst) {
      float acc = 0.f;
      for (int j = 0; j < THREADS / 16; ++j) acc += red[j * 16 + sub];
      *dst = acc;
    }
    __syncthreads();
  };
  {
    float mu[8], rs[8];
    load_vec<8>(a.mean, ch0, mu);
    load_vec<8>(a.rstd, ch0, rs);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // (the pre-BN rows are stored without the conv bias, so they are centred: no cancellation)
      s2[e] = rs[e] * (s2[e] - mu[e] * s1[e]);
      reduce_store(s1[e], a.stats + (chunk * CIN + ch0 + e) * 2);
      reduce_store(s2[e], a.stats + (chunk * CIN + ch0 + e) * 2 + 1);
    }
  }
  float *wp = a.wpartial + chunk * (C * CIN + C);
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int e = 0; e < 8; ++e) reduce_store(dw[c][e], wp + c * CIN + ch0 + e);
    // every lane of a row holds the same db: sum over rows = over the sub-0 lanes
    reduce_store(db[c], sub == 0 ? wp + C * CIN + c : nullptr);
  }
  float ls = lsum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) ls += __shfl_xor(ls, o);
  if (lane == 0) red[wid] = ls;
  __syncthreads();
  if (tid == 0) {
    float acc = 0.f;
    for (int i = 0; i < THREADS / 64; ++i) acc += red[i];
    a.loss_partial[chunk] = acc;
  }
}

}  // namespace

// bf16, CE mode, C <= 4, no logits out (the fused train step); shapes / modes only
bool pcs_head_stream_class(const pcs_head_args &a) {
  return a.dtype == PCS_BF16 && a.mode == PCS_HEAD_CE && a.num_classes >= 1 && a.num_classes <= 4 &&
         !a.logits && a.Cin == CIN && a.num_scenes * a.scene_rows < ((int64_t)1 << 31);
}

#ifndef HS_TARGET
#define HS_TARGET 1024
#endif
int pcs_head_stream_target() { return HS_TARGET; }

int pcs_head_stream_launch(const pcs_head_args &a, int64_t rows_per_chunk, hipStream_t s) {
  if (rows_per_chunk % MS) return pcs_set_einval("pcs_head", "stream head: rows per chunk must be a multiple of 64");
  if (rows_per_chunk * ROWB >= ((int64_t)1 << 31)) return pcs_set_einval("pcs_head", "stream head: chunk too large");
  const int nb = (int)(a.num_scenes * a.chunks_per_scene);
  switch (a.num_classes) {
    case 1: hipLaunchKernelGGL(head_stream_kernel<1>, dim3(nb), dim3(THREADS), 0, s, a, rows_per_chunk); break;
    case 2: hipLaunchKernelGGL(head_stream_kernel<2>, dim3(nb), dim3(THREADS), 0, s, a, rows_per_chunk); break;
    case 3: hipLaunchKernelGGL(head_stream_kernel<3>, dim3(nb), dim3(THREADS), 0, s, a, rows_per_chunk); break;
    default: hipLaunchKernelGGL(head_stream_kernel<4>, dim3(nb), dim3(THREADS), 0, s, a, rows_per_chunk); break;
  }
  PCS_CHECK_LAUNCH();
  return 0;
}

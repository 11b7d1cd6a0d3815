// Streaming forward GEMM for shallow-K, write-heavy layers (pcs_gemm, bf16): seg_conv1's
// local half (64 -> 512, per-scene bias, BN statistics; P:117-123).  The template also
// covers conv2-5 and seg_conv3 shapes (see kShapes for why they are not routed here).
//
// With K <= 256 the MFMA work per output row is small and the pass is bound by writing the
// output (and reading A), so the tile pipeline of the 256x256 kernels -- K-steps staged per
// tile, a prologue and an epilogue per tile -- spends most of its time in per-tile overhead
// (gemm_big at K = 128 runs at 645 TF/s with no epilogue at all).  Here a workgroup keeps its
// NB-column block of W resident in LDS for its whole life and streams MS-row slabs of A:
//   A slab (BN+ReLU [+ dropout] prologue) -> LDS; NB x K MFMAs; epilogue in registers
//   (bias / per-scene bias, BN statistics or this layer's BN+ReLU) -> bf16 tile in LDS ->
//   coalesced 16-B row stores;  the next slab's loads are in flight during all of it.
// BN statistics: per-lane sums of (y - K_c) and (y - K_c)^2 with K_c the chunk's first row
// (same shift for every lane of a column, so lanes and waves merge by plain adds), written
// once per chunk as (mean, M2) in pcs_gemm's partial layout; computed on the stored (bf16)
// values, like the other kernels.
#include "common.h"

namespace {

constexpr int THREADS = 512;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

PCS_DEV void lds_vec8(const float *p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4 *>(p);
  const float4 b = *reinterpret_cast<const float4 *>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <int K, int NB, int MS> struct SG {
  static constexpr int W_ROWB = K * 2;              // W block [NB][K], XOR-swizzled 16-B slots
  static constexpr int A_ROWB = K * 2 + 16;         // A slab [MS][K] (+16 B: conflict-free b128 reads)
  static constexpr int O_ROWB = NB * 2;             // output tile [MS][NB] bf16
  static constexpr int OFF_A = NB * W_ROWB;
  static constexpr int OFF_O = OFF_A + MS * A_ROWB;
  static constexpr int OFF_C = OFF_O + MS * O_ROWB; // pa | pb [K], ebias | es | et [NB], shift [NB]
  static constexpr int BYTES = OFF_C + (2 * K + 4 * NB) * 4;
  static_assert(BYTES <= 160 * 1024, "LDS budget");
  static constexpr int NCB = NB / 16, NMB = MS / 16;
  static constexpr int CBW = NCB >= 8 ? NCB / 8 : 1;    // column blocks per wave
  static constexpr int GROUPS = NCB / CBW;              // column groups
  static constexpr int WPG = 8 / GROUPS;                // waves per column group
  static constexpr int MBW = NMB / WPG;                 // row blocks per wave
  static_assert(GROUPS * CBW == NCB && WPG * GROUPS == 8 && MBW * WPG == NMB, "wave tiling");
  static constexpr int NCH_A = MS * K / 8 / THREADS;    // A chunks per thread
  static constexpr int NCH_O = MS * NB / 8 / THREADS;   // output chunks per thread
  static_assert(NCH_A >= 1 && NCH_O >= 1, "staging");
};

// EPI: PCS_EPI_FWD (bias / scene bias, optional stats, optional store) or PCS_EPI_BNRELU
template <int K, int NB, int MS, int EPI, bool AMASK>
__global__ __launch_bounds__(THREADS) void gemm_stream_kernel(pcs_gemm_args a, int64_t rows_per_chunk, int ncb) {
  typedef SG<K, NB, MS> S;
  __shared__ __attribute__((aligned(16))) char lds[S::BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = L / ncb, cbk = L % ncb;
  const int cps = a.chunks_per_scene;
  const int scene = chunk / cps, cis = chunk % cps;
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)cis * rows_per_chunk;
  const int64_t hi = pcs_min64(lo + rows_per_chunk, N);
  const int64_t sbase = (int64_t)scene * N;
  const int n0 = cbk * NB;
  const int Ncols = a.Ncols;
  const bf16_t *__restrict__ Ag = reinterpret_cast<const bf16_t *>(a.A);
  const bf16_t *__restrict__ Wg = reinterpret_cast<const bf16_t *>(a.W);
  bf16_t *__restrict__ Cg = reinterpret_cast<bf16_t *>(a.C);
  const bool pro = a.prologue == PCS_PRO_BNRELU;
  const bool do_stats = EPI == PCS_EPI_FWD && a.stats != nullptr;

  for (int i = tid; i < NB * K / 8; i += THREADS) {   // W block [NB][K] -> LDS
    const int c = i / (K / 8), slot = i % (K / 8);
    *reinterpret_cast<u32x4 *>(lds + c * S::W_ROWB + ((slot ^ (c & 7)) << 4)) =
        *reinterpret_cast<const u32x4 *>(Wg + (int64_t)(n0 + c) * K + slot * 8);
  }
  float *cf = reinterpret_cast<float *>(lds + S::OFF_C);
  float *ebias = cf + 2 * K, *ces = ebias + NB, *cet = ces + NB, *csh = cet + NB;
  for (int i = tid; i < K; i += THREADS) {
    cf[i] = pro ? a.pa[i] : 1.f;
    cf[K + i] = pro ? a.pb[i] : 0.f;
  }
  const float *bias = a.scene_bias ? a.scene_bias + (int64_t)scene * Ncols : a.bias;
  for (int i = tid; i < NB; i += THREADS) {
    ebias[i] = bias ? bias[n0 + i] : 0.f;
    if constexpr (EPI == PCS_EPI_BNRELU) { ces[i] = a.es[n0 + i]; cet[i] = a.et[n0 + i]; }
  }
  __syncthreads();

  u32x4 ra[S::NCH_A];
  uint32_t rm[AMASK ? S::NCH_A : 1];
  auto load_step = [&](int64_t m0) {
#pragma unroll
    for (int i = 0; i < S::NCH_A; ++i) {
      const int q = tid + THREADS * i, rl = q / (K / 8), cc = q % (K / 8);
      const int64_t off = (sbase + pcs_min64(m0 + rl, hi - 1)) * K + cc * 8;
      ra[i] = *reinterpret_cast<const u32x4 *>(Ag + off);
      if constexpr (AMASK) rm[i] = a.a_mask[off >> 3];
    }
  };
  auto store_step = [&]() {
#pragma unroll
    for (int i = 0; i < S::NCH_A; ++i) {
      const int q = tid + THREADS * i, rl = q / (K / 8), cc = q % (K / 8);
      u32x4 out = ra[i];
      if (pro) {
        float s8[8], t8[8], v[8];
        lds_vec8(cf + cc * 8, s8); lds_vec8(cf + K + cc * 8, t8);
        unpack_chunk(ra[i], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = fmaxf(fmaf(v[e], s8[e], t8[e]), 0.f);
          if constexpr (AMASK) x = ((rm[i] >> e) & 1u) ? x * a.a_keep_scale : 0.f;
          v[e] = x;
        }
        out = pack_chunk(v);
      }
      *reinterpret_cast<u32x4 *>(lds + S::OFF_A + rl * S::A_ROWB + cc * 16) = out;
    }
  };

  const int g = lane >> 4, l16 = lane & 15;
  const int grp = wid % S::GROUPS, part = wid / S::GROUPS;
  const int cb0 = grp * S::CBW, mb0 = part * S::MBW;
  // per-lane column statistics (sums of y - shift); the shift and the epilogue coefficients
  // are read from LDS where used (fewer live registers at NB = 512)
  float s1[S::CBW][4], s2[S::CBW][4];
#pragma unroll
  for (int j = 0; j < S::CBW; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
  if (do_stats)
    for (int i = tid; i < NB; i += THREADS) csh[i] = 0.f;   // step 0 sums unshifted

  const int nsteps = (int)((hi - lo + MS - 1) / MS);
  if (nsteps > 0) {
    load_step(lo);
    store_step();
    __builtin_amdgcn_sched_barrier(0);
    load_step(lo + MS);
  }
  __syncthreads();

  for (int st = 0; st < nsteps; ++st) {
    const int64_t m0 = lo + (int64_t)st * MS;
    f32x4 acc[S::MBW][S::CBW];
#pragma unroll
    for (int i = 0; i < S::MBW; ++i)
#pragma unroll
      for (int j = 0; j < S::CBW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < K / 32; ++kk) {
      const int slot = 4 * kk + g;
      bf16x8 wf[S::CBW];
#pragma unroll
      for (int j = 0; j < S::CBW; ++j) {
        const int c = (cb0 + j) * 16 + l16;
        wf[j] = *reinterpret_cast<const bf16x8 *>(lds + c * S::W_ROWB + ((slot ^ (c & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < S::MBW; ++i) {
        const int r = (mb0 + i) * 16 + l16;
        const bf16x8 af = *reinterpret_cast<const bf16x8 *>(lds + S::OFF_A + r * S::A_ROWB + slot * 16);
#pragma unroll
        for (int j = 0; j < S::CBW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af, acc[i][j], 0, 0, 0);
      }
    }
    // epilogue in registers: lane holds y[m = 16 (mb0 + i) + l16][c = 16 (cb0 + j) + 4 g + r]
#pragma unroll
    for (int i = 0; i < S::MBW; ++i) {
      const int ml = (mb0 + i) * 16 + l16;
      const bool live = m0 + ml < hi;
#pragma unroll
      for (int j = 0; j < S::CBW; ++j) {
        const int c = (cb0 + j) * 16 + 4 * g;
        const float4 eb = *reinterpret_cast<const float4 *>(ebias + c);
        float v[4] = {acc[i][j][0] + eb.x, acc[i][j][1] + eb.y, acc[i][j][2] + eb.z, acc[i][j][3] + eb.w};
        if constexpr (EPI == PCS_EPI_BNRELU) {
          const float4 e4 = *reinterpret_cast<const float4 *>(ces + c);
          const float4 t4 = *reinterpret_cast<const float4 *>(cet + c);
          v[0] = fmaxf(fmaf(v[0], e4.x, t4.x), 0.f); v[1] = fmaxf(fmaf(v[1], e4.y, t4.y), 0.f);
          v[2] = fmaxf(fmaf(v[2], e4.z, t4.z), 0.f); v[3] = fmaxf(fmaf(v[3], e4.w, t4.w), 0.f);
        }
        const uint2 pk = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        *reinterpret_cast<uint2 *>(lds + S::OFF_O + ml * S::O_ROWB + c * 2) = pk;
        if (do_stats && live) {
          const float4 k4 = *reinterpret_cast<const float4 *>(csh + c);
          const float y[4] = {__uint_as_float(pk.x << 16) - k4.x, __uint_as_float(pk.x & 0xffff0000u) - k4.y,
                              __uint_as_float(pk.y << 16) - k4.z, __uint_as_float(pk.y & 0xffff0000u) - k4.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1[j][r] += y[r];
            s2[j][r] = fmaf(y[r], y[r], s2[j][r]);
          }
        }
      }
    }
    lds_barrier();   // slab consumed, output tile complete
    float ksh[S::CBW][4];
    if (st == 0 && do_stats) {
      // shift = the chunk's first row (step 0 summed unshifted; re-based below):
      // sum (y - K) = sum y - n K, sum (y - K)^2 = sum y^2 - 2 K sum y + n K^2
#pragma unroll
      for (int j = 0; j < S::CBW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = (cb0 + j) * 16 + 4 * g + r;
          ksh[j][r] = __uint_as_float((uint32_t)*reinterpret_cast<const unsigned short *>(lds + S::OFF_O + c * 2) << 16);
        }
      for (int c = tid; c < NB; c += THREADS)
        csh[c] = __uint_as_float((uint32_t)*reinterpret_cast<const unsigned short *>(lds + S::OFF_O + c * 2) << 16);
    }
#pragma unroll
    for (int i = 0; i < S::NCH_O; ++i) {
      const int q = tid + THREADS * i, rl = q / (NB / 8), cc = q % (NB / 8);
      if (Cg && m0 + rl < hi)
        *reinterpret_cast<u32x4 *>(Cg + (sbase + m0 + rl) * Ncols + n0 + cc * 8) =
            *reinterpret_cast<const u32x4 *>(lds + S::OFF_O + rl * S::O_ROWB + cc * 16);
    }
    if (st + 1 < nsteps) {
      store_step();
      __builtin_amdgcn_sched_barrier(0);
      load_step(m0 + 2 * MS);
    }
    lds_barrier();
    if (st == 0 && do_stats) {
      float nl = 0.f;   // rows of step 0 this lane summed (same for every column)
#pragma unroll
      for (int i = 0; i < S::MBW; ++i) nl += (m0 + (mb0 + i) * 16 + l16 < hi) ? 1.f : 0.f;
#pragma unroll
      for (int j = 0; j < S::CBW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float k = ksh[j][r];
          s2[j][r] = s2[j][r] - 2.f * k * s1[j][r] + nl * k * k;
          s1[j][r] = s1[j][r] - nl * k;
        }
    }
  }

  if (do_stats) {
    // lanes l16 of a column (rows) by xor-shuffles, then the WPG waves of a column group
#pragma unroll
    for (int j = 0; j < S::CBW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[j][r] += __shfl_xor(s1[j][r], o);
          s2[j][r] += __shfl_xor(s2[j][r], o);
        }
    float2 *red = reinterpret_cast<float2 *>(lds);   // [WPG][NB] over the W block (no longer read)
    if (l16 == 0) {
#pragma unroll
      for (int j = 0; j < S::CBW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[part * NB + (cb0 + j) * 16 + 4 * g + r] = make_float2(s1[j][r], s2[j][r]);
    }
    __syncthreads();
    const float n = (float)pcs_max64(hi - lo, 0);
    for (int c = tid; c < NB; c += THREADS) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int p = 0; p < S::WPG; ++p) { t1 += red[p * NB + c].x; t2 += red[p * NB + c].y; }
      const float d1 = n > 0.f ? t1 / n : 0.f;
      *reinterpret_cast<float2 *>(a.stats + ((int64_t)chunk * Ncols + n0 + c) * 2) =
          make_float2(csh[c] + d1, fmaxf(t2 - t1 * d1, 0.f));
    }
  }
}

// Shapes served.  Measured at cfg2 against the kernels they replace: seg_conv1 (64 -> 512)
// 2.83 ms vs 3.15 ms (gemm_nt 128x128); conv5 (128 -> 1024, NB 256) 7.1 ms vs 4.9 ms
// (gemm_big), seg_conv3 (256 -> 128) 2.6 vs 1.6, conv4 0.93 vs 0.66, conv2/3 0.59 vs 0.44:
// with one 512-thread workgroup per CU the slab barriers serialise the output stores, so only
// the write-heaviest shape (1 KB out per 128 B in) is routed here.  The kernel template keeps
// the shape-generic tiling so another shape is one table entry away.
struct StreamShape { int K, Ncols, NB, MS; };
constexpr StreamShape kShapes[] = {{64, 512, 512, 64}};

const StreamShape *stream_shape(const pcs_gemm_args &a) {
  if (a.dtype != PCS_BF16 || (a.flags & PCS_FLAG_GENERIC)) return nullptr;
  if (a.prologue != PCS_PRO_BNRELU && a.prologue != PCS_PRO_RAW) return nullptr;
  if (a.epilogue != PCS_EPI_FWD && a.epilogue != PCS_EPI_BNRELU) return nullptr;
  for (const StreamShape &s : kShapes)
    if (s.K == a.K && s.Ncols == a.Ncols) return &s;
  return nullptr;
}

template <int K, int NB, int MS>
int launch_shape(const pcs_gemm_args &a, int64_t rpc, hipStream_t s) {
  const int ncb = a.Ncols / NB;
  const int nb = ncb * (int)(a.num_scenes * a.chunks_per_scene);
  if (a.epilogue == PCS_EPI_BNRELU) {
    if (a.a_mask) hipLaunchKernelGGL((gemm_stream_kernel<K, NB, MS, PCS_EPI_BNRELU, true>), dim3(nb), dim3(THREADS), 0, s, a, rpc, ncb);
    else hipLaunchKernelGGL((gemm_stream_kernel<K, NB, MS, PCS_EPI_BNRELU, false>), dim3(nb), dim3(THREADS), 0, s, a, rpc, ncb);
  } else {
    if (a.a_mask) hipLaunchKernelGGL((gemm_stream_kernel<K, NB, MS, PCS_EPI_FWD, true>), dim3(nb), dim3(THREADS), 0, s, a, rpc, ncb);
    else hipLaunchKernelGGL((gemm_stream_kernel<K, NB, MS, PCS_EPI_FWD, false>), dim3(nb), dim3(THREADS), 0, s, a, rpc, ncb);
  }
  PCS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// Geometry: ~256 workgroups (one per CU at the LDS sizes of the wide shapes); chunks are a
// multiple of 256 rows, so the 128- and 256-row kernels can walk the same chunks when an
// operand combination this kernel does not take falls back to them.
int64_t pcs_gemm_stream_geometry(pcs_gemm_args *a) {
  const StreamShape *sh = stream_shape(*a);
  if (!sh) return 0;
  return pcs_fill_geometry(a, 256, 256, a->Ncols / sh->NB);
}

bool pcs_gemm_stream_applicable(const pcs_gemm_args &a) {
  if (!stream_shape(a) || a.pool || (a.epilogue == PCS_EPI_BNRELU && (!a.es || !a.et))) return false;
  return a.prologue != PCS_PRO_RAW || !a.a_mask;
}

int pcs_gemm_stream_launch(const pcs_gemm_args &a, int64_t rows_per_chunk, hipStream_t s) {
  (void)stream_shape(a);
  return launch_shape<64, 512, 64>(a, rows_per_chunk, s);
}

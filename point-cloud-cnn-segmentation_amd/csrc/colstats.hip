// Streaming per-chunk column statistics of a stored points-major activation Y [M, C]:
// BatchNorm batch statistics (per-thread Welford, Chan-merged per chunk) and, optionally,
// the global max-pool candidates (max/min and their first row) of P:113-114.  One HBM
// pass at full bandwidth replaces the cross-lane reductions a wide GEMM epilogue would
// need (those cost ~1/3 of the global_feat forward GEMM when fused).  Output formats are
// those of pcs_gemm's epilogue, so pcs_bn_fwd_finalize / pcs_pool_finalize consume them.
#include "common.h"

namespace {

constexpr int THREADS = 256;

template <typename T, bool POOL>
__global__ __launch_bounds__(THREADS) void colstats_kernel(const T *__restrict__ Y, int64_t N, int C,
                                                           int cps, int64_t rows_per_chunk, float *stats,
                                                           float *pool) {
  constexpr int EPC = Elem<T>::EPC;
  __shared__ float4 red[THREADS];
  const int cpr = C / EPC;                 // chunks per row
  const int rpp = THREADS / cpr;           // rows per pass (cpr <= THREADS, THREADS % cpr == 0)
  const int tid = threadIdx.x, cc = tid % cpr, r0 = tid / cpr;
  const int chunk = blockIdx.x, scene = chunk / cps, cis = chunk % cps;
  const int64_t lo = (int64_t)cis * rows_per_chunk;
  const int64_t hi = pcs_min64(lo + rows_per_chunk, N);
  float mean[EPC], m2[EPC], cnt = 0.f, mx[EPC], mn[EPC];
  int mxi[EPC], mni[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    mean[e] = 0.f; m2[e] = 0.f;
    mx[e] = -__builtin_huge_valf(); mn[e] = __builtin_huge_valf();
    mxi[e] = 0x7fffffff; mni[e] = 0x7fffffff;
  }
  const T *base = Y + scene * N * C + cc * EPC;
#pragma unroll 4
  for (int64_t r = lo + r0; r < hi; r += rpp) {
    float v[EPC];
    unpack_chunk(*reinterpret_cast<const u32x4 *>(base + r * C), v);
    cnt += 1.f;
    const float rn = 1.f / cnt;
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const float d = v[e] - mean[e];
      mean[e] = fmaf(d, rn, mean[e]);
      m2[e] = fmaf(d, v[e] - mean[e], m2[e]);
      if constexpr (POOL) {
        const int g = (int)(scene * N + r);
        if (pool_max_step(v[e], mx[e], mxi[e])) { mx[e] = v[e]; mxi[e] = g; }   // rows ascend: first max kept
        if (pool_min_step(v[e], mn[e], mni[e])) { mn[e] = v[e]; mni[e] = g; }
      }
    }
  }
  // merge the rpp threads that share a column chunk, one column at a time per pass
  for (int e = 0; e < EPC; ++e) {
    if (stats) {
    red[tid] = make_float4(cnt, mean[e], m2[e], 0.f);
    __syncthreads();
    if (r0 == 0) {
      float n = 0.f, mu = 0.f, q = 0.f;
      for (int j = 0; j < rpp; ++j) {
        const float4 p = red[j * cpr + cc];
        chan_merge(n, mu, q, p.x, p.y, p.z);
      }
      *reinterpret_cast<float2 *>(stats + ((int64_t)chunk * C + cc * EPC + e) * 2) = make_float2(mu, q);
    }
    __syncthreads();
    }
    if constexpr (POOL) {
      red[tid] = make_float4(mx[e], __int_as_float(mxi[e]), mn[e], __int_as_float(mni[e]));
      __syncthreads();
      if (r0 == 0) {
        float a = -__builtin_huge_valf(), b = __builtin_huge_valf();
        int ai = 0x7fffffff, bi = 0x7fffffff;
        for (int j = 0; j < rpp; ++j) {
          const float4 p = red[j * cpr + cc];
          const int pi = __float_as_int(p.y), pj = __float_as_int(p.w);
          if (pool_max_wins(p.x, pi, a, ai)) { a = p.x; ai = pi; }
          if (pool_min_wins(p.z, pj, b, bi)) { b = p.z; bi = pj; }
        }
        *reinterpret_cast<float4 *>(pool + ((int64_t)chunk * C + cc * EPC + e) * 4) =
            make_float4(a, __int_as_float(ai), b, __int_as_float(bi));
      }
      __syncthreads();
    }
  }
}

}  // namespace

extern "C" int64_t pcs_colstats_geometry(int64_t num_scenes, int64_t scene_rows, int32_t C,
                                         int32_t *chunks_per_scene) {
  if (!chunks_per_scene || num_scenes <= 0 || scene_rows <= 0 || C <= 0)
    return pcs_set_einval("pcs_colstats_geometry", "bad arguments");
  pcs_gemm_args g{};
  g.num_scenes = num_scenes;
  g.scene_rows = scene_rows;
  g.chunks_per_scene = *chunks_per_scene;
  const int64_t rpc = pcs_fill_geometry(&g, 64, 4096, 1);   // ~16 blocks per CU
  *chunks_per_scene = g.chunks_per_scene;
  return rpc;
}

extern "C" int pcs_colstats(const void *Y, int64_t num_scenes, int64_t scene_rows, int32_t C, int32_t dtype,
                            int32_t chunks_per_scene, int64_t rows_per_chunk, float *stats, float *pool,
                            pcs_stream_t stream) {
  const int epc = dtype == PCS_BF16 ? 8 : 4;
  if (!Y || !(stats || pool) || C % epc || C / epc > THREADS || THREADS % (C / epc) || chunks_per_scene <= 0 ||
      rows_per_chunk <= 0)
    return pcs_set_einval("pcs_colstats", "bad arguments (C/epc must divide 256)");
  const int nb = (int)(num_scenes * chunks_per_scene);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define PCS_CS(T, P)                                                                                   \
  hipLaunchKernelGGL((colstats_kernel<T, P>), dim3(nb), dim3(THREADS), 0, s,                          \
                     reinterpret_cast<const T *>(Y), scene_rows, (int)C, (int)chunks_per_scene,       \
                     rows_per_chunk, stats, pool)
  if (dtype == PCS_BF16) { if (pool) PCS_CS(bf16_t, true); else PCS_CS(bf16_t, false); }
  else if (dtype == PCS_F32) { if (pool) PCS_CS(float, true); else PCS_CS(float, false); }
  else return pcs_set_einval("pcs_colstats", "bad dtype");
#undef PCS_CS
  PCS_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// Streaming BN_{l-1} backward input stage, in place on a raw dgrad output:
//   v = dA (+ addend) (* keep * keep_scale);  dz = (Yp*s + t > 0) ? v : 0;  store dz;
//   per-chunk S1 = sum dz, S2 = sum dz * (Yp - mean) * rstd.
// (the EPI_DGRAD epilogue of pcs_gemm as a separate HBM pass, for the wide layer)
// ---------------------------------------------------------------------------------------
namespace {
template <typename T>
__global__ __launch_bounds__(THREADS) void bnrelu_bwd_kernel(T *__restrict__ D, const T *__restrict__ Yp,
                                                             const T *__restrict__ addend, const uint8_t *mask,
                                                             float keep_scale, const float *es, const float *et,
                                                             const float *em, const float *er, int64_t N, int C,
                                                             int cps, int64_t rows_per_chunk, float *stats) {
  constexpr int EPC = Elem<T>::EPC;
  __shared__ float2 red[THREADS];
  const int cpr = C / EPC, rpp = THREADS / cpr;
  const int tid = threadIdx.x, cc = tid % cpr, r0 = tid / cpr, c0 = cc * EPC;
  const int chunk = blockIdx.x, scene = chunk / cps, cis = chunk % cps;
  const int64_t lo = (int64_t)cis * rows_per_chunk;
  const int64_t hi = pcs_min64(lo + rows_per_chunk, N);
  float s[EPC], t[EPC], mu[EPC], rs[EPC], s1[EPC], s2[EPC];
  load_vec<EPC>(es, c0, s); load_vec<EPC>(et, c0, t);
  load_vec<EPC>(em, c0, mu); load_vec<EPC>(er, c0, rs);
#pragma unroll
  for (int e = 0; e < EPC; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
#pragma unroll 4
  for (int64_t r = lo + r0; r < hi; r += rpp) {
    const int64_t row = scene * N + r;
    const int64_t off = row * C + c0;
    float v[EPC], y[EPC];
    unpack_chunk(*reinterpret_cast<const u32x4 *>(D + off), v);
    unpack_chunk(*reinterpret_cast<const u32x4 *>(Yp + off), y);
    if (addend) {
      float ad[EPC];
      unpack_chunk(*reinterpret_cast<const u32x4 *>(addend + off), ad);
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] += ad[e];
    }
    if (mask) {
      const uint32_t bits = mask_bits(mask, row, C, c0, EPC);
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] *= ((bits >> e) & 1u) ? keep_scale : 0.f;
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const float dz = fmaf(y[e], s[e], t[e]) > 0.f ? v[e] : 0.f;
      v[e] = dz;
      s1[e] += dz;
      s2[e] = fmaf(dz, (y[e] - mu[e]) * rs[e], s2[e]);
    }
    *reinterpret_cast<u32x4 *>(D + off) = pack_chunk(v);
  }
  for (int e = 0; e < EPC; ++e) {
    red[tid] = make_float2(s1[e], s2[e]);
    __syncthreads();
    if (r0 == 0) {
      float a1 = 0.f, a2 = 0.f;
      for (int j = 0; j < rpp; ++j) { a1 += red[j * cpr + cc].x; a2 += red[j * cpr + cc].y; }
      *reinterpret_cast<float2 *>(stats + ((int64_t)chunk * C + c0 + e) * 2) = make_float2(a1, a2);
    }
    __syncthreads();
  }
}
}  // namespace

extern "C" int pcs_bnrelu_bwd(void *D, const void *Yp, const void *addend, const uint8_t *mask,
                              float keep_scale, const float *s, const float *t, const float *mean,
                              const float *rstd, int64_t num_scenes, int64_t scene_rows, int32_t C,
                              int32_t dtype, int32_t chunks_per_scene, int64_t rows_per_chunk, float *stats,
                              pcs_stream_t stream) {
  const int epc = dtype == PCS_BF16 ? 8 : 4;
  if (!D || !Yp || !s || !t || !mean || !rstd || !stats || C % epc || C / epc > THREADS ||
      THREADS % (C / epc) || chunks_per_scene <= 0 || rows_per_chunk <= 0)
    return pcs_set_einval("pcs_bnrelu_bwd", "bad arguments");
  const int nb = (int)(num_scenes * chunks_per_scene);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == PCS_BF16)
    hipLaunchKernelGGL(bnrelu_bwd_kernel<bf16_t>, dim3(nb), dim3(THREADS), 0, st, reinterpret_cast<bf16_t *>(D),
                       reinterpret_cast<const bf16_t *>(Yp), reinterpret_cast<const bf16_t *>(addend), mask,
                       keep_scale, s, t, mean, rstd, scene_rows, (int)C, (int)chunks_per_scene, rows_per_chunk,
                       stats);
  else if (dtype == PCS_F32)
    hipLaunchKernelGGL(bnrelu_bwd_kernel<float>, dim3(nb), dim3(THREADS), 0, st, reinterpret_cast<float *>(D),
                       reinterpret_cast<const float *>(Yp), reinterpret_cast<const float *>(addend), mask,
                       keep_scale, s, t, mean, rstd, scene_rows, (int)C, (int)chunks_per_scene, rows_per_chunk,
                       stats);
  else return pcs_set_einval("pcs_bnrelu_bwd", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

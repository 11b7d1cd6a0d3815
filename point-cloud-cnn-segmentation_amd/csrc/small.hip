// Small / bandwidth-light kernels of the PointNetSegmentation training step:
// conv1 (Cin = 4) forward and weight gradient, BatchNorm statistic finalisation (forward
// and backward), the global max-pool finalisation and its backward, the per-scene GEMV of
// seg_conv1's global half, dropout keep bits (Philox4x32-7), the CE weight sum, fp32
// partial reduction, weight casting and the fused Adam step.
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int C1_BM = 128;  // conv1 row tile (same chunk geometry rules as pcs_gemm)

// ---------------------------------------------------------------------------------------
// conv1 forward: y[m, c] = b[c] + sum_k W[c,k] x[m,k]  (P:70, P:106), K = input_dim
// (KD = 1..8; 4 for the reference's x, y, z, e), fp32 math
// ---------------------------------------------------------------------------------------
// one input row x[m, 0..KD) into registers (one 16-B load for the reference's KD = 4)
template <int KD>
PCS_DEV void load_xrow(const float *X, int64_t row, float (&x)[KD]) {
  if constexpr (KD == 4) {
    const float4 v = *reinterpret_cast<const float4 *>(X + row * 4);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else {
#pragma unroll
    for (int k = 0; k < KD; ++k) x[k] = X[row * KD + k];
  }
}

template <typename T, int KD>
__global__ __launch_bounds__(THREADS) void conv1_fwd_kernel(pcs_gemm_args a, int tiles_per_scene,
                                                            int tiles_per_chunk) {
  constexpr int EPC = Elem<T>::EPC;
  constexpr int COLS = 64;
  constexpr int CPR = COLS / EPC;
  constexpr int RPP = THREADS / CPR;
  __shared__ float4 red[RPP * COLS];
  const int tid = threadIdx.x;
  const int cps = a.chunks_per_scene;
  const int scene = blockIdx.x / cps, cis = blockIdx.x % cps;
  const int64_t N = a.scene_rows;
  const int cc = tid % CPR, r0 = tid / CPR, c0 = cc * EPC;
  const float *X = reinterpret_cast<const float *>(a.A);
  const float *W = reinterpret_cast<const float *>(a.W);
  T *Cg = reinterpret_cast<T *>(a.C);
  float w[EPC][KD], bias[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    bias[e] = a.bias ? a.bias[c0 + e] : 0.f;
#pragma unroll
    for (int k = 0; k < KD; ++k) w[e][k] = W[(c0 + e) * KD + k];
  }
  float mean[EPC], m2[EPC], cnt = 0.f;
#pragma unroll
  for (int e = 0; e < EPC; ++e) { mean[e] = 0.f; m2[e] = 0.f; }
  const int64_t r_begin = (int64_t)cis * tiles_per_chunk * C1_BM;
  const int64_t r_end = pcs_min64(r_begin + (int64_t)tiles_per_chunk * C1_BM, N);
  // four rows per thread per pass: their input loads are issued together (one dependent load
  // -> compute -> store chain per row left the kernel waiting on memory 80 % of its cycles);
  // the rows are still folded into the statistics in the same order
  constexpr int U = 4;
  for (int64_t r = r_begin + r0; r < r_end; r += U * RPP) {
    float x[U][KD];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (r + u * RPP < r_end) load_xrow<KD>(X, scene * N + r + u * RPP, x[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r + u * RPP >= r_end) break;
      const int64_t grow = scene * N + r + u * RPP;
      float v[EPC];
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        float acc = bias[e];
#pragma unroll
        for (int k = 0; k < KD; ++k) acc = fmaf(w[e][k], x[u][k], acc);
        v[e] = acc;
      }
      const u32x4 packed = pack_chunk(v);
      st16(Cg + grow * COLS + c0, packed);
      unpack_chunk(packed, v);  // statistics of the stored (rounded) values
      cnt += 1.f;
      const float rn = 1.f / cnt;
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        const float d = v[e] - mean[e];
        mean[e] = fmaf(d, rn, mean[e]);
        m2[e] = fmaf(d, v[e] - mean[e], m2[e]);
      }
    }
  }
  if (!a.stats) return;
#pragma unroll
  for (int e = 0; e < EPC; ++e) red[r0 * COLS + c0 + e] = make_float4(cnt, mean[e], m2[e], 0.f);
  __syncthreads();
  if (tid < COLS) {
    float n = 0.f, mu = 0.f, q = 0.f;
    for (int j = 0; j < RPP; ++j) {
      const float4 p = red[j * COLS + tid];
      chan_merge(n, mu, q, p.x, p.y, p.z);
    }
    *reinterpret_cast<float2 *>(a.stats + ((int64_t)blockIdx.x * COLS + tid) * 2) = make_float2(mu, q);
  }
}

// ---------------------------------------------------------------------------------------
// conv1 weight gradient: dW[c,k] = sum_m dy[m,c] x[m,k]; dy = alpha dz + beta + gamma y
// ---------------------------------------------------------------------------------------
template <typename T, int KD>
__global__ __launch_bounds__(THREADS) void conv1_wgrad_kernel(pcs_wgrad_args a, int64_t rows_per_split) {
  constexpr int EPC = Elem<T>::EPC;
  constexpr int COLS = 64;
  constexpr int CPR = COLS / EPC;
  constexpr int RPP = THREADS / CPR;
  __shared__ float red[RPP][COLS * KD];
  const int tid = threadIdx.x;
  const int sps = a.splits_per_scene;
  const int scene = blockIdx.x / sps, sis = blockIdx.x % sps;
  const int64_t N = a.scene_rows;
  const int cc = tid % CPR, r0 = tid / CPR, c0 = cc * EPC;
  const T *dZ = reinterpret_cast<const T *>(a.dZ);
  const T *Y = reinterpret_cast<const T *>(a.Y);
  const float *X = reinterpret_cast<const float *>(a.X);
  float ca[EPC], cb[EPC], cg[EPC];
  load_vec<EPC>(a.alpha, c0, ca); load_vec<EPC>(a.beta, c0, cb); load_vec<EPC>(a.gamma, c0, cg);
  float acc[EPC][KD];
#pragma unroll
  for (int e = 0; e < EPC; ++e)
#pragma unroll
    for (int k = 0; k < KD; ++k) acc[e][k] = 0.f;
  const int64_t lo = (int64_t)sis * rows_per_split, hi = pcs_min64(lo + rows_per_split, N);
  // four rows per thread per pass, their loads issued together (one row's dependent
  // load -> FMA chain at a time kept the kernel waiting on memory 90 % of its cycles)
  constexpr int U = 4;
  for (int64_t r = lo + r0; r < hi; r += U * RPP) {
    u32x4 dzr[U], yr[U];
    float x[U][KD];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t grow = scene * N + pcs_min64(r + u * RPP, hi - 1);   // (clamped; skipped below)
      dzr[u] = *reinterpret_cast<const u32x4 *>(dZ + grow * COLS + c0);
      yr[u] = *reinterpret_cast<const u32x4 *>(Y + grow * COLS + c0);
      load_xrow<KD>(X, grow, x[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r + u * RPP >= hi) break;
      float dz[EPC], y[EPC];
      unpack_chunk(dzr[u], dz);
      unpack_chunk(yr[u], y);
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        const float dy = fmaf(ca[e], dz[e], fmaf(cg[e], y[e], cb[e]));
#pragma unroll
        for (int k = 0; k < KD; ++k) acc[e][k] = fmaf(dy, x[u][k], acc[e][k]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPC; ++e)
#pragma unroll
    for (int k = 0; k < KD; ++k) red[r0][(c0 + e) * KD + k] = acc[e][k];
  __syncthreads();
  for (int i = tid; i < COLS * KD; i += THREADS) {
    float s = 0.f;
    for (int j = 0; j < RPP; ++j) s += red[j][i];
    a.partial[(int64_t)blockIdx.x * COLS * KD + i] = s;
  }
}

// ---------------------------------------------------------------------------------------
// BatchNorm statistics
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void bn_fwd_finalize_kernel(
    const float *stats, int64_t B, int64_t N, int C, int cps, int64_t rpc, const float *gamma,
    const float *beta, const float *moff, float *rmean, float *rvar, float momentum, float eps, int update,
    float *mean_o, float *rstd_o, float *scale_o, float *shift_o, float *scene_sum) {
  __shared__ double sh[THREADS][3];
  const int c = blockIdx.x, tid = threadIdx.x;
  double gn = 0, gmean = 0, gm2 = 0;
  for (int64_t b = 0; b < B; ++b) {
    double n = 0, mu = 0, q = 0;
    for (int j = tid; j < cps; j += THREADS) {
      const double nb = (double)pcs_min64(rpc, N - (int64_t)j * rpc);
      const float2 p = *reinterpret_cast<const float2 *>(stats + ((b * cps + j) * C + c) * 2);
      const double nn = n + nb, d = (double)p.x - mu;
      mu += d * nb / nn;
      q += (double)p.y + d * d * n * nb / nn;
      n = nn;
    }
    sh[tid][0] = n; sh[tid][1] = mu; sh[tid][2] = q;
    __syncthreads();
    for (int s = THREADS / 2; s > 0; s >>= 1) {
      if (tid < s) {
        const double na = sh[tid][0], nb = sh[tid + s][0];
        if (nb > 0) {
          const double nn = na + nb, d = sh[tid + s][1] - sh[tid][1];
          sh[tid][1] += d * nb / nn;
          sh[tid][2] += sh[tid + s][2] + d * d * na * nb / nn;
          sh[tid][0] = nn;
        }
      }
      __syncthreads();
    }
    if (tid == 0) {
      const double nb = sh[0][0], mb = sh[0][1], qb = sh[0][2];
      if (scene_sum) scene_sum[b * C + c] = (float)(nb * mb);
      const double nn = gn + nb, d = mb - gmean;
      gmean += d * nb / nn;
      gm2 += qb + d * d * gn * nb / nn;
      gn = nn;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const double var = gm2 / gn;  // biased (normalisation)
    const double rstd = 1.0 / sqrt(var + (double)eps);
    const double sc = (double)gamma[c] * rstd;
    mean_o[c] = (float)gmean;
    rstd_o[c] = (float)rstd;
    scale_o[c] = (float)sc;
    shift_o[c] = (float)((double)beta[c] - gmean * sc);
    if (update) {
      const double unb = gn > 1 ? gm2 / (gn - 1) : gm2;
      const double tm = gmean + (moff ? (double)moff[c] : 0.0);
      rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * tm);
      rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
    }
  }
}

__global__ void bn_eval_kernel(const float *gamma, const float *beta, const float *rm,
                               const float *rv, const float *moff, float eps, int C, float *scale,
                               float *shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double sc = (double)gamma[c] / sqrt((double)rv[c] + (double)eps);
  scale[c] = (float)sc;
  shift[c] = (float)((double)beta[c] - ((double)rm[c] - (moff ? (double)moff[c] : 0.0)) * sc);
}

__global__ __launch_bounds__(THREADS) void bn_bwd_finalize_kernel(
    const float *stats, int64_t B, int64_t N, int C, int cps, const float *mean, const float *rstd,
    const float *gamma, const float *scene_sum, float *alpha, float *beta_c, float *gamma_c,
    float *dgamma, float *dbeta, float *dbias, float *scene_s1) {
  __shared__ double sh[THREADS][2];
  const int c = blockIdx.x, tid = threadIdx.x;
  double S1 = 0, S2 = 0, Sy = 0;
  for (int64_t b = 0; b < B; ++b) {
    double s1 = 0, s2 = 0;
    for (int j = tid; j < cps; j += THREADS) {
      const float2 p = *reinterpret_cast<const float2 *>(stats + ((b * cps + j) * C + c) * 2);
      s1 += p.x; s2 += p.y;
    }
    sh[tid][0] = s1; sh[tid][1] = s2;
    __syncthreads();
    for (int s = THREADS / 2; s > 0; s >>= 1) {
      if (tid < s) { sh[tid][0] += sh[tid + s][0]; sh[tid][1] += sh[tid + s][1]; }
      __syncthreads();
    }
    if (tid == 0) {
      if (scene_s1) scene_s1[b * C + c] = (float)sh[0][0];
      S1 += sh[0][0]; S2 += sh[0][1];
      if (scene_sum) Sy += scene_sum[b * C + c];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const double M = (double)(B * N);
    const double r = rstd[c], g = gamma[c], mu = mean[c];
    const double al = g * r;
    const double ga = -g * r * r * S2 / M;
    const double be = -g * r * S1 / M - ga * mu;
    alpha[c] = (float)al; gamma_c[c] = (float)ga; beta_c[c] = (float)be;
    if (dgamma) dgamma[c] = (float)S2;
    if (dbeta) dbeta[c] = (float)S1;
    if (dbias) dbias[c] = scene_sum ? (float)(al * S1 + M * be + ga * Sy) : 0.f;
  }
}

// ---------------------------------------------------------------------------------------
// global max-pool (P:114) finalisation and backward
// ---------------------------------------------------------------------------------------
__global__ void pool_finalize_kernel(const float *pool, int64_t B, int64_t N, int C, int cps,
                                     const float *s, const float *t, float *g, int32_t *am,
                                     float *ysel) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = (int)(i / C), c = (int)(i % C);
  float mx = -__builtin_huge_valf(), mn = __builtin_huge_valf();
  int mxi = 0x7fffffff, mni = 0x7fffffff;
  for (int j = 0; j < cps; ++j) {
    const float4 q = *reinterpret_cast<const float4 *>(pool + (((int64_t)b * cps + j) * C + c) * 4);
    const int qi = __float_as_int(q.y), qj = __float_as_int(q.w);
    if (pool_max_wins(q.x, qi, mx, mxi)) { mx = q.x; mxi = qi; }
    if (pool_min_wins(q.z, qj, mn, mni)) { mn = q.z; mni = qj; }
  }
  const float sc = s[c];
  float y; int idx;
  if (sc > 0.f) { y = mx; idx = mxi; }
  else if (sc < 0.f) { y = mn; idx = mni; }
  else { y = mx; idx = (int)(b * N); }  // constant z (or a NaN scale): torch's first index
  // never hand on the "no candidate" sentinel (or any row outside the scene) as a row index:
  // the backward's pool kernels read the row it names
  if ((int64_t)idx < b * N || (int64_t)idx >= (b + 1) * N) idx = (int)(b * N);
  const float z = fmaf(y, sc, t[c]);
  g[i] = (z > 0.f || z != z) ? z : 0.f;   // ReLU that keeps a NaN, as torch.relu does
  am[i] = idx;
  ysel[i] = y;
}

__global__ void scene_gemv_kernel(const float *g, int64_t B, int Kg, const float *W, int64_t ldw,
                                  int col_off, const float *bias, int Nout, float *out,
                                  float *offset) {
  // one wave per output channel n, looping over the scenes
  const int n = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (n >= Nout) return;
  const float *w = W + (int64_t)n * ldw + col_off;
  const float bn = bias ? bias[n] : 0.f;
  double mean = 0.0;
  for (int64_t b = 0; b < B; ++b) {
    const float *x = g + b * Kg;
    float acc = 0.f;
    for (int k = lane; k < Kg; k += 64) acc = fmaf(w[k], x[k], acc);
    acc = wave_sum(acc) + bn;
    mean += acc;
    if (lane == 0) out[b * Nout + n] = acc;
  }
  if (!offset) return;
  const float m = (float)(mean / (double)B);
  if (lane == 0) {
    for (int64_t b = 0; b < B; ++b) out[b * Nout + n] -= m;
    offset[n] = m;
  }
}

// csum[b,n] = sum over the rows of scene b of dy_seg1[:, n]
__global__ void pool_bwd_csum_kernel(pcs_pool_bwd_args a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.num_scenes * a.Cs) return;
  const int n = (int)(i % a.Cs);
  a.csum[i] = a.s1_alpha[n] * a.s1_scene_s1[i] + (float)a.scene_rows * a.s1_beta[n] +
              a.s1_gamma[n] * a.s1_scene_sum[i];
}

// dW_seg1[n, off+k] = sum_b csum[b,n] g[b,k]
__global__ void pool_bwd_dw_kernel(pcs_pool_bwd_args a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.Cs * a.Cg) return;
  const int n = (int)(i / a.Cg), k = (int)(i % a.Cg);
  float acc = 0.f;
  for (int64_t b = 0; b < a.num_scenes; ++b) acc = fmaf(a.csum[b * a.Cs + n], a.g[b * a.Cg + k], acc);
  a.dW_s1_global[(int64_t)n * a.ldw + a.col_off + k] = acc;
}

// dg = W_g^T csum; dz_g = dg*(g>0); bn_global backward from the B sparse entries.
// Block: 64 channels k x 4 parts of the n reduction (fixed-order combine through LDS).
constexpr int PBC_MAXB = 64;
// 16 parts of seg_conv1's 512 rows per column (1024 threads), 8 scenes per pass: each W entry is
// loaded once per pass and feeds 8 accumulators (was 4 parts, one scene at a time: a 512-long
// dependent load chain per thread on 16 workgroups)
constexpr int PBC_PARTS = 16, PBC_SB = 8;
__global__ __launch_bounds__(1024) void pool_bwd_coef_kernel(pcs_pool_bwd_args a) {
  __shared__ float part[PBC_PARTS][PBC_SB][64];
  __shared__ float dgall[PBC_MAXB][64];
  const int kk = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + kk;
  const int B = (int)a.num_scenes;
  const int n0 = (int)((int64_t)a.Cs * pr / PBC_PARTS), n1 = (int)((int64_t)a.Cs * (pr + 1) / PBC_PARTS);
  for (int b0 = 0; b0 < B; b0 += PBC_SB) {
    float dg[PBC_SB];
#pragma unroll
    for (int u = 0; u < PBC_SB; ++u) dg[u] = 0.f;
    if (k < a.Cg) {
      for (int n = n0; n < n1; ++n) {
        const float w = a.W_s1[(int64_t)n * a.ldw + a.col_off + k];
#pragma unroll
        for (int u = 0; u < PBC_SB; ++u)
          if (b0 + u < B) dg[u] = fmaf(w, a.csum[(int64_t)(b0 + u) * a.Cs + n], dg[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < PBC_SB; ++u) part[pr][u][kk] = dg[u];
    __syncthreads();
    if (pr == 0) {
      for (int u = 0; u < PBC_SB && b0 + u < B; ++u) {
        float t = 0.f;
        for (int q = 0; q < PBC_PARTS; ++q) t += part[q][u][kk];
        dgall[b0 + u][kk] = t;
      }
    }
    __syncthreads();
  }
  if (pr != 0 || k >= a.Cg) return;
  const double M = (double)(a.num_scenes * a.scene_rows);
  const double r = a.g_rstd[k], gm = a.g_gamma[k], mu = a.g_mean[k];
  double S1 = 0, S2 = 0, Sy = 0;
  for (int b = 0; b < B; ++b) {
    const float dg = dgall[b][kk];
    const float dz = a.g[(int64_t)b * a.Cg + k] > 0.f ? dg : 0.f;
    a.sp[(int64_t)b * a.Cg + k] = dz;  // scaled by alpha below
    S1 += dz;
    S2 += (double)dz * ((double)a.ysel[(int64_t)b * a.Cg + k] - mu) * r;
    Sy += a.g_scene_sum[(int64_t)b * a.Cg + k];
  }
  const double al = gm * r;
  const double ga = -gm * r * r * S2 / M;
  const double be = -gm * r * S1 / M - ga * mu;
  for (int b = 0; b < B; ++b) a.sp[(int64_t)b * a.Cg + k] = (float)(al * a.sp[(int64_t)b * a.Cg + k]);
  a.alpha[k] = (float)al; a.beta_c[k] = (float)be; a.gamma_c[k] = (float)ga;
  a.dgamma[k] = (float)S2; a.dbeta[k] = (float)S1;
  a.dbias[k] = (float)(al * S1 + M * be + ga * Sy);
}

// ---------------------------------------------------------------------------------------
// segmentation head: seg_conv4 (P:128) + weighted CE (P:216,251) + head backward
// ---------------------------------------------------------------------------------------
constexpr int HEAD_R = 64;      // rows per tile
constexpr int HEAD_CIN = 128;
constexpr int HEAD_MAXC = 64;   // classes: <= 16 in the 16-class instantiation (2 WGs / CU), else 64
constexpr int HEAD_LD = HEAD_CIN + 1;

template <typename T, int MODE, int HEAD_MAXC>
__global__ __launch_bounds__(THREADS) void head_kernel(pcs_head_args a, int tiles_per_scene,
                                                       int tiles_per_chunk) {
  constexpr int EPC = Elem<T>::EPC;
  constexpr int QCH = 32;  // channels per thread
  __shared__ float av[HEAD_R * HEAD_LD];
  __shared__ float xh[HEAD_R * HEAD_LD];
  __shared__ float wl[HEAD_MAXC * HEAD_CIN];
  __shared__ float dl[HEAD_R * HEAD_MAXC];
  __shared__ float lred[THREADS / 64];
  const int tid = threadIdx.x;
  const int C = a.num_classes;
  const int cps = a.chunks_per_scene;
  const int scene = blockIdx.x / cps, cis = blockIdx.x % cps;
  const int64_t N = a.scene_rows;
  const int r = tid >> 2, q = tid & 3, ch0 = q * QCH;
  const T *Y = reinterpret_cast<const T *>(a.Y);
  T *dZ = reinterpret_cast<T *>(a.dZ);

  for (int i = tid; i < C * HEAD_CIN; i += THREADS) wl[i] = a.W[i];
  float s1[QCH], s2[QCH];
#pragma unroll
  for (int e = 0; e < QCH; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  constexpr int NPAIR = (HEAD_MAXC * (HEAD_CIN + 1) + THREADS - 1) / THREADS;
  float wacc[NPAIR];
#pragma unroll
  for (int i = 0; i < NPAIR; ++i) wacc[i] = 0.f;
  float loss_acc = 0.f;
  __syncthreads();

  const int t_begin = cis * tiles_per_chunk;
  const int t_end = min(t_begin + tiles_per_chunk, tiles_per_scene);
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int64_t row_base = scene * N + (int64_t)tile * HEAD_R;
    const int valid = (int)pcs_min64(HEAD_R, N - (int64_t)tile * HEAD_R);
    const bool rv = r < valid;
    const int64_t grow = row_base + r;
    // phase 1: load y, a = relu(y*s+t), xhat
    if (rv) {
#pragma unroll
      for (int c = 0; c < QCH; c += EPC) {
        float y[EPC], s[EPC], t[EPC], mu[EPC], rs[EPC];
        unpack_chunk(*reinterpret_cast<const u32x4 *>(Y + grow * HEAD_CIN + ch0 + c), y);
        load_vec<EPC>(a.s, ch0 + c, s); load_vec<EPC>(a.t, ch0 + c, t);
        if constexpr (MODE != PCS_HEAD_FWD) { load_vec<EPC>(a.mean, ch0 + c, mu); load_vec<EPC>(a.rstd, ch0 + c, rs); }
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          av[r * HEAD_LD + ch0 + c + e] = relu(fmaf(y[e], s[e], t[e]));
          if constexpr (MODE != PCS_HEAD_FWD) xh[r * HEAD_LD + ch0 + c + e] = (y[e] - mu[e]) * rs[e];
        }
      }
    }
    __syncthreads();
    // phase 2: logits (quad reduction), CE and dlogits
    {
      float lg[HEAD_MAXC];
#pragma unroll
      for (int c = 0; c < HEAD_MAXC; ++c) {
        float p = 0.f;
        if (c < C && rv) {
          for (int e = 0; e < QCH; ++e) p = fmaf(av[r * HEAD_LD + ch0 + e], wl[c * HEAD_CIN + ch0 + e], p);
        }
        p += __shfl_xor(p, 1);
        p += __shfl_xor(p, 2);
        lg[c] = c < C ? p + a.bias[c] : 0.f;
      }
      if (rv) {
        if (a.logits) {
          for (int c = q; c < C; c += 4) a.logits[grow * C + c] = lg[c];
        }
        if constexpr (MODE == PCS_HEAD_CE) {
          float mx = -__builtin_huge_valf();
#pragma unroll
          for (int c = 0; c < HEAD_MAXC; ++c) if (c < C) mx = fmaxf(mx, lg[c]);
          float se = 0.f;
#pragma unroll
          for (int c = 0; c < HEAD_MAXC; ++c) if (c < C) se += expf(lg[c] - mx);
          const float lse = mx + logf(se);
          const int64_t lab = a.labels[grow];
          const bool ok = lab >= 0 && lab < C;
          const float w = ok ? a.class_weight[lab] : 0.f;
          const float gsc = a.wsum ? 1.f / *a.wsum : 1.f;
          if (q == 0 && ok) {
            float zl = 0.f;
#pragma unroll
            for (int c = 0; c < HEAD_MAXC; ++c) if (c == lab) zl = lg[c];
            loss_acc += w * (lse - zl);
          }
          for (int c = q; c < C; c += 4) {
            const float p = expf(lg[c] - lse);
            dl[r * HEAD_MAXC + c] = ok ? w * gsc * (p - (c == lab ? 1.f : 0.f)) : 0.f;
          }
        } else if constexpr (MODE == PCS_HEAD_BWD) {
          for (int c = q; c < C; c += 4)
            dl[r * HEAD_MAXC + c] = a.dlogits[grow * a.dl_stride_row + c * a.dl_stride_col];
        }
      } else if constexpr (MODE != PCS_HEAD_FWD) {
        for (int c = q; c < C; c += 4) dl[r * HEAD_MAXC + c] = 0.f;
      }
    }
    if constexpr (MODE != PCS_HEAD_FWD) {
      __syncthreads();
      // phase 3: dA = dl W, dz = relu'(z) dA, store, S1/S2
      if (rv) {
#pragma unroll
        for (int c = 0; c < QCH; c += EPC) {
          float v[EPC];
#pragma unroll
          for (int e = 0; e < EPC; ++e) {
            const int ch = ch0 + c + e;
            float d = 0.f;
            for (int k = 0; k < C; ++k) d = fmaf(dl[r * HEAD_MAXC + k], wl[k * HEAD_CIN + ch], d);
            const float dz = av[r * HEAD_LD + ch] > 0.f ? d : 0.f;
            v[e] = dz;
            s1[c + e] += dz;
            s2[c + e] = fmaf(dz, xh[r * HEAD_LD + ch], s2[c + e]);
          }
          st16(dZ + grow * HEAD_CIN + ch0 + c, pack_chunk(v));
        }
      }
      // phase 4: dW / db partials (each weight or bias entry owned by one thread);
      // layout [C*Cin weights | C biases] = flat parameter order of seg_conv4
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        const int p = tid + i * THREADS;
        if (p < C * (HEAD_CIN + 1)) {
          const bool isb = p >= C * HEAD_CIN;
          const int c = isb ? p - C * HEAD_CIN : p / HEAD_CIN, ch = isb ? 0 : p % HEAD_CIN;
          float acc = wacc[i];
          for (int rr = 0; rr < valid; ++rr)
            acc = fmaf(dl[rr * HEAD_MAXC + c], isb ? 1.f : av[rr * HEAD_LD + ch], acc);
          wacc[i] = acc;
        }
      }
    }
    __syncthreads();
  }
  if constexpr (MODE != PCS_HEAD_FWD) {
    if (t_begin >= t_end) return;
    // S1/S2: reduce the 64 row-threads that share a channel quarter
    float *red = av;  // reuse [64][129] x 2 (av, xh contiguous)
#pragma unroll
    for (int e = 0; e < QCH; ++e) {
      av[r * HEAD_LD + ch0 + e] = s1[e];
      xh[r * HEAD_LD + ch0 + e] = s2[e];
    }
    __syncthreads();
    if (tid < HEAD_CIN) {
      float a1 = 0.f, a2 = 0.f;
      for (int j = 0; j < HEAD_R; ++j) { a1 += av[j * HEAD_LD + tid]; a2 += xh[j * HEAD_LD + tid]; }
      *reinterpret_cast<float2 *>(a.stats + ((int64_t)blockIdx.x * HEAD_CIN + tid) * 2) = make_float2(a1, a2);
    }
    (void)red;
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      const int p = tid + i * THREADS;
      if (p < C * (HEAD_CIN + 1)) a.wpartial[(int64_t)blockIdx.x * C * (HEAD_CIN + 1) + p] = wacc[i];
    }
    if constexpr (MODE == PCS_HEAD_CE) {
      const float ls = wave_sum(loss_acc);
      if ((tid & 63) == 0) lred[tid >> 6] = ls;
      __syncthreads();
      if (tid == 0) a.loss_partial[blockIdx.x] = lred[0] + lred[1] + lred[2] + lred[3];
    }
  }
}

// Wide head for 64 < C <= 256 classes (the reference takes any class count, P:83 / P:153).
// 16 rows per tile, 16 threads per row (8 channels each); the whole fp32 W (C x 128) stays in
// LDS.  Each thread keeps the logits of its own classes (c = 16 j + q): max / sum-exp and the
// label's logit come from 16-lane reductions, so no thread holds all C logits.  The dW / db
// partials are register-blocked, 8 classes x 16 channels per thread.  Same arguments, output
// layout and numerics (fp32 accumulation, the same operation order per logit up to the
// reduction tree) as head_kernel.
constexpr int HW_R = 16, HW_TPR = 16, HW_QCH = HEAD_CIN / HW_TPR, HW_MAXC = 256;
constexpr int HW_AL = HEAD_CIN + 4;   // a row stride (floats; 16-B aligned rows)
constexpr int HW_DL = HW_MAXC + 4;    // dl row stride
static_assert(HW_R * HW_TPR == THREADS && HW_QCH == 8, "wide head geometry");

PCS_DEV float grp16_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
PCS_DEV float grp16_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

template <typename T, int MODE>
__global__ __launch_bounds__(THREADS) void head_wide_kernel(pcs_head_args a, int tiles_per_scene,
                                                            int tiles_per_chunk) {
  constexpr int EPC = Elem<T>::EPC;
  constexpr int NJ = HW_MAXC / HW_TPR;   // own classes per thread
  __shared__ __attribute__((aligned(16))) float wl[HW_MAXC * HEAD_CIN];
  __shared__ __attribute__((aligned(16))) float av[HW_R * HW_AL];
  __shared__ __attribute__((aligned(16))) float dl[HW_R * HW_DL];
  __shared__ float lred[THREADS / 64];
  const int tid = threadIdx.x;
  const int C = a.num_classes;
  const int cps = a.chunks_per_scene;
  const int scene = blockIdx.x / cps, cis = blockIdx.x % cps;
  const int64_t N = a.scene_rows;
  const int r = tid / HW_TPR, q = tid % HW_TPR, ch0 = q * HW_QCH;
  const int cbk = tid >> 3, chb = tid & 7;   // dW ownership: classes 8 cbk .., channels 16 chb ..
  const bool own_w = 8 * cbk < C;
  const T *Y = reinterpret_cast<const T *>(a.Y);
  T *dZ = reinterpret_cast<T *>(a.dZ);

  for (int i = tid; i < C * HEAD_CIN; i += THREADS) wl[i] = a.W[i];
  float s1[HW_QCH], s2[HW_QCH];
#pragma unroll
  for (int e = 0; e < HW_QCH; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  float wacc[8][16], bacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    bacc[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) wacc[i][j] = 0.f;
  }
  float loss_acc = 0.f;
  __syncthreads();

  const int t_begin = cis * tiles_per_chunk;
  const int t_end = min(t_begin + tiles_per_chunk, tiles_per_scene);
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int64_t row_base = scene * N + (int64_t)tile * HW_R;
    const int valid = (int)pcs_min64(HW_R, N - (int64_t)tile * HW_R);
    const bool rv = r < valid;
    const int64_t grow = row_base + r;
    // phase 1: a = relu(y s + t) (registers + LDS), xhat (registers)
    float ar[HW_QCH], xr[HW_QCH];
#pragma unroll
    for (int e = 0; e < HW_QCH; ++e) { ar[e] = 0.f; xr[e] = 0.f; }
    if (rv) {
#pragma unroll
      for (int c = 0; c < HW_QCH; c += EPC) {
        float y[EPC], sv[EPC], tv[EPC], mu[EPC], rs[EPC];
        unpack_chunk(*reinterpret_cast<const u32x4 *>(Y + grow * HEAD_CIN + ch0 + c), y);
        load_vec<EPC>(a.s, ch0 + c, sv); load_vec<EPC>(a.t, ch0 + c, tv);
        if constexpr (MODE != PCS_HEAD_FWD) { load_vec<EPC>(a.mean, ch0 + c, mu); load_vec<EPC>(a.rstd, ch0 + c, rs); }
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          ar[c + e] = relu(fmaf(y[e], sv[e], tv[e]));
          if constexpr (MODE != PCS_HEAD_FWD) xr[c + e] = (y[e] - mu[e]) * rs[e];
        }
      }
    }
    *reinterpret_cast<float4 *>(av + r * HW_AL + ch0) = make_float4(ar[0], ar[1], ar[2], ar[3]);
    *reinterpret_cast<float4 *>(av + r * HW_AL + ch0 + 4) = make_float4(ar[4], ar[5], ar[6], ar[7]);
    // phase 2: logits of the thread's own classes c = 16 j + q
    float own[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float v = 0.f;
      if (16 * j < C) {   // block-uniform
        for (int i = 0; i < 16; ++i) {
          const int c = 16 * j + i;
          float p = 0.f;
          if (c < C) {
            const float4 w0 = *reinterpret_cast<const float4 *>(wl + c * HEAD_CIN + ch0);
            const float4 w1 = *reinterpret_cast<const float4 *>(wl + c * HEAD_CIN + ch0 + 4);
            p = fmaf(ar[0], w0.x, p); p = fmaf(ar[1], w0.y, p); p = fmaf(ar[2], w0.z, p); p = fmaf(ar[3], w0.w, p);
            p = fmaf(ar[4], w1.x, p); p = fmaf(ar[5], w1.y, p); p = fmaf(ar[6], w1.z, p); p = fmaf(ar[7], w1.w, p);
          }
          p = grp16_sum(p);
          v = i == q ? p : v;
        }
      }
      const int c = 16 * j + q;
      own[j] = c < C ? v + a.bias[c] : -__builtin_huge_valf();
    }
    if (rv && a.logits) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (16 * j + q < C) a.logits[grow * C + 16 * j + q] = own[j];
    }
    if constexpr (MODE == PCS_HEAD_CE) {
      float mx = -__builtin_huge_valf();
#pragma unroll
      for (int j = 0; j < NJ; ++j) mx = fmaxf(mx, own[j]);
      mx = grp16_max(mx);
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) se += 16 * j + q < C ? expf(own[j] - mx) : 0.f;
      const float lse = mx + logf(grp16_sum(se));
      const int64_t lab = rv ? a.labels[grow] : -1;
      const bool ok = lab >= 0 && lab < C;
      const float w = ok ? a.class_weight[lab] : 0.f;
      const float gsc = a.wsum ? 1.f / *a.wsum : 1.f;
      if (ok && (int)(lab & 15) == q) {
        float zl = 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) zl = j == (int)(lab >> 4) ? own[j] : zl;
        loss_acc += w * (lse - zl);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = 16 * j + q;
        if (c < C) dl[r * HW_DL + c] = ok ? w * gsc * (expf(own[j] - lse) - (c == lab ? 1.f : 0.f)) : 0.f;
      }
    } else if constexpr (MODE == PCS_HEAD_BWD) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = 16 * j + q;
        if (c < C) dl[r * HW_DL + c] = rv ? a.dlogits[grow * a.dl_stride_row + c * a.dl_stride_col] : 0.f;
      }
    }
    if constexpr (MODE != PCS_HEAD_FWD) {
      __syncthreads();
      // phase 3: dA = dl W for the thread's 8 channels, dz = relu'(z) dA, store, S1 / S2
      if (rv) {
        float d[HW_QCH];
#pragma unroll
        for (int e = 0; e < HW_QCH; ++e) d[e] = 0.f;
        for (int k = 0; k < C; ++k) {
          const float dk = dl[r * HW_DL + k];
          const float4 w0 = *reinterpret_cast<const float4 *>(wl + k * HEAD_CIN + ch0);
          const float4 w1 = *reinterpret_cast<const float4 *>(wl + k * HEAD_CIN + ch0 + 4);
          d[0] = fmaf(dk, w0.x, d[0]); d[1] = fmaf(dk, w0.y, d[1]); d[2] = fmaf(dk, w0.z, d[2]); d[3] = fmaf(dk, w0.w, d[3]);
          d[4] = fmaf(dk, w1.x, d[4]); d[5] = fmaf(dk, w1.y, d[5]); d[6] = fmaf(dk, w1.z, d[6]); d[7] = fmaf(dk, w1.w, d[7]);
        }
#pragma unroll
        for (int c = 0; c < HW_QCH; c += EPC) {
          float v[EPC];
#pragma unroll
          for (int e = 0; e < EPC; ++e) {
            const float dz = ar[c + e] > 0.f ? d[c + e] : 0.f;
            v[e] = dz;
            s1[c + e] += dz;
            s2[c + e] = fmaf(dz, xr[c + e], s2[c + e]);
          }
          st16(dZ + grow * HEAD_CIN + ch0 + c, pack_chunk(v));
        }
      }
      // phase 4: dW / db partials over the tile's rows, 8 classes x 16 channels per thread
      if (own_w) {
        for (int rr = 0; rr < valid; ++rr) {
          float dv[8], xv[16];
#pragma unroll
          for (int i = 0; i < 8; ++i) dv[i] = 8 * cbk + i < C ? dl[rr * HW_DL + 8 * cbk + i] : 0.f;
#pragma unroll
          for (int j = 0; j < 16; j += 4) {
            const float4 x4 = *reinterpret_cast<const float4 *>(av + rr * HW_AL + 16 * chb + j);
            xv[j] = x4.x; xv[j + 1] = x4.y; xv[j + 2] = x4.z; xv[j + 3] = x4.w;
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            bacc[i] += dv[i];
#pragma unroll
            for (int j = 0; j < 16; ++j) wacc[i][j] = fmaf(dv[i], xv[j], wacc[i][j]);
          }
        }
      }
    }
    __syncthreads();
  }
  if constexpr (MODE != PCS_HEAD_FWD) {
    if (t_begin >= t_end) return;
    // S1 / S2: reduce the 16 row-threads of each channel (dl reused: [2][16][128])
#pragma unroll
    for (int e = 0; e < HW_QCH; ++e) {
      dl[r * HEAD_CIN + ch0 + e] = s1[e];
      dl[HW_R * HEAD_CIN + r * HEAD_CIN + ch0 + e] = s2[e];
    }
    __syncthreads();
    if (tid < HEAD_CIN) {
      float a1 = 0.f, a2 = 0.f;
      for (int j = 0; j < HW_R; ++j) { a1 += dl[j * HEAD_CIN + tid]; a2 += dl[HW_R * HEAD_CIN + j * HEAD_CIN + tid]; }
      *reinterpret_cast<float2 *>(a.stats + ((int64_t)blockIdx.x * HEAD_CIN + tid) * 2) = make_float2(a1, a2);
    }
    // layout [C * Cin weights | C biases] = flat parameter order of seg_conv4
    float *wp = a.wpartial + (int64_t)blockIdx.x * C * (HEAD_CIN + 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = 8 * cbk + i;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < 16; j += 4)
          *reinterpret_cast<float4 *>(wp + c * HEAD_CIN + 16 * chb + j) =
              make_float4(wacc[i][j], wacc[i][j + 1], wacc[i][j + 2], wacc[i][j + 3]);
        if (chb == 0) wp[C * HEAD_CIN + c] = bacc[i];
      }
    }
    if constexpr (MODE == PCS_HEAD_CE) {
      const float ls = wave_sum(loss_acc);
      if ((tid & 63) == 0) lred[tid >> 6] = ls;
      __syncthreads();
      if (tid == 0) a.loss_partial[blockIdx.x] = lred[0] + lred[1] + lred[2] + lred[3];
    }
  }
}

#ifndef HEAD_BATCH
#define HEAD_BATCH 4
#endif
// Register-resident head for C <= 4 classes: 16 threads per point (one 8-channel bf16 /
// 4-channel fp32 chunk each; 2 chunks per thread for fp32), logits all-reduced across
// those 16 lanes by shuffles, seg_conv4 weights, dW/db partials and bn_seg3 S1/S2 kept
// in registers for the whole chunk, row loads batched.  No LDS in the main loop.
template <typename T, int C, int MODE>
__global__ __launch_bounds__(THREADS) void head_small_kernel(pcs_head_args a, int64_t rows_per_chunk) {
  constexpr int EPC = Elem<T>::EPC;
  constexpr int CPT = 8 / EPC;            // chunks per thread (8 channels per thread)
  constexpr int TPR = HEAD_CIN / 8;       // 16 threads per row
  constexpr int RPP = THREADS / TPR;      // 16 rows per pass
  constexpr int BATCH = HEAD_BATCH;
  __shared__ float red[THREADS];
  const int tid = threadIdx.x, sub = tid % TPR, r0 = tid / TPR, ch0 = sub * 8;
  const int cps = a.chunks_per_scene;
  const int scene = blockIdx.x / cps, cis = blockIdx.x % cps;
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)cis * rows_per_chunk, hi = pcs_min64(lo + rows_per_chunk, N);
  const T *Y = reinterpret_cast<const T *>(a.Y);
  T *dZ = reinterpret_cast<T *>(a.dZ);
  float s[8], t[8], mu[8], rs[8], w[C][8], bias[C];
  load_vec<8>(a.s, ch0, s);
  load_vec<8>(a.t, ch0, t);
  if constexpr (MODE != PCS_HEAD_FWD) { load_vec<8>(a.mean, ch0, mu); load_vec<8>(a.rstd, ch0, rs); }
#pragma unroll
  for (int c = 0; c < C; ++c) { load_vec<8>(a.W + c * HEAD_CIN, ch0, w[c]); bias[c] = a.bias[c]; }
  float s1[8], s2[8], dw[C][8], db[C], lsum = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    db[c] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) dw[c][e] = 0.f;
  }
  const float gsc = (MODE == PCS_HEAD_CE && a.wsum) ? 1.f / *a.wsum : 1.f;
  for (int64_t rb = lo; rb < hi; rb += (int64_t)RPP * BATCH) {
    u32x4 yv[BATCH][CPT];
    int64_t lab[BATCH];
    float dlg[BATCH][C];
#pragma unroll
    for (int q = 0; q < BATCH; ++q) {
      const int64_t r = rb + r0 + RPP * q;
      const int64_t row = scene * N + (r < hi ? r : hi - 1);
#pragma unroll
      for (int k = 0; k < CPT; ++k)
        yv[q][k] = *reinterpret_cast<const u32x4 *>(Y + row * HEAD_CIN + ch0 + k * EPC);
      if constexpr (MODE == PCS_HEAD_CE) lab[q] = a.labels[row];
      if constexpr (MODE == PCS_HEAD_BWD) {
#pragma unroll
        for (int c = 0; c < C; ++c) dlg[q][c] = a.dlogits[row * a.dl_stride_row + c * a.dl_stride_col];
      }
    }
#pragma unroll
    for (int q = 0; q < BATCH; ++q) {
      const int64_t r = rb + r0 + RPP * q;
      const bool ok = r < hi;
      const int64_t row = scene * N + (ok ? r : hi - 1);
      float y[8], av[8];
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        float tmp[EPC];
        unpack_chunk(yv[q][k], tmp);
#pragma unroll
        for (int e = 0; e < EPC; ++e) y[k * EPC + e] = tmp[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = relu(fmaf(y[e], s[e], t[e]));
      float lg[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float p = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) p = fmaf(av[e], w[c][e], p);
#pragma unroll
        for (int o = 1; o < TPR; o <<= 1) p += __shfl_xor(p, o);
        lg[c] = p + bias[c];
      }
      if (ok && a.logits && sub < C) {
#pragma unroll
        for (int c = 0; c < C; ++c)
          if (c == sub) a.logits[row * C + c] = lg[c];
      }
      if constexpr (MODE == PCS_HEAD_FWD) continue;
      float dl[C];
      if constexpr (MODE == PCS_HEAD_CE) {
        float mx = lg[0];
#pragma unroll
        for (int c = 1; c < C; ++c) mx = fmaxf(mx, lg[c]);
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) se += expf(lg[c] - mx);
        const float lse = mx + logf(se);
        const int64_t l = lab[q];
        const bool valid = ok && l >= 0 && l < C;
        const float wt = valid ? a.class_weight[l] : 0.f;
        float zl = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          if (c == l) zl = lg[c];
          dl[c] = valid ? wt * gsc * (expf(lg[c] - lse) - (c == l ? 1.f : 0.f)) : 0.f;
        }
        if (valid && sub == 0) lsum += wt * (lse - zl);
      } else {
#pragma unroll
        for (int c = 0; c < C; ++c) dl[c] = ok ? dlg[q][c] : 0.f;
      }
      float dz[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) d = fmaf(dl[c], w[c][e], d);
        dz[e] = av[e] > 0.f ? d : 0.f;
        s1[e] += dz[e];
        s2[e] = fmaf(dz[e], (y[e] - mu[e]) * rs[e], s2[e]);
#pragma unroll
        for (int c = 0; c < C; ++c) dw[c][e] = fmaf(dl[c], av[e], dw[c][e]);
      }
#pragma unroll
      for (int c = 0; c < C; ++c) db[c] += dl[c];
      if (ok) {
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          float tmp[EPC];
#pragma unroll
          for (int e = 0; e < EPC; ++e) tmp[e] = dz[k * EPC + e];
          st16(dZ + row * HEAD_CIN + ch0 + k * EPC, pack_chunk(tmp));
        }
      }
    }
  }
  if constexpr (MODE != PCS_HEAD_FWD) {
    // reduce over the RPP threads sharing a channel chunk (same `sub`), one value at a time
    const int64_t chunk = blockIdx.x;
    auto reduce_store = [&](float v, float *dst) {
      red[tid] = v;
      __syncthreads();
      if (r0 == 0 && dst) {
        float acc = 0.f;
        for (int j = 0; j < RPP; ++j) acc += red[j * TPR + sub];
        *dst = acc;
      }
      __syncthreads();
    };
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      reduce_store(s1[e], a.stats + (chunk * HEAD_CIN + ch0 + e) * 2);
      reduce_store(s2[e], a.stats + (chunk * HEAD_CIN + ch0 + e) * 2 + 1);
    }
    float *wp = a.wpartial + chunk * (C * HEAD_CIN + C);
#pragma unroll
    for (int c = 0; c < C; ++c) {
#pragma unroll
      for (int e = 0; e < 8; ++e) reduce_store(dw[c][e], wp + c * HEAD_CIN + ch0 + e);
      // every thread of a row holds the same db: sum over rows = over the r0 threads of sub 0
      reduce_store(db[c], sub == 0 ? wp + C * HEAD_CIN + c : nullptr);
    }
    if constexpr (MODE == PCS_HEAD_CE) {
      const float ls = wave_sum(lsum);
      if ((tid & 63) == 0) red[tid >> 6] = ls;
      __syncthreads();
      if (tid == 0) a.loss_partial[chunk] = red[0] + red[1] + red[2] + red[3];
    }
  }
}

// ---------------------------------------------------------------------------------------
// misc
// ---------------------------------------------------------------------------------------
__global__ void ce_count_kernel(const int64_t *labels, int64_t M, int C, unsigned long long *counts) {
  __shared__ unsigned int h[HW_MAXC];
  for (int i = threadIdx.x; i < HW_MAXC; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = labels[i];
    if (l >= 0 && l < C) atomicAdd(&h[l], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += blockDim.x)
    if (h[i]) atomicAdd(&counts[i], (unsigned long long)h[i]);
}

__global__ void ce_wsum_kernel(const unsigned long long *counts, const float *w, int C, float *out) {
  if (threadIdx.x != 0) return;
  double s = 0, n = 0;
  for (int c = 0; c < C; ++c) { s += (double)counts[c] * (double)w[c]; n += (double)counts[c]; }
  out[0] = (float)s;
  out[1] = (float)n;
  out[2] = s > 0 ? (float)(1.0 / s) : 0.f;
}

// Philox4x32-7 (Salmon et al. 2011: 7 rounds already pass BigCrush; the 10-round default's
// margin cost 0.5 ms per step in dropout_bits, which is ALU-bound)
PCS_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // a ^ b ^ c in one v_bitop3_b32
}
PCS_DEV void philox(uint32_t (&ctr)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = xor3(h1, ctr[1], k0), n2 = xor3(h0, ctr[3], k1);
    ctr[0] = n0; ctr[1] = l1; ctr[2] = n2; ctr[3] = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// per 16-bit half of x: 1 where the half is below thr (dropped), at bits 0 and 16
// (one2 = {1, 1} passed opaque: with a known 1 hipcc folds min(sat_sub(.), 1) back into a
// compare + select per half)
PCS_DEV uint32_t drop2(uint32_t x, uint32_t thr2, u16x2 one2) {
  const u16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, thr2), __builtin_bit_cast(u16x2, x));
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(d, one2));
}
__global__ void dropout_bits_kernel(uint64_t seed, uint64_t offset, int64_t nbytes, uint32_t thr,
                                    uint8_t *bits) {
  const uint32_t thr2 = thr | (thr << 16);   // (thr <= 65535: host)
  u16x2 one2 = {1, 1};
  asm volatile("" : "+v"(one2));
  // A thread makes 4 consecutive keep bytes (elements 32 w .. 32 w + 31 of word w) from two
  // Philox calls (counters 2 w, 2 w + 1) and stores them as one word.  Call q's 16 random bytes
  // r0..r15 give 16 elements the 16-bit uniforms (r_e << 8) | r_(e^1): every element keeps with
  // probability exactly 1 - thr / 65536 (two independent bytes), and the two elements that share
  // a byte pair depend on each other only through the low byte (only when one high byte equals
  // thr >> 8).  Random word i's half h (natural, v = 1) and its byte swap (v = 0) go to bit
  // 16 h + 8 q + 2 i + v: the two elements of a pair are adjacent (2k, 2k + 1).  Each
  // v_pk_sub_u16 (clamped) + v_pk_min_u16 turns two uniforms into two drop bits.  Half the
  // Philox calls of one call per byte (the kernel is ALU-bound on the 64-bit multiplies); a grid
  // smaller than the words (pcs_dropout_bits_bounded) strides over them: the bits depend on
  // w only
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; j0 < nbytes; j0 += stride) {
  uint32_t word = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int64_t k = (j0 >> 1) + q;
    uint32_t ctr[4] = {(uint32_t)k, (uint32_t)((uint64_t)k >> 32), (uint32_t)offset, (uint32_t)(offset >> 32)};
    philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t x = ctr[i];
      const uint32_t sw = __builtin_amdgcn_perm(0u, x, 0x02030001u);   // both halves byte-swapped
      word |= drop2(sw, thr2, one2) << (8 * q + 2 * i);
      word |= drop2(x, thr2, one2) << (8 * q + 2 * i + 1);
    }
  }
  word = ~word;   // keep = not dropped
  if (j0 + 4 <= nbytes && ((reinterpret_cast<uintptr_t>(bits) & 3) == 0)) {
    *reinterpret_cast<uint32_t *>(bits + j0) = word;
  } else {
    for (int q = 0; q < 4 && j0 + q < nbytes; ++q) bits[j0 + q] = (uint8_t)(word >> (8 * q));
  }
  }
}

// The independent form (pcs_dropout_bits_independent, opt-in for parity runs): every element
// draws its own 16-bit uniform from its own two Philox bytes, as nn.Dropout's i.i.d. Bernoulli
// draws (P:96), at twice the Philox calls: a thread's word (32 elements) takes four calls,
// counters 4 w .. 4 w + 3, and call q's word i half h is element 8 q + 2 i + h.
__global__ void dropout_bits_indep_kernel(uint64_t seed, uint64_t offset, int64_t nbytes, uint32_t thr,
                                          uint8_t *bits) {
  const uint32_t thr2 = thr | (thr << 16);
  u16x2 one2 = {1, 1};
  asm volatile("" : "+v"(one2));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; j0 < nbytes; j0 += stride) {
    uint32_t word = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t k = j0 + q;   // = 4 w + q
      uint32_t ctr[4] = {(uint32_t)k, (uint32_t)((uint64_t)k >> 32), (uint32_t)offset, (uint32_t)(offset >> 32)};
      philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t d = drop2(ctr[i], thr2, one2);   // bits 0 and 16: halves 0 and 1
        word |= ((d & 1u) | ((d >> 15) & 2u)) << (8 * q + 2 * i);
      }
    }
    word = ~word;
    if (j0 + 4 <= nbytes && ((reinterpret_cast<uintptr_t>(bits) & 3) == 0)) {
      *reinterpret_cast<uint32_t *>(bits + j0) = word;
    } else {
      for (int q = 0; q < 4 && j0 + q < nbytes; ++q) bits[j0 + q] = (uint8_t)(word >> (8 * q));
    }
  }
}

// out = scale * sum over slabs.  TPO threads share one 4-float output (slabs k = sub,
// sub + TPO, ...) and combine with a fixed xor-shuffle tree: deterministic, and wide enough
// for the thousand-slab reductions of the small layers' weight gradients.
template <int TPO>
__global__ void reduce_partials_kernel(const float *partial, int64_t nslabs, int64_t len, float scale,
                                       float *out, int64_t ldo, int64_t row_len) {
  partial += (int64_t)blockIdx.y * nslabs * len;   // grouped form: group y's slabs / outputs
  out += (int64_t)blockIdx.y * len;
  const int sub = threadIdx.x % TPO;
  const int64_t i4 = ((int64_t)blockIdx.x * (blockDim.x / TPO) + threadIdx.x / TPO) * 4;
  const bool vec = (row_len & 3) == 0 && i4 + 4 <= len;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (i4 < len) {
    if (vec) {
      for (int64_t k = sub; k < nslabs; k += TPO) {
        const float4 p = *reinterpret_cast<const float4 *>(partial + k * len + i4);
        v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
      }
    } else {
      for (int64_t k = sub; k < nslabs; k += TPO)
        for (int e = 0; e < 4 && i4 + e < len; ++e) v[e] += partial[k * len + i4 + e];
    }
  }
#pragma unroll
  for (int off = TPO / 2; off > 0; off >>= 1)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += __shfl_xor(v[e], off);
  if (sub != 0 || i4 >= len) return;
  if (vec) {
    const int64_t row = i4 / row_len, col = i4 % row_len;
    *reinterpret_cast<float4 *>(out + row * ldo + col) =
        make_float4(v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale);
  } else {
    for (int e = 0; e < 4 && i4 + e < len; ++e) {
      const int64_t i = i4 + e;
      out[(i / row_len) * ldo + i % row_len] = v[e] * scale;
    }
  }
}

template <typename T>
__global__ void cast_weight_kernel(const float *W, int64_t rows, int64_t cols, int64_t ldw, T *Wc, T *WcT) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const float v = W[(i / cols) * ldw + i % cols];
  T o;
  if constexpr (sizeof(T) == 4) o = v;
  else o = (T)(pack2bf(v, 0.f) & 0xffffu);
  if (Wc) Wc[i] = o;
  if (WcT) WcT[(i % cols) * rows + i / cols] = o;
}

__global__ void adam_kernel(float *p, float *g, float *m, float *v, int64_t n,
                            const float *gscale, float lr, float b1, float b2, float eps, float wd,
                            float bc1, float bc2_sqrt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float pi = p[i];
  float gr = g[i];
  if (gscale) {   // scaled gradient written back: the caller's grad buffer holds dL/dp
    gr *= *gscale;
    g[i] = gr;
  }
  const float gi = gr + wd * pi;
  const float mi = b1 * m[i] + (1.f - b1) * gi;
  const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = pi - (lr / bc1) * (mi / denom);
}

int blocks_for(int64_t n, int per) { return (int)((n + per - 1) / per); }

}  // namespace

// =========================================================================================
// C ABI
// =========================================================================================
static int64_t chunk_geo(int64_t N, int64_t B, int64_t tile, int32_t *cps_io, int64_t target) {
  const int64_t tps = (N + tile - 1) / tile;
  int64_t cps = *cps_io;
  if (cps <= 0) cps = (target + B - 1) / B;
  if (cps > tps) cps = tps;
  if (cps < 1) cps = 1;
  const int64_t tpc = (tps + cps - 1) / cps;
  cps = (tps + tpc - 1) / tpc;
  *cps_io = (int32_t)cps;
  return tpc;
}

namespace {
constexpr int C1_MAXK = 8;   // input_dim 1..8 (the reference's points carry 4: x, y, z, e)
#define PCS_C1_SWITCH(KD_, CALL)                                 \
  switch (KD_) {                                                 \
    case 1: CALL(1); break; case 2: CALL(2); break;              \
    case 3: CALL(3); break; case 4: CALL(4); break;              \
    case 5: CALL(5); break; case 6: CALL(6); break;              \
    case 7: CALL(7); break; default: CALL(8); break;             \
  }
}  // namespace

extern "C" int pcs_conv1_fwd(const pcs_gemm_args *ap, pcs_stream_t stream) {
  if (!ap || !ap->A || !ap->W || !ap->C) return pcs_set_einval("pcs_conv1_fwd", "missing operand");
  if (ap->K < 1 || ap->K > C1_MAXK || ap->Ncols != 64) return pcs_set_einval("pcs_conv1_fwd", "conv1 is input_dim (1..8) -> 64");
  pcs_gemm_args a = *ap;
  const int64_t tpc = pcs_fill_geometry(&a, C1_BM, 2048, 1) / C1_BM;
  const int tps = (int)((a.scene_rows + C1_BM - 1) / C1_BM);
  const int nb = (int)(a.num_scenes * a.chunks_per_scene);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define PCS_C1F_BF(KD) hipLaunchKernelGGL((conv1_fwd_kernel<bf16_t, KD>), dim3(nb), dim3(THREADS), 0, s, a, tps, (int)tpc)
#define PCS_C1F_F32(KD) hipLaunchKernelGGL((conv1_fwd_kernel<float, KD>), dim3(nb), dim3(THREADS), 0, s, a, tps, (int)tpc)
  if (a.dtype == PCS_BF16) { PCS_C1_SWITCH(a.K, PCS_C1F_BF) }
  else if (a.dtype == PCS_F32) { PCS_C1_SWITCH(a.K, PCS_C1F_F32) }
  else return pcs_set_einval("pcs_conv1_fwd", "bad dtype");
#undef PCS_C1F_BF
#undef PCS_C1F_F32
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_conv1_wgrad(const pcs_wgrad_args *ap, pcs_stream_t stream) {
  if (!ap || !ap->dZ || !ap->Y || !ap->X || !ap->partial || !ap->dW)
    return pcs_set_einval("pcs_conv1_wgrad", "missing operand");
  if (ap->Cout != 64 || ap->Cin < 1 || ap->Cin > C1_MAXK)
    return pcs_set_einval("pcs_conv1_wgrad", "conv1 is input_dim (1..8) -> 64");
  pcs_wgrad_args a = *ap;
  if (a.splits_per_scene <= 0) {
    int64_t sps = (1024 + a.num_scenes - 1) / a.num_scenes;
    const int64_t maxs = (a.scene_rows + 255) / 256;
    if (sps > maxs) sps = maxs;
    if (sps < 1) sps = 1;
    a.splits_per_scene = (int32_t)sps;
  }
  const int64_t rps = (a.scene_rows + a.splits_per_scene - 1) / a.splits_per_scene;
  const int nb = (int)(a.num_scenes * a.splits_per_scene);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define PCS_C1W_BF(KD) hipLaunchKernelGGL((conv1_wgrad_kernel<bf16_t, KD>), dim3(nb), dim3(THREADS), 0, s, a, rps)
#define PCS_C1W_F32(KD) hipLaunchKernelGGL((conv1_wgrad_kernel<float, KD>), dim3(nb), dim3(THREADS), 0, s, a, rps)
  if (a.dtype == PCS_BF16) { PCS_C1_SWITCH(a.Cin, PCS_C1W_BF) }
  else if (a.dtype == PCS_F32) { PCS_C1_SWITCH(a.Cin, PCS_C1W_F32) }
  else return pcs_set_einval("pcs_conv1_wgrad", "bad dtype");
#undef PCS_C1W_BF
#undef PCS_C1W_F32
  PCS_CHECK_LAUNCH();
  return pcs_reduce_partials(a.partial, nb, 64 * a.Cin, 1.f, a.dW, a.ldw ? a.ldw : a.Cin, a.Cin, stream);
}
#undef PCS_C1_SWITCH

extern "C" int pcs_bn_fwd_finalize(const float *stats, int64_t B, int64_t N, int32_t C, int32_t cps,
                                   int64_t rpc, const float *gamma, const float *beta,
                                   const float *mean_offset, float *running_mean,
                                   float *running_var, float momentum,
                                   float eps, int32_t update_running, float *mean, float *rstd,
                                   float *scale, float *shift, float *scene_sum,
                                   pcs_stream_t stream) {
  if (!stats || !gamma || !beta || !mean || !rstd || !scale || !shift || C <= 0 || cps <= 0 || rpc <= 0)
    return pcs_set_einval("pcs_bn_fwd_finalize", "bad arguments");
  if (update_running && (!running_mean || !running_var))
    return pcs_set_einval("pcs_bn_fwd_finalize", "running buffers required");
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(C), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     stats, B, N, (int)C, (int)cps, rpc, gamma, beta, mean_offset, running_mean, running_var,
                     momentum, eps, (int)update_running, mean, rstd, scale, shift, scene_sum);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_bn_eval_coefs(const float *gamma, const float *beta, const float *rm,
                                 const float *rv, const float *mean_offset, float eps, int32_t C,
                                 float *scale, float *shift, pcs_stream_t stream) {
  if (!gamma || !beta || !rm || !rv || !scale || !shift) return pcs_set_einval("pcs_bn_eval_coefs", "null");
  hipLaunchKernelGGL(bn_eval_kernel, dim3(blocks_for(C, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), gamma, beta, rm, rv, mean_offset, eps, (int)C, scale, shift);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_bn_bwd_finalize(const float *stats, int64_t B, int64_t N, int32_t C, int32_t cps,
                                   const float *mean, const float *rstd, const float *gamma,
                                   const float *scene_sum, float *alpha, float *beta_c,
                                   float *gamma_c, float *dgamma, float *dbeta, float *dbias,
                                   float *scene_s1, pcs_stream_t stream) {
  if (!stats || !mean || !rstd || !gamma || !alpha || !beta_c || !gamma_c)
    return pcs_set_einval("pcs_bn_bwd_finalize", "null argument");
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     stats, B, N, (int)C, (int)cps, mean, rstd, gamma, scene_sum, alpha, beta_c,
                     gamma_c, dgamma, dbeta, dbias, scene_s1);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_pool_finalize(const float *pool, int64_t B, int64_t N, int32_t C, int32_t cps,
                                 const float *s, const float *t, float *g, int32_t *am, float *ysel,
                                 pcs_stream_t stream) {
  if (!pool || !s || !t || !g || !am || !ysel) return pcs_set_einval("pcs_pool_finalize", "null argument");
  hipLaunchKernelGGL(pool_finalize_kernel, dim3(blocks_for(B * C, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), pool, B, N, (int)C, (int)cps, s, t, g, am, ysel);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_scene_gemv(const float *g, int64_t B, int32_t Kg, const float *W, int64_t ldw,
                              int32_t col_off, const float *bias, int32_t Nout, float *out, float *offset,
                              pcs_stream_t stream) {
  if (!g || !W || !out) return pcs_set_einval("pcs_scene_gemv", "null argument");
  hipLaunchKernelGGL(scene_gemv_kernel, dim3(blocks_for((int64_t)Nout * 64, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), g, B, (int)Kg, W, ldw, (int)col_off, bias,
                     (int)Nout, out, offset);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_pool_bwd(const pcs_pool_bwd_args *ap, pcs_stream_t stream) {
  if (!ap) return pcs_set_einval("pcs_pool_bwd", "null args");
  const pcs_pool_bwd_args &a = *ap;
  if (!a.s1_alpha || !a.s1_beta || !a.s1_gamma || !a.s1_scene_s1 || !a.s1_scene_sum || !a.W_s1 ||
      !a.g || !a.ysel || !a.g_mean || !a.g_rstd || !a.g_gamma || !a.g_scene_sum ||
      !a.dW_s1_global || !a.csum || !a.alpha || !a.beta_c || !a.gamma_c || !a.dgamma || !a.dbeta ||
      !a.dbias || !a.sp)
    return pcs_set_einval("pcs_pool_bwd", "null argument");
  if (a.num_scenes < 1 || a.num_scenes > PBC_MAXB) return pcs_set_einval("pcs_pool_bwd", "1 <= scenes <= 64 per call");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(pool_bwd_csum_kernel, dim3(blocks_for(a.num_scenes * a.Cs, 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(pool_bwd_dw_kernel, dim3(blocks_for((int64_t)a.Cs * a.Cg, 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(pool_bwd_coef_kernel, dim3(blocks_for(a.Cg, 64)), dim3(1024), 0, s, a);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t pcs_head_geometry(pcs_head_args *a) {
  if (!a || a->num_scenes <= 0 || a->scene_rows <= 0) return pcs_set_einval("pcs_head_geometry", "bad geometry");
  if (pcs_head_stream_class(*a)) {   // the streamed CE head (head_stream.hip): 64-row steps
    const int64_t tpc = chunk_geo(a->scene_rows, a->num_scenes, 64, &a->chunks_per_scene,
                                  pcs_head_stream_target());
    return tpc * 64;
  }
  if (a->num_classes <= 4) {   // register-resident kernel: 64-row granules, ~8 WGs per CU
    const int64_t tpc = chunk_geo(a->scene_rows, a->num_scenes, 64, &a->chunks_per_scene, 2048);
    return tpc * 64;
  }
  const int64_t tpc = chunk_geo(a->scene_rows, a->num_scenes, HEAD_R, &a->chunks_per_scene, 2048);
  return tpc * HEAD_R;
}

extern "C" int pcs_head(const pcs_head_args *ap, pcs_stream_t stream) {
  if (!ap) return pcs_set_einval("pcs_head", "null args");
  pcs_head_args a = *ap;
  if (a.Cin != HEAD_CIN) return pcs_set_einval("pcs_head", "head input must have 128 channels");
  if (a.num_classes < 1 || a.num_classes > HW_MAXC) return pcs_set_einval("pcs_head", "1 <= C <= 256");
  if (!a.Y || !a.s || !a.t || !a.W || !a.bias) return pcs_set_einval("pcs_head", "missing operand");
  if (a.mode == PCS_HEAD_CE && (!a.labels || !a.class_weight || !a.loss_partial))
    return pcs_set_einval("pcs_head", "CE mode needs labels, class_weight, loss_partial");
  if (a.mode == PCS_HEAD_BWD && !a.dlogits) return pcs_set_einval("pcs_head", "BWD mode needs dlogits");
  if (a.mode != PCS_HEAD_FWD && (!a.dZ || !a.mean || !a.rstd || !a.stats || !a.wpartial))
    return pcs_set_einval("pcs_head", "backward outputs missing");
  const int64_t rpc = pcs_head_geometry(&a);
  if (rpc < 0) return (int)rpc;
  const int tps = (int)((a.scene_rows + HEAD_R - 1) / HEAD_R);
  const int tpc = (int)(rpc / HEAD_R);
  const int nb = (int)(a.num_scenes * a.chunks_per_scene);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (pcs_head_stream_class(a)) return pcs_head_stream_launch(a, rpc, s);
  if (a.num_classes <= 4) {
#define PCS_HS(T, CC, MODE) \
  hipLaunchKernelGGL((head_small_kernel<T, CC, MODE>), dim3(nb), dim3(THREADS), 0, s, a, rpc)
#define PCS_HS_C(T, MODE)                                                   \
  switch (a.num_classes) {                                                 \
    case 1: PCS_HS(T, 1, MODE); break;                                     \
    case 2: PCS_HS(T, 2, MODE); break;                                     \
    case 3: PCS_HS(T, 3, MODE); break;                                     \
    default: PCS_HS(T, 4, MODE); break;                                    \
  }
#define PCS_HS_M(T)                                                          \
  if (a.mode == PCS_HEAD_FWD) { PCS_HS_C(T, PCS_HEAD_FWD) }                   \
  else if (a.mode == PCS_HEAD_CE) { PCS_HS_C(T, PCS_HEAD_CE) }                \
  else { PCS_HS_C(T, PCS_HEAD_BWD) }
    if (a.dtype == PCS_BF16) { PCS_HS_M(bf16_t) }
    else if (a.dtype == PCS_F32) { PCS_HS_M(float) }
    else return pcs_set_einval("pcs_head", "bad dtype");
#undef PCS_HS_M
#undef PCS_HS_C
#undef PCS_HS
    PCS_CHECK_LAUNCH();
    return 0;
  }
#define PCS_HEAD_LAUNCH(T, MODE)                                                                  \
  do {                                                                                            \
    if (a.num_classes > HEAD_MAXC)                                                                \
      hipLaunchKernelGGL((head_wide_kernel<T, MODE>), dim3(nb), dim3(THREADS), 0, s, a,           \
                         (int)((a.scene_rows + HW_R - 1) / HW_R), (int)(rpc / HW_R));             \
    else if (a.num_classes <= 16)                                                                 \
      hipLaunchKernelGGL((head_kernel<T, MODE, 16>), dim3(nb), dim3(THREADS), 0, s, a, tps, tpc); \
    else                                                                                          \
      hipLaunchKernelGGL((head_kernel<T, MODE, 64>), dim3(nb), dim3(THREADS), 0, s, a, tps, tpc); \
  } while (0)
  if (a.dtype == PCS_BF16) {
    if (a.mode == PCS_HEAD_FWD) PCS_HEAD_LAUNCH(bf16_t, PCS_HEAD_FWD);
    else if (a.mode == PCS_HEAD_CE) PCS_HEAD_LAUNCH(bf16_t, PCS_HEAD_CE);
    else PCS_HEAD_LAUNCH(bf16_t, PCS_HEAD_BWD);
  } else if (a.dtype == PCS_F32) {
    if (a.mode == PCS_HEAD_FWD) PCS_HEAD_LAUNCH(float, PCS_HEAD_FWD);
    else if (a.mode == PCS_HEAD_CE) PCS_HEAD_LAUNCH(float, PCS_HEAD_CE);
    else PCS_HEAD_LAUNCH(float, PCS_HEAD_BWD);
  } else {
    return pcs_set_einval("pcs_head", "bad dtype");
  }
#undef PCS_HEAD_LAUNCH
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_ce_weight_sum(const int64_t *labels, int64_t M, const float *class_weight, int32_t C,
                                 int64_t *counts_ws, float *out, pcs_stream_t stream) {
  if (!labels || !class_weight || !counts_ws || !out || C < 1 || C > HW_MAXC)
    return pcs_set_einval("pcs_ce_weight_sum", "bad arguments");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(counts_ws, 0, sizeof(int64_t) * C, s);
  if (e != hipSuccess) return pcs_set_error(e, "pcs_ce_weight_sum");
  int nb = blocks_for(M, 256);
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(ce_count_kernel, dim3(nb), dim3(256), 0, s, labels, M, (int)C,
                     reinterpret_cast<unsigned long long *>(counts_ws));
  hipLaunchKernelGGL(ce_wsum_kernel, dim3(1), dim3(64), 0, s,
                     reinterpret_cast<const unsigned long long *>(counts_ws), class_weight, (int)C, out);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_dropout_bits_bounded(uint64_t seed, uint64_t offset, int64_t M, int32_t C, float p,
                                        uint8_t *bits, int32_t max_workgroups, pcs_stream_t stream) {
  if (!bits || C % 8 != 0 || p < 0.f || p >= 1.f) return pcs_set_einval("pcs_dropout_bits", "bad arguments");
  const int64_t nbytes = M * (C / 8);
  if (nbytes <= 0) return 0;
  const uint32_t thr = (uint32_t)(p * 65536.0f + 0.5f);
  if (thr > 65535u) {   // every 16-bit uniform is below 65536: nothing kept
    const hipError_t e = hipMemsetAsync(bits, 0, (size_t)nbytes, reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : pcs_set_error(e, "pcs_dropout_bits");
  }
  int64_t nb = blocks_for((nbytes + 3) / 4, 256);
  if (max_workgroups > 0 && nb > max_workgroups) nb = max_workgroups;
  hipLaunchKernelGGL(dropout_bits_kernel, dim3((unsigned)nb), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), seed, offset, nbytes, thr, bits);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_dropout_bits(uint64_t seed, uint64_t offset, int64_t M, int32_t C, float p,
                                uint8_t *bits, pcs_stream_t stream) {
  return pcs_dropout_bits_bounded(seed, offset, M, C, p, bits, 0, stream);
}

extern "C" int pcs_dropout_bits_independent(uint64_t seed, uint64_t offset, int64_t M, int32_t C, float p,
                                            uint8_t *bits, pcs_stream_t stream) {
  if (!bits || C % 8 != 0 || p < 0.f || p >= 1.f)
    return pcs_set_einval("pcs_dropout_bits_independent", "bad arguments");
  const int64_t nbytes = M * (C / 8);
  if (nbytes <= 0) return 0;
  const uint32_t thr = (uint32_t)(p * 65536.0f + 0.5f);
  if (thr > 65535u) {
    const hipError_t e = hipMemsetAsync(bits, 0, (size_t)nbytes, reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : pcs_set_error(e, "pcs_dropout_bits_independent");
  }
  hipLaunchKernelGGL(dropout_bits_indep_kernel, dim3((unsigned)blocks_for((nbytes + 3) / 4, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), seed, offset, nbytes, thr, bits);
  PCS_CHECK_LAUNCH();
  return 0;
}

namespace {
int reduce_partials_launch(const float *partial, int64_t ngroups, int64_t nslabs, int64_t len, float scale,
                           float *out, int64_t ldo, int64_t row_len, hipStream_t st) {
  const int64_t n4 = (len + 3) / 4;
  const dim3 g256(blocks_for(n4, 256 / 32), (unsigned)ngroups), g8(blocks_for(n4, 256 / 8), (unsigned)ngroups),
      g1(blocks_for(n4, 256), (unsigned)ngroups);
  if (nslabs >= 64)
    hipLaunchKernelGGL(reduce_partials_kernel<32>, g256, dim3(256), 0, st, partial, nslabs, len, scale, out, ldo,
                       row_len);
  else if (nslabs >= 8)
    hipLaunchKernelGGL(reduce_partials_kernel<8>, g8, dim3(256), 0, st, partial, nslabs, len, scale, out, ldo, row_len);
  else
    hipLaunchKernelGGL(reduce_partials_kernel<1>, g1, dim3(256), 0, st, partial, nslabs, len, scale, out, ldo, row_len);
  PCS_CHECK_LAUNCH();
  return 0;
}
}  // namespace

extern "C" int pcs_reduce_partials_grouped(const float *partial, int64_t ngroups, int64_t nslabs, int64_t len,
                                           float scale, float *out, pcs_stream_t stream) {
  if (!partial || !out || len <= 0 || nslabs <= 0 || ngroups <= 0 || ngroups > 65535)
    return pcs_set_einval("pcs_reduce_partials_grouped", "bad arguments (0 < ngroups <= 65535)");
  return reduce_partials_launch(partial, ngroups, nslabs, len, scale, out, len, len, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int pcs_reduce_partials(const float *partial, int64_t nslabs, int64_t len, float scale, float *out,
                                   int64_t ldo, int64_t row_len, pcs_stream_t stream) {
  if (!partial || !out || len <= 0 || nslabs <= 0 || row_len <= 0) return pcs_set_einval("pcs_reduce_partials", "bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n4 = (len + 3) / 4;
  if (nslabs >= 64)
    hipLaunchKernelGGL(reduce_partials_kernel<32>, dim3(blocks_for(n4, 256 / 32)), dim3(256), 0, st, partial, nslabs,
                       len, scale, out, ldo, row_len);
  else if (nslabs >= 8)
    hipLaunchKernelGGL(reduce_partials_kernel<8>, dim3(blocks_for(n4, 256 / 8)), dim3(256), 0, st, partial, nslabs,
                       len, scale, out, ldo, row_len);
  else
    hipLaunchKernelGGL(reduce_partials_kernel<1>, dim3(blocks_for(n4, 256)), dim3(256), 0, st, partial, nslabs, len,
                       scale, out, ldo, row_len);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_cast_weight(const float *W, int64_t rows, int64_t cols, int64_t ldw, int32_t dtype, void *Wc,
                               void *WcT, pcs_stream_t stream) {
  if (!W) return pcs_set_einval("pcs_cast_weight", "null W");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = blocks_for(rows * cols, 256);
  if (dtype == PCS_BF16)
    hipLaunchKernelGGL(cast_weight_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, W, rows, cols, ldw,
                       reinterpret_cast<bf16_t *>(Wc), reinterpret_cast<bf16_t *>(WcT));
  else if (dtype == PCS_F32)
    hipLaunchKernelGGL(cast_weight_kernel<float>, dim3(nb), dim3(256), 0, s, W, rows, cols, ldw,
                       reinterpret_cast<float *>(Wc), reinterpret_cast<float *>(WcT));
  else return pcs_set_einval("pcs_cast_weight", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_adam(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                        const float *grad_scale, float lr, float beta1, float beta2, float eps,
                        float weight_decay, int64_t step, pcs_stream_t stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || step < 1) return pcs_set_einval("pcs_adam", "bad arguments");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     param, grad, exp_avg, exp_avg_sq, n, grad_scale, lr, beta1, beta2, eps,
                     weight_decay, (float)bc1, (float)sqrt(bc2));
  PCS_CHECK_LAUNCH();
  return 0;
}

namespace {
__global__ void round_weight_kernel(const float *__restrict__ W, int64_t n, float *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = bf2f(pack2bf(W[i], 0.f) & 0xffffu);
}
}  // namespace

// fp32 copy of the weights as the compute dtype sees them (bf16: round-to-nearest-even, the
// rounding pcs_cast_weight applies), so the Gram-form weight gradients use the forward's W.
extern "C" int pcs_round_weight(const float *W, int64_t n, int32_t dtype, float *out, pcs_stream_t stream) {
  if (!W || !out || n < 0 || (dtype != PCS_F32 && dtype != PCS_BF16)) return pcs_set_einval("pcs_round_weight", "bad arguments");
  if (n == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == PCS_F32) return hipMemcpyAsync(out, W, n * 4, hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : PCS_EINVAL;
  hipLaunchKernelGGL(round_weight_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, W, n, out);
  PCS_CHECK_LAUNCH();
  return 0;
}

namespace {
// one thread per 8 channels of a row: two 16-B loads of Y, one (two, split) 16-B bf16 stores
template <bool SPLIT>
__global__ __launch_bounds__(256) void bnrelu_bf16_kernel(const float *__restrict__ Y, int64_t M, int K,
                                                         const float *__restrict__ s, const float *__restrict__ t,
                                                         bf16_t *__restrict__ out) {
  const int K8 = K >> 3;
  const int64_t n = M * K8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / K8;
    const int k = (int)(i - m * K8) * 8;
    const float4 y0 = *reinterpret_cast<const float4 *>(Y + m * K + k);
    const float4 y1 = *reinterpret_cast<const float4 *>(Y + m * K + k + 4);
    const float yv[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
    float hi[8], lo[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float a = relu(fmaf(yv[e], s[k + e], t[k + e]));
      hi[e] = bf2f(pack2bf(a, 0.f) & 0xffffu);
      lo[e] = a - hi[e];   // exact in fp32
    }
    const int64_t ld = SPLIT ? 2 * (int64_t)K : K;
    *reinterpret_cast<u32x4 *>(out + m * ld + k) = pack_chunk(hi);
    if constexpr (SPLIT) *reinterpret_cast<u32x4 *>(out + m * ld + K + k) = pack_chunk(lo);
  }
}
}  // namespace

extern "C" int pcs_bnrelu_bf16(const float *Y, int64_t M, int32_t K, const float *s, const float *t, int32_t split,
                               void *out, pcs_stream_t stream) {
  if (!Y || !s || !t || !out || M < 0 || K <= 0 || K % 8 != 0)
    return pcs_set_einval("pcs_bnrelu_bf16", "bad arguments (K must be a positive multiple of 8)");
  if (M == 0) return 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = (int)pcs_min64(blocks_for(M * (K / 8), 256), 8192);
  if (split)
    hipLaunchKernelGGL(bnrelu_bf16_kernel<true>, dim3(nb), dim3(256), 0, st, Y, M, K, s, t,
                       reinterpret_cast<bf16_t *>(out));
  else
    hipLaunchKernelGGL(bnrelu_bf16_kernel<false>, dim3(nb), dim3(256), 0, st, Y, M, K, s, t,
                       reinterpret_cast<bf16_t *>(out));
  PCS_CHECK_LAUNCH();
  return 0;
}

// Weight gradient of global_feat (P:113, autograd at P:254) from the Gram of its input.
//
// The max-pool feeds bn_global's backward a dy of the form (see pcs_pool_bwd)
//     dy[m, c] = beta[c] + gamma[c] * y[m, c] + [m == am[b, c]] * sp[b, c],
// and y = a W^T with a = relu(bn5(Y5)) (bias-free centred storage), so
//     dW = dy^T a = beta (x) S + diag(gamma) W G + sum_b sp[b, c] a[am[b, c], :]
// with G = a^T a and S = column sums of a (pcs_gram).  This replaces the M x 1024 x 1024
// weight-gradient GEMM by the symmetric Gram (upper tiles only) plus this O(C^3) assemble.
//
// A BN-fed layer (conv5: 128 -> 1024) has dy = alpha*dz + beta + gamma*y with y = a W^T, so
//     dW = diag(alpha) (dz^T a) + beta (x) S + diag(gamma) W G     (R = dz^T a: pcs_wgrad RAW)
//     dA = dz (diag(alpha) W) + a (W^T diag(gamma) W) + 1 (W^T beta)^T
// neither of which reads the layer's own (wide) output y: pcs_bn_fold builds the folded
// operands of the input-gradient form.
#include "common.h"

namespace {

constexpr int TILE = 64, KC = 32, THREADS = 256;

// TL x TL output tile per block (32 for the wide layer: 4x the blocks of 64), W and G chunks of
// KC along j through LDS with the next chunk prefetched in registers, (TL/16)^2 outputs per thread
template <typename T, int TL>
__global__ __launch_bounds__(THREADS) void gram_wgrad_kernel(
    const float *__restrict__ G, const float *__restrict__ S, const float *__restrict__ W, int64_t ldwin,
    const float *__restrict__ beta, const float *__restrict__ gamma, const float *__restrict__ sp,
    const int *__restrict__ am, const T *__restrict__ Y, const float *__restrict__ s,
    const float *__restrict__ t, int B, int Cout, int Cin, const float *__restrict__ R,
    const float *__restrict__ alpha, float *__restrict__ dW, int64_t ldw) {
  constexpr int RR = TL / 16, NE = TL * KC / THREADS;
  __shared__ float Ws[TL][KC + 1];
  __shared__ float Gs[KC][TL];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int c0 = blockIdx.y * TL, k0 = blockIdx.x * TL;
  float acc[RR][RR] = {};
  float pw[NE], pg[NE];
  auto load = [&](int j0) {
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + THREADS * u;
      pw[u] = W[(int64_t)(c0 + e / KC) * ldwin + j0 + e % KC];
      pg[u] = G[(int64_t)(j0 + e / TL) * Cin + k0 + e % TL];
    }
  };
  load(0);
  for (int j0 = 0; j0 < Cin; j0 += KC) {
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + THREADS * u;
      Ws[e / KC][e % KC] = pw[u];
      Gs[e / TL][e % TL] = pg[u];
    }
    __syncthreads();
    if (j0 + KC < Cin) load(j0 + KC);
#pragma unroll 8
    for (int q = 0; q < KC; ++q) {
      float wv[RR], gv[RR];
#pragma unroll
      for (int i = 0; i < RR; ++i) wv[i] = Ws[ty * RR + i][q];
#pragma unroll
      for (int j = 0; j < RR; ++j) gv[j] = Gs[q][tx * RR + j];
#pragma unroll
      for (int i = 0; i < RR; ++i)
#pragma unroll
        for (int j = 0; j < RR; ++j) acc[i][j] = fmaf(wv[i], gv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < RR; ++i) {
    const int c = c0 + ty * RR + i;
    const float gc = gamma[c], bc = beta[c];
    float o[RR];
#pragma unroll
    for (int j = 0; j < RR; ++j) {
      const int k = k0 + tx * RR + j;
      o[j] = fmaf(gc, acc[i][j], bc * S[k]);
      if (R) o[j] = fmaf(alpha[c], R[(int64_t)c * Cin + k], o[j]);
    }
    for (int b = 0; sp && b < B; ++b) {   // the max-pool rows: a recomputed from the stored Y
      const float w = sp[(int64_t)b * Cout + c];
      const int64_t m = am[(int64_t)b * Cout + c];
#pragma unroll
      for (int j = 0; j < RR; ++j) {
        const int k = k0 + tx * RR + j;
        o[j] = fmaf(w, relu(fmaf(load_elem(Y, m * Cin + k), s[k], t[k])), o[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < RR; ++j) dW[(int64_t)c * ldw + k0 + tx * RR + j] = o[j];
  }
}

}  // namespace

extern "C" int pcs_gram_wgrad(const float *G, const float *S, const float *W, int64_t ldw_in,
                              const float *beta, const float *gamma, const float *sp, const int32_t *am,
                              const void *Y, const float *s, const float *t, int64_t num_scenes,
                              int32_t Cout, int32_t Cin, int32_t dtype, const float *R, const float *alpha,
                              float *dW, int64_t ldw, pcs_stream_t stream) {
  if (!G || !S || !W || !beta || !gamma || !dW) return pcs_set_einval("pcs_gram_wgrad", "missing operand");
  if (sp && (!am || !Y || !s || !t)) return pcs_set_einval("pcs_gram_wgrad", "max-pool term needs am, Y, s, t");
  if (R && !alpha) return pcs_set_einval("pcs_gram_wgrad", "R needs alpha");
  if (Cout % TILE || Cin % TILE || num_scenes <= 0 || ldw % 4 || ldw < Cin || ldw_in < Cin)
    return pcs_set_einval("pcs_gram_wgrad", "Cout/Cin must be multiples of 64, ldw >= Cin (multiple of 4)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(Cin / 32, Cout / 32);   // 32 x 32 tiles: enough blocks for the wide layer and conv5
  if (dtype == PCS_BF16)
    hipLaunchKernelGGL((gram_wgrad_kernel<bf16_t, 32>), grid, dim3(THREADS), 0, st, G, S, W, ldw_in, beta, gamma,
                       sp, am, reinterpret_cast<const bf16_t *>(Y), s, t, (int)num_scenes, Cout, Cin, R, alpha,
                       dW, ldw);
  else if (dtype == PCS_F32)
    hipLaunchKernelGGL((gram_wgrad_kernel<float, 32>), grid, dim3(THREADS), 0, st, G, S, W, ldw_in, beta, gamma,
                       sp, am, reinterpret_cast<const float *>(Y), s, t, (int)num_scenes, Cout, Cin, R, alpha,
                       dW, ldw);
  else if (dtype == PCS_FP8)   // the fp8 path's e4m3 a5 (max-pool rows' term)
    hipLaunchKernelGGL((gram_wgrad_kernel<fp8_t, 32>), grid, dim3(THREADS), 0, st, G, S, W, ldw_in, beta, gamma,
                       sp, am, reinterpret_cast<const fp8_t *>(Y), s, t, (int)num_scenes, Cout, Cin, R, alpha,
                       dW, ldw);
  else
    return pcs_set_einval("pcs_gram_wgrad", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// pcs_bn_fold: operands of the input gradient of a BN-fed layer without reading its output
// ---------------------------------------------------------------------------------------
namespace {

// WsT[n][k] = W[k][n] * alpha[k]   (one thread per (n, k))
template <typename T>
__global__ void fold_wt_kernel(const float *__restrict__ W, int64_t ldw, int Cout, int Cin,
                               const float *__restrict__ alpha, T *__restrict__ WsT) {
  const int64_t n_el = (int64_t)Cout * Cin;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_el; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / Cout), k = (int)(i % Cout);
    const float v = W[(int64_t)k * ldw + n] * alpha[k];
    if constexpr (sizeof(T) == 2) WsT[i] = (T)(pack2bf(v, 0.f) & 0xffffu);
    else WsT[i] = v;
  }
}

// c[n] = sum_k beta[k] W[k][n]: block = 64 columns n x 4 parts of k (fixed-order combine)
__global__ __launch_bounds__(256) void fold_c_kernel(const float *__restrict__ W, int64_t ldw, int Cout, int Cin,
                                                     const float *__restrict__ beta, float *__restrict__ c) {
  __shared__ float red[4][64];
  const int nn = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + nn;
  const int k0 = (int)((int64_t)Cout * pr / 4), k1 = (int)((int64_t)Cout * (pr + 1) / 4);
  float acc = 0.f;
  if (n < Cin) {
#pragma unroll 8
    for (int k = k0; k < k1; ++k) acc = fmaf(beta[k], W[(int64_t)k * ldw + n], acc);
  }
  red[pr][nn] = acc;
  __syncthreads();
  if (pr == 0 && n < Cin) c[n] = ((red[0][nn] + red[1][nn]) + red[2][nn]) + red[3][nn];
}

// H[i][j] = sum_k (W[k][i] gamma[k]) W[k][j]: TILE x TILE output tile per block (32 for a
// 1024-wide H: 1024 blocks instead of 256, 4x the latency hiding), k in steps of 32 through LDS
// (rows of W are contiguous in i and j: coalesced), (TILE/16)^2 outputs per thread
template <typename T, int TILE>
__global__ __launch_bounds__(256) void fold_h_tiled_kernel(const float *__restrict__ W, int64_t ldw, int Cout,
                                                           int Cin, const float *__restrict__ gamma,
                                                           T *__restrict__ H) {
  constexpr int R = TILE / 16;
  __shared__ float Xs[32][TILE + 4];
  __shared__ float Ys[32][TILE + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int i0 = blockIdx.y * TILE, j0 = blockIdx.x * TILE;
  float acc[R][R] = {};
  // the next k-chunk is loaded into registers while this one is multiplied (few blocks per CU
  // for the small H: nothing else hides the load latency)
  constexpr int NE = 32 * TILE / 256;
  float px[NE], py[NE];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u, kk = e / TILE, cc = e % TILE, k = k0 + kk;
      const bool ok = k < Cout;
      px[u] = ok ? W[(int64_t)k * ldw + i0 + cc] * gamma[k] : 0.f;
      py[u] = ok ? W[(int64_t)k * ldw + j0 + cc] : 0.f;
    }
  };
  load(0);
  for (int k0 = 0; k0 < Cout; k0 += 32) {
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      Xs[e / TILE][e % TILE] = px[u];
      Ys[e / TILE][e % TILE] = py[u];
    }
    __syncthreads();
    if (k0 + 32 < Cout) load(k0 + 32);
#pragma unroll 8
    for (int kk = 0; kk < 32; ++kk) {
      float xa[R], ya[R];
#pragma unroll
      for (int p = 0; p < R; ++p) { xa[p] = Xs[kk][ty * R + p]; ya[p] = Ys[kk][tx * R + p]; }
#pragma unroll
      for (int p = 0; p < R; ++p)
#pragma unroll
        for (int q = 0; q < R; ++q) acc[p][q] = fmaf(xa[p], ya[q], acc[p][q]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int p = 0; p < R; ++p)
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int64_t o = (int64_t)(i0 + ty * R + p) * Cin + j0 + tx * R + q;
      if constexpr (sizeof(T) == 2) H[o] = (T)(pack2bf(acc[p][q], 0.f) & 0xffffu);
      else H[o] = acc[p][q];
    }
}

// BN statistics of y = a W^T from G = a^T a and S: one block per output channel c,
// mean = w.S / n, M2 = sum_jk w_j w_k (G_jk - S_j S_k / n), fp64 (w cached in LDS)
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_gram_kernel(const float *__restrict__ G, const float *__restrict__ S,
                                                            double n, const T *__restrict__ W, int64_t ldw, int C,
                                                            int Cin, int B, float *__restrict__ stats) {
  __shared__ double w[1024];
  __shared__ double sh[256][2];
  const int c = blockIdx.x, tid = threadIdx.x;
  double dm = 0.0;
  for (int k = tid; k < Cin; k += 256) {
    w[k] = (double)load_elem(W, (int64_t)c * ldw + k);
    dm += w[k] * (double)S[k];
  }
  __syncthreads();
  double q = 0.0;
  for (int j = tid; j < Cin; j += 256) {
    const double sj = (double)S[j] / n;
    double row = 0.0;
    for (int k = 0; k < Cin; ++k) row += ((double)G[(int64_t)j * Cin + k] - sj * (double)S[k]) * w[k];
    q += w[j] * row;
  }
  sh[tid][0] = dm; sh[tid][1] = q;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) { sh[tid][0] += sh[tid + st][0]; sh[tid][1] += sh[tid + st][1]; }
    __syncthreads();
  }
  if (tid < B) {
    const double mean = sh[0][0] / n, m2 = sh[0][1] < 0.0 ? 0.0 : sh[0][1];   // clamp; a NaN stays
    *reinterpret_cast<float2 *>(stats + ((int64_t)tid * C + c) * 2) = make_float2((float)mean, (float)(m2 / B));
  }
}

// bn_global's statistics from G = a^T a (C x C, full) and per-scene column sums Sb [B, Cin]:
// mean_b = Sb[b] w / N exactly, M2 = w (G - S S^T / M) w^T (S = sum_b Sb), and per-scene
// M2_b chosen so that merging the B partials (Chan) gives M2:
//   M2_b = (M2 - N sum_b (mean_b - mean)^2) / B   (clamped at 0)
// Pass 1 (gram_quad_kernel): part[kz][jt][c] = sum_{j in 64-tile jt} w_c[j] (G_{:, kz} w_c^T)[j]
// as an fp64 64x64-tiled product over one of QK_SPLIT k-ranges (G read k-major: it is
// symmetric; the split gives 1024 workgroups at C = 1024 instead of 256 one-wave-per-SIMD
// ones); pass 2 adds the partials in a fixed order, subtracts (S w)^2 / M and forms the
// per-scene pairs.
constexpr int QK_SPLIT = 4;

template <typename T>
__global__ __launch_bounds__(256) void gram_quad_kernel(const float *__restrict__ G, const T *__restrict__ W,
                                                        int64_t ldw, int Cin, double *__restrict__ part) {
  __shared__ double gs[16][64];   // gs[k][j] = G[k0 + k][j0 + j] (= G[j][k])
  __shared__ double wt[16][65];   // wt[k][c] = W[c0 + c][k0 + k]
  __shared__ double red[16][64];
  const int C = gridDim.x * 64, c0 = blockIdx.x * 64, j0 = blockIdx.y * 64;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  double acc[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  const int kz0 = (int)((int64_t)Cin / 16 * blockIdx.z / QK_SPLIT) * 16;
  const int kz1 = (int)((int64_t)Cin / 16 * (blockIdx.z + 1) / QK_SPLIT) * 16;
  for (int k0 = kz0; k0 < kz1; k0 += 16) {
#pragma unroll
    for (int e = tid; e < 1024; e += 256) {
      gs[e >> 6][e & 63] = (double)G[(int64_t)(k0 + (e >> 6)) * Cin + j0 + (e & 63)];
      wt[e & 15][e >> 4] = (double)load_elem(W, (int64_t)(c0 + (e >> 4)) * ldw + k0 + (e & 15));
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < 16; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) { a[p] = gs[kk][ty * 4 + p]; b[p] = wt[kk][tx * 4 + p]; }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][q] = fma(a[p], b[q], acc[p][q]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t wr = (int64_t)(c0 + tx * 4 + q) * ldw + j0 + ty * 4;
    double s = 0.0;
#pragma unroll
    for (int p = 0; p < 4; ++p) s = fma((double)load_elem(W, wr + p), acc[p][q], s);
    red[ty][tx * 4 + q] = s;
  }
  __syncthreads();
  if (tid < 64) {
    double s = 0.0;
    for (int r = 0; r < 16; ++r) s += red[r][tid];
    part[((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * C + c0 + tid] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_stats_scenes_kernel(const double *__restrict__ part, int njt,
                                                              const float *__restrict__ Sb, double nb,
                                                              const T *__restrict__ W, int64_t ldw, int C, int Cin,
                                                              int B, float *__restrict__ stats) {
  __shared__ double sh[256];
  __shared__ double d[64];
  const int c = blockIdx.x, tid = threadIdx.x;
  for (int b = 0; b < B; ++b) {
    double x = 0.0;
    for (int k = tid; k < Cin; k += 256)
      x = fma((double)load_elem(W, (int64_t)c * ldw + k), (double)Sb[(int64_t)b * Cin + k], x);
    sh[tid] = x;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (tid < st) sh[tid] += sh[tid + st];
      __syncthreads();
    }
    if (tid == 0) d[b] = sh[0];
    __syncthreads();
  }
  double qp = 0.0;   // the partials: strided per thread, then a fixed-order tree
  for (int jt = tid; jt < njt; jt += 256) qp += part[(int64_t)jt * C + c];
  sh[tid] = qp;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) sh[tid] += sh[tid + st];
    __syncthreads();
  }
  if (tid == 0) {
    const double n = nb * B;
    double q = sh[0], s = 0.0, between = 0.0;
    for (int b = 0; b < B; ++b) s += d[b];
    const double mean = s / n;
    for (int b = 0; b < B; ++b) between += nb * (d[b] / nb - mean) * (d[b] / nb - mean);
    double m2b = (q - s * s / n - between) / B;
    m2b = m2b < 0.0 ? 0.0 : m2b;   // clamp the rounding; a NaN (a diverged a5) stays NaN, as torch's var
    for (int b = 0; b < B; ++b)
      *reinterpret_cast<float2 *>(stats + ((int64_t)b * C + c) * 2) = make_float2((float)(d[b] / nb), (float)m2b);
  }
}

// S2 of a BN-fed layer from R = dz^T a: rstd (sum_k W[c,k] R[c,k] - mean S1), rewritten into
// the per-chunk partials (chunk 0 = total, others 0).  One block per channel, fp64 sums.
template <typename T>
__global__ __launch_bounds__(256) void bn_s2_kernel(float *__restrict__ stats, int64_t nch, int C,
                                                    const float *__restrict__ R, const T *__restrict__ W,
                                                    int64_t ldw, int Cin, const float *__restrict__ mean,
                                                    const float *__restrict__ rstd) {
  __shared__ double sh[256][2];
  const int c = blockIdx.x, tid = threadIdx.x;
  double dot = 0.0, s1 = 0.0;
  for (int k = tid; k < Cin; k += 256) dot += (double)load_elem(W, (int64_t)c * ldw + k) * (double)R[(int64_t)c * Cin + k];
  for (int64_t ch = tid; ch < nch; ch += 256) s1 += (double)stats[(ch * C + c) * 2];
  sh[tid][0] = dot; sh[tid][1] = s1;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) { sh[tid][0] += sh[tid + st][0]; sh[tid][1] += sh[tid + st][1]; }
    __syncthreads();
  }
  for (int64_t ch = tid; ch < nch; ch += 256)
    stats[(ch * C + c) * 2 + 1] = ch == 0 ? (float)((double)rstd[c] * (sh[0][0] - (double)mean[c] * sh[0][1])) : 0.f;
}

// H[i][j] = sum_k W[k][i] gamma[k] W[k][j]: block = row i, 4 parts of k (fixed-order combine)
template <typename T>
__global__ __launch_bounds__(256) void fold_h_kernel(const float *__restrict__ W, int64_t ldw, int Cout, int Cin,
                                                     const float *__restrict__ gamma, T *__restrict__ H) {
  __shared__ float red[4][64];
  const int i = blockIdx.x, jj = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int k0 = (int)((int64_t)Cout * pr / 4), k1 = (int)((int64_t)Cout * (pr + 1) / 4);
  for (int j0 = 0; j0 < Cin; j0 += 64) {
    const int j = j0 + jj;
    float acc = 0.f;
    if (j < Cin)
      for (int k = k0; k < k1; ++k) acc = fmaf(W[(int64_t)k * ldw + i] * gamma[k], W[(int64_t)k * ldw + j], acc);
    red[pr][jj] = acc;
    __syncthreads();
    if (pr == 0 && j < Cin) {
      const float v = ((red[0][jj] + red[1][jj]) + red[2][jj]) + red[3][jj];
      if constexpr (sizeof(T) == 2) H[(int64_t)i * Cin + j] = (T)(pack2bf(v, 0.f) & 0xffffu);
      else H[(int64_t)i * Cin + j] = v;
    }
    __syncthreads();
  }
}

}  // namespace

template <typename T>
void launch_fold(const float *W, int Cout, int Cin, int64_t ldw, const float *alpha, const float *beta,
                 const float *gamma, T *WsT, float *c, T *H, hipStream_t st) {
  if (WsT) {
    const int nb = (int)pcs_min64(1024, ((int64_t)Cout * Cin + 255) / 256);
    hipLaunchKernelGGL(fold_wt_kernel<T>, dim3(nb), dim3(256), 0, st, W, ldw, Cout, Cin, alpha, WsT);
  }
  if (c) hipLaunchKernelGGL(fold_c_kernel, dim3((Cin + 63) / 64), dim3(256), 0, st, W, ldw, Cout, Cin, beta, c);
  if (Cin % 64 == 0 && Cin >= 512)
    hipLaunchKernelGGL((fold_h_tiled_kernel<T, 32>), dim3(Cin / 32, Cin / 32), dim3(256), 0, st, W, ldw, Cout, Cin,
                       gamma, H);
  else if (Cin % 64 == 0)   // small H (conv5's 128, seg_conv1's 64): 16 x 16 tiles, more blocks
    hipLaunchKernelGGL((fold_h_tiled_kernel<T, 16>), dim3(Cin / 16, Cin / 16), dim3(256), 0, st, W, ldw, Cout, Cin,
                       gamma, H);
  else
    hipLaunchKernelGGL(fold_h_kernel<T>, dim3(Cin), dim3(256), 0, st, W, ldw, Cout, Cin, gamma, H);
}

extern "C" int pcs_bn_fold(const float *W, int32_t Cout, int32_t Cin, int64_t ldw, const float *alpha,
                           const float *beta, const float *gamma, int32_t dtype, void *WsT, float *c, void *H,
                           pcs_stream_t stream) {
  if (!W || !gamma || (WsT && !alpha) || (c && !beta) || !H || Cout <= 0 || Cin <= 0 || ldw < Cin)
    return pcs_set_einval("pcs_bn_fold", "bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == PCS_BF16)
    launch_fold<bf16_t>(W, Cout, Cin, ldw, alpha, beta, gamma, reinterpret_cast<bf16_t *>(WsT), c,
                        reinterpret_cast<bf16_t *>(H), st);
  else if (dtype == PCS_F32)
    launch_fold<float>(W, Cout, Cin, ldw, alpha, beta, gamma, reinterpret_cast<float *>(WsT), c,
                       reinterpret_cast<float *>(H), st);
  else
    return pcs_set_einval("pcs_bn_fold", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_bn_s2_from_r(float *stats, int64_t num_chunks, int32_t C, const float *R, const void *W,
                                int32_t dtype, int64_t ldw, int32_t Cin, const float *mean, const float *rstd,
                                pcs_stream_t stream) {
  if (!stats || !R || !W || !mean || !rstd || num_chunks <= 0 || C <= 0 || Cin <= 0 || ldw < Cin)
    return pcs_set_einval("pcs_bn_s2_from_r", "bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == PCS_BF16)
    hipLaunchKernelGGL(bn_s2_kernel<bf16_t>, dim3(C), dim3(256), 0, st, stats, num_chunks, (int)C, R,
                       reinterpret_cast<const bf16_t *>(W), ldw, (int)Cin, mean, rstd);
  else if (dtype == PCS_F32)
    hipLaunchKernelGGL(bn_s2_kernel<float>, dim3(C), dim3(256), 0, st, stats, num_chunks, (int)C, R,
                       reinterpret_cast<const float *>(W), ldw, (int)Cin, mean, rstd);
  else
    return pcs_set_einval("pcs_bn_s2_from_r", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t pcs_bn_stats_from_gram_scenes_workspace(int32_t C, int32_t Cin) {
  if (C <= 0 || Cin <= 0 || C % 64 || Cin % 64) return pcs_set_einval("pcs_bn_stats_from_gram_scenes_workspace", "C, Cin must be positive multiples of 64");
  return (int64_t)QK_SPLIT * (Cin / 64) * C * (int64_t)sizeof(double);
}

template <typename T>
static void launch_stats_scenes(const float *G, const float *Sb, int64_t nb, const T *W, int64_t ldw, int C, int Cin,
                                int B, double *part, float *stats, hipStream_t st) {
  hipLaunchKernelGGL(gram_quad_kernel<T>, dim3(C / 64, Cin / 64, QK_SPLIT), dim3(256), 0, st, G, W, ldw, Cin, part);
  hipLaunchKernelGGL(bn_stats_scenes_kernel<T>, dim3(C), dim3(256), 0, st, part, QK_SPLIT * (Cin / 64), Sb,
                     (double)nb, W, ldw,
                     C, Cin, B, stats);
}

extern "C" int pcs_bn_stats_from_gram_scenes(const float *G, const float *Sb, int64_t scene_rows, const void *W,
                                             int32_t dtype, int64_t ldw, int32_t C, int32_t Cin, int64_t num_scenes,
                                             void *workspace, int64_t workspace_bytes, float *stats,
                                             pcs_stream_t stream) {
  if (!G || !Sb || !W || !stats || !workspace || scene_rows <= 0 || C <= 0 || Cin <= 0 || C % 64 || Cin % 64 ||
      ldw < Cin || C != Cin || num_scenes <= 0 || num_scenes > 64)
    return pcs_set_einval("pcs_bn_stats_from_gram_scenes",
                          "bad arguments (C == Cin, multiples of 64; 1 <= num_scenes <= 64)");
  if (workspace_bytes < (int64_t)QK_SPLIT * (Cin / 64) * C * (int64_t)sizeof(double))
    return pcs_set_einval("pcs_bn_stats_from_gram_scenes", "workspace too small");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double *part = static_cast<double *>(workspace);
  if (dtype == PCS_BF16)
    launch_stats_scenes<bf16_t>(G, Sb, scene_rows, reinterpret_cast<const bf16_t *>(W), ldw, C, Cin,
                                (int)num_scenes, part, stats, st);
  else if (dtype == PCS_F32)
    launch_stats_scenes<float>(G, Sb, scene_rows, reinterpret_cast<const float *>(W), ldw, C, Cin, (int)num_scenes,
                               part, stats, st);
  else
    return pcs_set_einval("pcs_bn_stats_from_gram_scenes", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_bn_stats_from_gram(const float *G, const float *S, int64_t count, const void *W, int32_t dtype,
                                      int64_t ldw, int32_t C, int32_t Cin, int64_t num_scenes, float *stats,
                                      pcs_stream_t stream) {
  if (!G || !S || !W || !stats || count <= 0 || C <= 0 || Cin <= 0 || Cin > 1024 || ldw < Cin ||
      num_scenes <= 0 || num_scenes > 256)
    return pcs_set_einval("pcs_bn_stats_from_gram", "bad arguments (Cin <= 1024, num_scenes <= 256)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == PCS_BF16)
    hipLaunchKernelGGL(bn_stats_gram_kernel<bf16_t>, dim3(C), dim3(256), 0, st, G, S, (double)count,
                       reinterpret_cast<const bf16_t *>(W), ldw, (int)C, (int)Cin, (int)num_scenes, stats);
  else if (dtype == PCS_F32)
    hipLaunchKernelGGL(bn_stats_gram_kernel<float>, dim3(C), dim3(256), 0, st, G, S, (double)count,
                       reinterpret_cast<const float *>(W), ldw, (int)C, (int)Cin, (int)num_scenes, stats);
  else
    return pcs_set_einval("pcs_bn_stats_from_gram", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

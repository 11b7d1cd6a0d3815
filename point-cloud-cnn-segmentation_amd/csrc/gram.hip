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

template <typename T>
__global__ __launch_bounds__(THREADS) void gram_wgrad_kernel(
    const float *__restrict__ G, const float *__restrict__ S, const float *__restrict__ W, int64_t ldwin,
    const float *__restrict__ beta, const float *__restrict__ gamma, const float *__restrict__ sp,
    const int *__restrict__ am, const T *__restrict__ Y, const float *__restrict__ s,
    const float *__restrict__ t, int B, int Cout, int Cin, const float *__restrict__ R,
    const float *__restrict__ alpha, float *__restrict__ dW, int64_t ldw) {
  __shared__ float Ws[TILE][KC + 1];
  __shared__ float Gs[KC][TILE];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int c0 = blockIdx.y * TILE, k0 = blockIdx.x * TILE;
  float acc[4][4] = {};
  for (int j0 = 0; j0 < Cin; j0 += KC) {
    for (int e = tid; e < TILE * KC; e += THREADS) {
      const int r = e / KC, q = e % KC;
      Ws[r][q] = W[(int64_t)(c0 + r) * ldwin + j0 + q];
      const int gr = e / TILE, gq = e % TILE;
      Gs[gr][gq] = G[(int64_t)(j0 + gr) * Cin + k0 + gq];
    }
    __syncthreads();
#pragma unroll 8
    for (int q = 0; q < KC; ++q) {
      float wv[4], gv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) wv[i] = Ws[ty * 4 + i][q];
#pragma unroll
      for (int j = 0; j < 4; ++j) gv[j] = Gs[q][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(wv[i], gv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = c0 + ty * 4 + i;
    const float gc = gamma[c], bc = beta[c];
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + tx * 4 + j;
      o[j] = fmaf(gc, acc[i][j], bc * S[k]);
      if (R) o[j] = fmaf(alpha[c], R[(int64_t)c * Cin + k], o[j]);
    }
    for (int b = 0; sp && b < B; ++b) {   // the max-pool rows: a recomputed from the stored Y
      const float w = sp[(int64_t)b * Cout + c];
      const int64_t m = am[(int64_t)b * Cout + c];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + tx * 4 + j;
        o[j] = fmaf(w, fmaxf(fmaf(load_elem(Y, m * Cin + k), s[k], t[k]), 0.f), o[j]);
      }
    }
    *reinterpret_cast<float4 *>(dW + (int64_t)c * ldw + k0 + tx * 4) = make_float4(o[0], o[1], o[2], o[3]);
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
  const dim3 grid(Cin / TILE, Cout / TILE);
  if (dtype == PCS_BF16)
    hipLaunchKernelGGL(gram_wgrad_kernel<bf16_t>, grid, dim3(THREADS), 0, st, G, S, W, ldw_in, beta, gamma,
                       sp, am, reinterpret_cast<const bf16_t *>(Y), s, t, (int)num_scenes, Cout, Cin, R, alpha,
                       dW, ldw);
  else if (dtype == PCS_F32)
    hipLaunchKernelGGL(gram_wgrad_kernel<float>, grid, dim3(THREADS), 0, st, G, S, W, ldw_in, beta, gamma,
                       sp, am, reinterpret_cast<const float *>(Y), s, t, (int)num_scenes, Cout, Cin, R, alpha,
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

// WsT[n][k] = W[k][n] * alpha[k];  c[n] = sum_k beta[k] W[k][n]       (one thread per (n, k) / n)
template <typename T>
__global__ void fold_wt_kernel(const float *__restrict__ W, int64_t ldw, int Cout, int Cin,
                               const float *__restrict__ alpha, const float *__restrict__ beta,
                               T *__restrict__ WsT, float *__restrict__ c) {
  const int64_t n_el = (int64_t)Cout * Cin;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_el; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / Cout), k = (int)(i % Cout);
    const float v = W[(int64_t)k * ldw + n] * alpha[k];
    if constexpr (sizeof(T) == 2) WsT[i] = (T)(pack2bf(v, 0.f) & 0xffffu);
    else WsT[i] = v;
  }
  if (blockIdx.x == 0) {
    for (int n = threadIdx.x; n < Cin; n += blockDim.x) {
      float acc = 0.f;
      for (int k = 0; k < Cout; ++k) acc = fmaf(beta[k], W[(int64_t)k * ldw + n], acc);
      c[n] = acc;
    }
  }
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

extern "C" int pcs_bn_fold(const float *W, int32_t Cout, int32_t Cin, int64_t ldw, const float *alpha,
                           const float *beta, const float *gamma, int32_t dtype, void *WsT, float *c, void *H,
                           pcs_stream_t stream) {
  if (!W || !alpha || !beta || !gamma || !WsT || !c || !H || Cout <= 0 || Cin <= 0 || ldw < Cin)
    return pcs_set_einval("pcs_bn_fold", "bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = (int)pcs_min64(1024, ((int64_t)Cout * Cin + 255) / 256);
  if (dtype == PCS_BF16) {
    hipLaunchKernelGGL(fold_wt_kernel<bf16_t>, dim3(nb), dim3(256), 0, st, W, ldw, Cout, Cin, alpha, beta,
                       reinterpret_cast<bf16_t *>(WsT), c);
    hipLaunchKernelGGL(fold_h_kernel<bf16_t>, dim3(Cin), dim3(256), 0, st, W, ldw, Cout, Cin, gamma,
                       reinterpret_cast<bf16_t *>(H));
  } else if (dtype == PCS_F32) {
    hipLaunchKernelGGL(fold_wt_kernel<float>, dim3(nb), dim3(256), 0, st, W, ldw, Cout, Cin, alpha, beta,
                       reinterpret_cast<float *>(WsT), c);
    hipLaunchKernelGGL(fold_h_kernel<float>, dim3(Cin), dim3(256), 0, st, W, ldw, Cout, Cin, gamma,
                       reinterpret_cast<float *>(H));
  } else {
    return pcs_set_einval("pcs_bn_fold", "bad dtype");
  }
  PCS_CHECK_LAUNCH();
  return 0;
}

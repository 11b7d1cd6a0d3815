// Device confusion matrix for the training/validation metrics (P:261-266, P:299-346):
// prediction = argmax over the C logits of a point (first maximum), rows = true label,
// columns = prediction, labels < 0 (padding, P:54) skipped.  Accumulates into cm (int64
// [C, C]) so a whole epoch needs one host read.
#include "common.h"

namespace {

constexpr int THREADS = 256, CMAX = 64, CMAX_ALL = 256;

// LDS = true: per-block histogram in LDS (C <= 64); otherwise straight to the global matrix
template <bool LDS>
__global__ __launch_bounds__(THREADS) void confusion_kernel(const float *__restrict__ logits, int64_t ld,
                                                            const int64_t *__restrict__ labels, int64_t M,
                                                            int C, unsigned long long *__restrict__ cm) {
  __shared__ unsigned int hist[LDS ? CMAX * CMAX : 1];
  if constexpr (LDS) {
    for (int i = threadIdx.x; i < C * C; i += THREADS) hist[i] = 0u;
    __syncthreads();
  }
  for (int64_t m = (int64_t)blockIdx.x * THREADS + threadIdx.x; m < M; m += (int64_t)gridDim.x * THREADS) {
    const int64_t y = labels[m];
    if (y < 0 || y >= C) continue;
    const float *z = logits + m * ld;
    int best = 0;
    float bz = z[0];
    for (int c = 1; c < C; ++c) {
      const float v = z[c];
      if (v > bz) { bz = v; best = c; }
    }
    if constexpr (LDS) atomicAdd(&hist[(int)y * C + best], 1u);
    else atomicAdd(&cm[(int)y * C + best], 1ull);
  }
  if constexpr (LDS) {
    __syncthreads();
    for (int i = threadIdx.x; i < C * C; i += THREADS)
      if (hist[i]) atomicAdd(&cm[i], (unsigned long long)hist[i]);
  }
}

}  // namespace

extern "C" int pcs_confusion(const float *logits, int64_t ld, const int64_t *labels, int64_t M, int32_t C,
                             int64_t *cm, pcs_stream_t stream) {
  if (!logits || !labels || !cm || M < 0 || C < 1 || C > CMAX_ALL || ld < C)
    return pcs_set_einval("pcs_confusion", "bad arguments (1 <= C <= 256, ld >= C)");
  if (M == 0) return 0;
  const int nb = (int)pcs_min64(2048, (M + THREADS - 1) / THREADS);
  if (C <= CMAX)
    hipLaunchKernelGGL(confusion_kernel<true>, dim3(nb), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                       logits, ld, labels, M, C, reinterpret_cast<unsigned long long *>(cm));
  else
    hipLaunchKernelGGL(confusion_kernel<false>, dim3(nb), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                       logits, ld, labels, M, C, reinterpret_cast<unsigned long long *>(cm));
  PCS_CHECK_LAUNCH();
  return 0;
}

namespace {

__global__ void argmax_kernel(const float *__restrict__ logits, int64_t ld, int64_t M, int C,
                              int64_t *__restrict__ out) {
  for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
    const float *z = logits + m * ld;
    int best = 0;
    float bz = z[0];
    for (int c = 1; c < C; ++c)
      if (z[c] > bz) { bz = z[c]; best = c; }
    out[m] = best;
  }
}

}  // namespace

// predictions = argmax over classes (first maximum), the inference path of P:448-452
extern "C" int pcs_argmax(const float *logits, int64_t ld, int64_t M, int32_t C, int64_t *out,
                          pcs_stream_t stream) {
  if (!logits || !out || M < 0 || C < 1 || ld < C) return pcs_set_einval("pcs_argmax", "bad arguments");
  if (M == 0) return 0;
  const int nb = (int)pcs_min64(4096, (M + 255) / 256);
  hipLaunchKernelGGL(argmax_kernel, dim3(nb), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), logits, ld, M,
                     C, out);
  PCS_CHECK_LAUNCH();
  return 0;
}

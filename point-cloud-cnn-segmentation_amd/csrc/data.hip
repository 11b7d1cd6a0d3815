// Device-side collate: ragged CSR batch -> the padded batch collate_fn builds
// on the host (P:44-63).  Scene b owns rows offsets[b] .. offsets[b+1] of the flat point /
// label arrays; the padded outputs are [B, N] with N >= every scene's length.  Pads are
// (0,0,0,0) points, label -1, mask 0 -- byte-identical to collate_fn.
//
// Pure byte movement: per padded point it reads 16 B of xyz+e and 4/8 B of label (real
// points only) and writes 16 + 8 + 1 B.  HBM-bound; one thread per point with 16-byte
// vector loads / stores, grid-stride, the scene of a row found once per thread from the
// row index (b = row / N), so no search over offsets is needed.
#include "common.h"

namespace {

constexpr int THREADS = 256;

template <typename LabT>
__global__ __launch_bounds__(THREADS) void pad_scatter_kernel(
    const f32x4 *__restrict__ pts, const LabT *__restrict__ lab, const int64_t *__restrict__ offsets,
    int64_t B, int64_t N, f32x4 *__restrict__ pts_out, int64_t *__restrict__ lab_out,
    uint8_t *__restrict__ mask_out) {
  const int64_t total = B * N;
  for (int64_t r = (int64_t)blockIdx.x * THREADS + threadIdx.x; r < total; r += (int64_t)gridDim.x * THREADS) {
    const int64_t b = r / N;
    const int64_t n = r - b * N;
    const int64_t lo = offsets[b];
    const bool real = n < offsets[b + 1] - lo;
    const int64_t src = lo + n;
    if (pts_out) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (real) v = pts[src];
      pts_out[r] = v;
    }
    if (lab_out) lab_out[r] = real ? (int64_t)lab[src] : (int64_t)-1;
    if (mask_out) mask_out[r] = real ? 1 : 0;
  }
}

}  // namespace

extern "C" int pcs_pad_scatter(const float *points, const void *labels, int32_t label_bytes,
                               const int64_t *offsets, int64_t num_scenes, int64_t scene_rows,
                               float *points_out, int64_t *labels_out, uint8_t *mask_out,
                               pcs_stream_t stream) {
  if (num_scenes < 0 || scene_rows < 0 || !offsets || (label_bytes != 4 && label_bytes != 8))
    return pcs_set_einval("pcs_pad_scatter", "bad arguments (label_bytes must be 4 or 8)");
  if ((points_out && !points) || (labels_out && !labels))
    return pcs_set_einval("pcs_pad_scatter", "an output is requested without its input");
  if ((reinterpret_cast<uintptr_t>(points) | reinterpret_cast<uintptr_t>(points_out)) & 15u)
    return pcs_set_einval("pcs_pad_scatter", "points buffers must be 16-byte aligned");
  const int64_t total = num_scenes * scene_rows;
  if (total == 0) return 0;
  const int nb = (int)pcs_min64(8192, (total + THREADS - 1) / THREADS);
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const f32x4 *p = reinterpret_cast<const f32x4 *>(points);
  f32x4 *po = reinterpret_cast<f32x4 *>(points_out);
  if (label_bytes == 8)
    hipLaunchKernelGGL(pad_scatter_kernel<int64_t>, dim3(nb), dim3(THREADS), 0, s, p,
                       static_cast<const int64_t *>(labels), offsets, num_scenes, scene_rows, po, labels_out,
                       mask_out);
  else
    hipLaunchKernelGGL(pad_scatter_kernel<int32_t>, dim3(nb), dim3(THREADS), 0, s, p,
                       static_cast<const int32_t *>(labels), offsets, num_scenes, scene_rows, po, labels_out,
                       mask_out);
  PCS_CHECK_LAUNCH();
  return 0;
}

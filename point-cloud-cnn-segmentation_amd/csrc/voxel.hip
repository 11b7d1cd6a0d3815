// Point -> voxel quantisation and the occupied-voxel (sparse) scatter / gather of the north
// star's voxel path (SURVEY §0 decision 3, §8 f4).  The reference has no voxelisation (its
// model consumes raw points, P:98-133), so this is build-defined and its oracle is the numpy
// restatement in oracle/voxel_oracle.py, labelled "not reference parity".
//
//   voxel id   v(p) = (ix * G + iy) * G + iz,  ix = clamp(floor((x - lo_x) / (hi_x - lo_x) * G), 0, G-1)
//              (fp32, IEEE division and multiply in this order: bit-exact with numpy float32)
//   key        scene(p) * G^3 + v(p)  (uint64), sorted stably with the point index as value
//   voxels     one per distinct key, in key order (scene-major, then voxel id):
//              x, y, z = mean of its points, e = sum of its points' e (fp32 sums in the sorted,
//              i.e. original, point order), label = most frequent label (ties: smaller label,
//              labels < 0 ignored, -1 if none), count
//   inverse    voxel_of_point[p] = global index of p's voxel (the gather that maps per-voxel
//              predictions back to points)
//
// Integer work is bit-exact by construction (radix sort, flag + scan, per-segment loops);
// the per-voxel float sums run sequentially in a fixed order, so results are deterministic.
#include "common.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

namespace {

constexpr int THREADS = 256;

struct Box {
  float lo[3], hi[3];
};

PCS_DEV int64_t voxel_of(const float *p, int G, const Box &b) {
  int64_t id = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float t = (p[d] - b.lo[d]) / (b.hi[d] - b.lo[d]);
    int i = (int)floorf(t * (float)G);
    i = i < 0 ? 0 : (i > G - 1 ? G - 1 : i);
    id = id * G + i;
  }
  return id;
}

__global__ __launch_bounds__(THREADS) void voxel_ids_kernel(const float *__restrict__ pts, int64_t T, int G, Box b,
                                                            int64_t *__restrict__ ids) {
  for (int64_t t = (int64_t)blockIdx.x * THREADS + threadIdx.x; t < T; t += (int64_t)gridDim.x * THREADS)
    ids[t] = voxel_of(pts + t * 4, G, b);
}

// key = scene * G^3 + voxel id; value = point index
__global__ __launch_bounds__(THREADS) void voxel_keys_kernel(const float *__restrict__ pts,
                                                             const int64_t *__restrict__ offsets, int B, int64_t T,
                                                             int G, Box b, uint64_t *__restrict__ keys,
                                                             int64_t *__restrict__ vals) {
  const uint64_t G3 = (uint64_t)G * G * G;
  for (int64_t t = (int64_t)blockIdx.x * THREADS + threadIdx.x; t < T; t += (int64_t)gridDim.x * THREADS) {
    int lo = 0, hi = B;   // scene: last b with offsets[b] <= t (offsets ascending, may repeat)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offsets[mid] <= t) lo = mid; else hi = mid;
    }
    keys[t] = (uint64_t)lo * G3 + (uint64_t)voxel_of(pts + t * 4, G, b);
    vals[t] = t;
  }
}

__global__ __launch_bounds__(THREADS) void head_flags_kernel(const uint64_t *__restrict__ k, int64_t T,
                                                             int64_t *__restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < T; i += (int64_t)gridDim.x * THREADS)
    flags[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// seg[i] = inclusive count of heads - 1: the voxel index of sorted position i
__global__ __launch_bounds__(THREADS) void seg_starts_kernel(const int64_t *__restrict__ seg, int64_t T,
                                                             int64_t *__restrict__ start, int64_t *__restrict__ nvox) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < T; i += (int64_t)gridDim.x * THREADS) {
    if (i == 0 || seg[i] != seg[i - 1]) start[seg[i] - 1] = i;
    if (i == T - 1) { start[seg[i]] = T; *nvox = seg[i]; }
  }
}

__global__ __launch_bounds__(THREADS) void aggregate_kernel(const float *__restrict__ pts,
                                                            const int64_t *__restrict__ labels,
                                                            const uint64_t *__restrict__ keys,
                                                            const int64_t *__restrict__ perm,
                                                            const int64_t *__restrict__ start,
                                                            const int64_t *__restrict__ nvox, int C,
                                                            f32x4 *__restrict__ vpts, int64_t *__restrict__ vlab,
                                                            int64_t *__restrict__ vcount,
                                                            int64_t *__restrict__ vox_of_point) {
  const int64_t V = *nvox;
  for (int64_t v = (int64_t)blockIdx.x * THREADS + threadIdx.x; v < V; v += (int64_t)gridDim.x * THREADS) {
    const int64_t s = start[v], e = start[v + 1];
    float sx = 0.f, sy = 0.f, sz = 0.f, se = 0.f;
    int hist[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) hist[c] = 0;
    for (int64_t i = s; i < e; ++i) {
      const int64_t p = perm[i];
      const f32x4 q = *reinterpret_cast<const f32x4 *>(pts + p * 4);
      sx += q.x; sy += q.y; sz += q.z; se += q.w;
      if (labels) {
        const int64_t l = labels[p];
        if (l >= 0 && l < C) ++hist[l];
      }
      vox_of_point[p] = v;
    }
    const float n = (float)(e - s);
    vpts[v] = f32x4{sx / n, sy / n, sz / n, se};
    int best = -1, bc = 0;
    for (int c = 0; c < C; ++c)
      if (hist[c] > bc) { bc = hist[c]; best = c; }
    if (vlab) vlab[v] = best;
    if (vcount) vcount[v] = e - s;
  }
  (void)keys;
}

// vox_offsets[b] = first voxel of scene b (keys sorted scene-major); vox_offsets[B] = V
__global__ __launch_bounds__(THREADS) void vox_offsets_kernel(const uint64_t *__restrict__ skeys,
                                                              const int64_t *__restrict__ start,
                                                              const int64_t *__restrict__ nvox, int B, uint64_t G3,
                                                              int64_t *__restrict__ vox_offsets) {
  const int b = blockIdx.x * THREADS + threadIdx.x;
  if (b > B) return;
  const int64_t V = *nvox;
  int64_t lo = 0, hi = V;   // first voxel whose scene >= b
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (skeys[start[mid]] / G3 < (uint64_t)b) lo = mid + 1; else hi = mid;
  }
  vox_offsets[b] = lo;
}

__global__ __launch_bounds__(THREADS) void gather_rows_kernel(const float *__restrict__ src, int64_t ld_src,
                                                              const int64_t *__restrict__ idx, int64_t n, int C,
                                                              float *__restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n * C; i += (int64_t)gridDim.x * THREADS) {
    const int64_t r = i / C;
    const int c = (int)(i - r * C);
    dst[i] = src[idx[r] * ld_src + c];
  }
}

// padded row (scene b, slot v - vox_offsets[b]) of each point's voxel in a [B, scene_rows] batch
__global__ __launch_bounds__(THREADS) void padded_index_kernel(const int64_t *__restrict__ vop, int64_t T,
                                                               const int64_t *__restrict__ voff, int B,
                                                               int64_t scene_rows, int64_t *__restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * THREADS + threadIdx.x; t < T; t += (int64_t)gridDim.x * THREADS) {
    const int64_t v = vop[t];
    int lo = 0, hi = B;   // last b with voff[b] <= v
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (voff[mid] <= v) lo = mid; else hi = mid;
    }
    out[t] = (int64_t)lo * scene_rows + (v - voff[lo]);
  }
}

int blocks(int64_t n) { return (int)pcs_max64(1, pcs_min64(8192, (n + THREADS - 1) / THREADS)); }

struct VoxWs {   // workspace carve-up (all 256-B aligned)
  uint64_t *keys, *skeys;
  int64_t *vals, *perm, *flags, *seg, *start;
  void *tmp;
  size_t tmp_bytes;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int carve(void *ws, size_t ws_bytes, int64_t T, VoxWs &w, size_t *need) {
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                  (int64_t *)nullptr, (int64_t *)nullptr, (size_t)T, 0, 64);
  (void)rocprim::inclusive_scan(nullptr, scan_bytes, (int64_t *)nullptr, (int64_t *)nullptr, (size_t)T,
                                rocprim::plus<int64_t>());
  const size_t tmp = align256(sort_bytes > scan_bytes ? sort_bytes : scan_bytes);
  const size_t arr = align256((size_t)T * 8), starr = align256(((size_t)T + 1) * 8);
  const size_t total = 6 * arr + starr + tmp;
  if (need) *need = total;
  if (!ws) return 0;
  if (ws_bytes < total) return -1;
  char *p = static_cast<char *>(ws);
  w.keys = (uint64_t *)p; p += arr;
  w.skeys = (uint64_t *)p; p += arr;
  w.vals = (int64_t *)p; p += arr;
  w.perm = (int64_t *)p; p += arr;
  w.flags = (int64_t *)p; p += arr;
  w.seg = (int64_t *)p; p += arr;
  w.start = (int64_t *)p; p += starr;
  w.tmp = p;
  w.tmp_bytes = tmp;
  return 0;
}

}  // namespace

extern "C" int pcs_voxel_ids(const float *points, int64_t T, int32_t grid, float lo_x, float lo_y, float lo_z,
                             float hi_x, float hi_y, float hi_z, int64_t *ids, pcs_stream_t stream) {
  if (!points || !ids || T < 0 || grid < 1 || grid > (1 << 20) || !(hi_x > lo_x) || !(hi_y > lo_y) || !(hi_z > lo_z))
    return pcs_set_einval("pcs_voxel_ids", "bad arguments (grid in [1, 2^20], hi > lo)");
  if (T == 0) return 0;
  const Box b = {{lo_x, lo_y, lo_z}, {hi_x, hi_y, hi_z}};
  hipLaunchKernelGGL(voxel_ids_kernel, dim3(blocks(T)), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     points, T, (int)grid, b, ids);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t pcs_voxelize_workspace(int64_t T) {
  if (T < 0) return pcs_set_einval("pcs_voxelize_workspace", "T < 0");
  VoxWs w;
  size_t need = 0;
  carve(nullptr, 0, T, w, &need);
  return (int64_t)need;
}

extern "C" int pcs_voxelize(const float *points, const int64_t *labels, const int64_t *offsets, int64_t num_scenes,
                            int64_t T, int32_t grid, float lo_x, float lo_y, float lo_z, float hi_x, float hi_y,
                            float hi_z, int32_t num_classes, void *workspace, int64_t workspace_bytes,
                            int64_t *voxel_of_point, float *vox_points, int64_t *vox_labels, int64_t *vox_counts,
                            int64_t *vox_offsets, int64_t *num_voxels, pcs_stream_t stream) {
  if (!points || !offsets || !voxel_of_point || !vox_points || !vox_offsets || !num_voxels || !workspace ||
      num_scenes < 1 || T < 1 || grid < 1 || !(hi_x > lo_x) || !(hi_y > lo_y) || !(hi_z > lo_z) ||
      num_classes < 1 || num_classes > 16 || (reinterpret_cast<uintptr_t>(points) & 15) ||
      (reinterpret_cast<uintptr_t>(vox_points) & 15))
    return pcs_set_einval("pcs_voxelize", "bad arguments (T >= 1, 1 <= num_classes <= 16, 16-B aligned points)");
  const double G3 = (double)grid * grid * grid;
  if (G3 * (double)num_scenes >= 18446744073709551615.0) return pcs_set_einval("pcs_voxelize", "key overflow");
  VoxWs w;
  if (carve(workspace, (size_t)workspace_bytes, T, w, nullptr)) return pcs_set_einval("pcs_voxelize", "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const Box b = {{lo_x, lo_y, lo_z}, {hi_x, hi_y, hi_z}};
  hipLaunchKernelGGL(voxel_keys_kernel, dim3(blocks(T)), dim3(THREADS), 0, s, points, offsets, (int)num_scenes, T,
                     (int)grid, b, w.keys, w.vals);
  PCS_CHECK_LAUNCH();
  int bits = 1;
  while (bits < 64 && (double)(1ull << bits) < G3 * (double)num_scenes) ++bits;
  size_t tb = w.tmp_bytes;
  if (rocprim::radix_sort_pairs(w.tmp, tb, w.keys, w.skeys, w.vals, w.perm, (size_t)T, 0, bits, s) != hipSuccess)
    return pcs_set_einval("pcs_voxelize", "radix sort failed");
  hipLaunchKernelGGL(head_flags_kernel, dim3(blocks(T)), dim3(THREADS), 0, s, w.skeys, T, w.flags);
  PCS_CHECK_LAUNCH();
  tb = w.tmp_bytes;
  if (rocprim::inclusive_scan(w.tmp, tb, w.flags, w.seg, (size_t)T, rocprim::plus<int64_t>(), s) != hipSuccess)
    return pcs_set_einval("pcs_voxelize", "scan failed");
  hipLaunchKernelGGL(seg_starts_kernel, dim3(blocks(T)), dim3(THREADS), 0, s, w.seg, T, w.start, num_voxels);
  PCS_CHECK_LAUNCH();
  hipLaunchKernelGGL(aggregate_kernel, dim3(blocks(T)), dim3(THREADS), 0, s, points, labels, w.skeys, w.perm, w.start,
                     num_voxels, (int)num_classes, reinterpret_cast<f32x4 *>(vox_points), vox_labels, vox_counts,
                     voxel_of_point);
  PCS_CHECK_LAUNCH();
  hipLaunchKernelGGL(vox_offsets_kernel, dim3((int)((num_scenes + 1 + THREADS - 1) / THREADS)), dim3(THREADS), 0, s,
                     w.skeys, w.start, num_voxels, (int)num_scenes, (uint64_t)G3, vox_offsets);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_gather_rows(const float *src, int64_t ld_src, const int64_t *idx, int64_t n, int32_t C,
                               float *dst, pcs_stream_t stream) {
  if (!src || !idx || !dst || n < 0 || C < 1 || ld_src < C) return pcs_set_einval("pcs_gather_rows", "bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks(n * C)), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     src, ld_src, idx, n, (int)C, dst);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_voxel_padded_index(const int64_t *voxel_of_point, int64_t T, const int64_t *vox_offsets,
                                      int64_t num_scenes, int64_t scene_rows, int64_t *out, pcs_stream_t stream) {
  if (!voxel_of_point || !vox_offsets || !out || T < 0 || num_scenes < 1 || scene_rows < 0)
    return pcs_set_einval("pcs_voxel_padded_index", "bad arguments");
  if (T == 0) return 0;
  hipLaunchKernelGGL(padded_index_kernel, dim3(blocks(T)), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     voxel_of_point, T, vox_offsets, (int)num_scenes, scene_rows, out);
  PCS_CHECK_LAUNCH();
  return 0;
}

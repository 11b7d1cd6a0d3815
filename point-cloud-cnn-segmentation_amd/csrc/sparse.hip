// Occupied-voxel (sparse) indexing for the north star's "sparse occupied-only voxel path
// (hash-indexed gather)" (BASELINE configs[2]).  Build-defined: the reference has no
// voxel grid, so the oracle is oracle/sparse_oracle.py (numpy, dict-based), "not reference parity".
//
//   key          scene * G^3 + (ix * G + iy) * G + iz, the voxel key of voxel.hip
//   hash table   open addressing over a power-of-two capacity (>= 2 n): slot = mix(key) & (cap-1),
//                linear probing; keys inserted with a 64-bit compare-and-swap, the value is the
//                voxel's row.  Keys are unique, so the final table (which slot holds which key)
//                can depend on insertion order but every lookup result cannot.
//   neighbours   nbr[v][t] = row of the voxel at (ix + a - 1, iy + b - 1, iz + c - 1) of the same
//                scene, t = (a * 3 + b) * 3 + c, or -1 (empty or outside the grid): the 27 taps of
//                a 3x3x3 submanifold convolution in the tap order of a torch Conv3d weight
//                [Cout, Cin, 3, 3, 3] applied to a dense [B, C, G(x), G(y), G(z)] grid.
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr uint64_t EMPTY = ~0ull;

PCS_DEV uint64_t mix64(uint64_t k) {   // splitmix64 finaliser
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

PCS_DEV int64_t voxel_of(const float *p, int G, const float *lo, const float *hi) {
  int64_t id = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {   // the expression order of voxel.hip (bit-exact ids)
    const float t = (p[d] - lo[d]) / (hi[d] - lo[d]);
    int i = (int)floorf(t * (float)G);
    i = i < 0 ? 0 : (i > G - 1 ? G - 1 : i);
    id = id * G + i;
  }
  return id;
}

struct Box {
  float lo[3], hi[3];
};

// keys[voxel_of_point[p]] = key of p (every point of a voxel writes the same value)
__global__ __launch_bounds__(THREADS) void voxel_keys_kernel(const float *__restrict__ pts,
                                                             const int64_t *__restrict__ offsets, int B, int64_t T,
                                                             int G, Box b, const int64_t *__restrict__ vop,
                                                             uint64_t *__restrict__ keys) {
  const uint64_t G3 = (uint64_t)G * G * G;
  for (int64_t t = (int64_t)blockIdx.x * THREADS + threadIdx.x; t < T; t += (int64_t)gridDim.x * THREADS) {
    int lo = 0, hi = B;   // scene: last b with offsets[b] <= t
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offsets[mid] <= t) lo = mid; else hi = mid;
    }
    keys[vop[t]] = (uint64_t)lo * G3 + (uint64_t)voxel_of(pts + t * 4, G, b.lo, b.hi);
  }
}

__global__ __launch_bounds__(THREADS) void hash_clear_kernel(uint64_t *__restrict__ tk, int32_t *__restrict__ tv, int64_t cap) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < cap; i += (int64_t)gridDim.x * THREADS) {
    tk[i] = EMPTY;
    tv[i] = -1;
  }
}

// every probe sequence ends: the capacity is at least twice the key count, so an empty slot or
// the key itself is always found within cap probes
__global__ __launch_bounds__(THREADS) void hash_insert_kernel(const uint64_t *__restrict__ keys, int64_t n,
                                                              unsigned long long *__restrict__ tk,
                                                              int32_t *__restrict__ tv, uint64_t mask) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * THREADS) {
    const uint64_t k = keys[i];
    uint64_t h = mix64(k) & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
      const unsigned long long prev = atomicCAS(tk + h, (unsigned long long)EMPTY, (unsigned long long)k);
      if (prev == EMPTY || prev == k) {
        tv[h] = (int32_t)i;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

PCS_DEV int32_t hash_find(const uint64_t *__restrict__ tk, const int32_t *__restrict__ tv, uint64_t mask, uint64_t k) {
  uint64_t h = mix64(k) & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const uint64_t s = tk[h];
    if (s == k) return tv[h];
    if (s == EMPTY) return -1;
    h = (h + 1) & mask;
  }
  return -1;
}

__global__ __launch_bounds__(THREADS) void hash_find_kernel(const uint64_t *__restrict__ tk, const int32_t *__restrict__ tv,
                                                            uint64_t mask, const uint64_t *__restrict__ q, int64_t nq,
                                                            int32_t *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < nq; i += (int64_t)gridDim.x * THREADS)
    out[i] = hash_find(tk, tv, mask, q[i]);
}

// one thread per (voxel, tap)
__global__ __launch_bounds__(THREADS) void neighbors_kernel(const uint64_t *__restrict__ tk, const int32_t *__restrict__ tv,
                                                            uint64_t mask, const uint64_t *__restrict__ keys, int64_t n,
                                                            int G, int32_t *__restrict__ nbr) {
  const uint64_t G3 = (uint64_t)G * G * G;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < n * 27; i += (int64_t)gridDim.x * THREADS) {
    const int64_t v = i / 27;
    const int t = (int)(i - v * 27);
    const uint64_t k = keys[v];
    const uint64_t scene = k / G3, loc = k - scene * G3;
    const int ix = (int)(loc / ((uint64_t)G * G)), iy = (int)((loc / G) % G), iz = (int)(loc % G);
    const int jx = ix + t / 9 - 1, jy = iy + (t / 3) % 3 - 1, jz = iz + t % 3 - 1;
    int32_t r = -1;
    if (jx >= 0 && jx < G && jy >= 0 && jy < G && jz >= 0 && jz < G)
      r = hash_find(tk, tv, mask, scene * G3 + ((uint64_t)jx * G + jy) * G + jz);
    nbr[i] = r;
  }
}

int blocks_for_n(int64_t n) {
  const int64_t b = (n + THREADS - 1) / THREADS;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

extern "C" int pcs_voxel_keys(const float *points, const int64_t *offsets, int64_t num_scenes, int64_t T, int32_t grid,
                              float lo_x, float lo_y, float lo_z, float hi_x, float hi_y, float hi_z,
                              const int64_t *voxel_of_point, uint64_t *keys, pcs_stream_t stream) {
  if (!points || !offsets || !voxel_of_point || !keys || num_scenes < 1 || T < 0 || grid < 1 || grid > (1 << 20) ||
      !(hi_x > lo_x && hi_y > lo_y && hi_z > lo_z))
    return pcs_set_einval("pcs_voxel_keys", "bad arguments");
  // keys are scene * G^3 + voxel: they must stay below the hash table's EMPTY sentinel (2^64 - 1)
  if ((double)grid * grid * grid * (double)num_scenes >= 18446744073709551615.0)
    return pcs_set_einval("pcs_voxel_keys", "key overflow (num_scenes * grid^3 >= 2^64 - 1)");
  if (T == 0) return 0;
  const Box b = {{lo_x, lo_y, lo_z}, {hi_x, hi_y, hi_z}};
  hipLaunchKernelGGL(voxel_keys_kernel, dim3(blocks_for_n(T)), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     points, offsets, (int)num_scenes, T, (int)grid, b, voxel_of_point, keys);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t pcs_voxel_hash_capacity(int64_t n) {
  if (n < 0 || n > ((int64_t)1 << 31)) return pcs_set_einval("pcs_voxel_hash_capacity", "0 <= n <= 2^31");
  int64_t cap = 64;
  while (cap < 2 * n) cap <<= 1;
  return cap;
}

extern "C" int pcs_voxel_hash_build(const uint64_t *keys, int64_t n, uint64_t *table_keys, int32_t *table_vals,
                                    int64_t capacity, pcs_stream_t stream) {
  if ((!keys && n > 0) || !table_keys || !table_vals || n < 0 || capacity < 2 * n || capacity < 1 ||
      (capacity & (capacity - 1)) != 0)
    return pcs_set_einval("pcs_voxel_hash_build", "bad arguments (capacity: a power of two >= 2 n)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(hash_clear_kernel, dim3(blocks_for_n(capacity)), dim3(THREADS), 0, s, table_keys, table_vals, capacity);
  if (n > 0)
    hipLaunchKernelGGL(hash_insert_kernel, dim3(blocks_for_n(n)), dim3(THREADS), 0, s, keys, n,
                       reinterpret_cast<unsigned long long *>(table_keys), table_vals, (uint64_t)(capacity - 1));
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_voxel_hash_find(const uint64_t *table_keys, const int32_t *table_vals, int64_t capacity,
                                   const uint64_t *queries, int64_t nq, int32_t *out, pcs_stream_t stream) {
  if (!table_keys || !table_vals || (!queries && nq > 0) || (!out && nq > 0) || nq < 0 || capacity < 1 ||
      (capacity & (capacity - 1)) != 0)
    return pcs_set_einval("pcs_voxel_hash_find", "bad arguments");
  if (nq == 0) return 0;
  hipLaunchKernelGGL(hash_find_kernel, dim3(blocks_for_n(nq)), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     table_keys, table_vals, (uint64_t)(capacity - 1), queries, nq, out);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_sparse_neighbors(const uint64_t *table_keys, const int32_t *table_vals, int64_t capacity,
                                    const uint64_t *keys, int64_t n, int32_t grid, int32_t *nbr, pcs_stream_t stream) {
  if (!table_keys || !table_vals || (!keys && n > 0) || (!nbr && n > 0) || n < 0 || grid < 1 || grid > (1 << 20) ||
      capacity < 1 || (capacity & (capacity - 1)) != 0)
    return pcs_set_einval("pcs_sparse_neighbors", "bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(neighbors_kernel, dim3(blocks_for_n(n * 27)), dim3(THREADS), 0,
                     reinterpret_cast<hipStream_t>(stream), table_keys, table_vals, (uint64_t)(capacity - 1), keys, n,
                     (int)grid, nbr);
  PCS_CHECK_LAUNCH();
  return 0;
}

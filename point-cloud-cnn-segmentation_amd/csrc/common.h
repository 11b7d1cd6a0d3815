// Shared device helpers for the pcs HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pcs.h"

#define PCS_DEV __device__ __forceinline__
#define PCS_DEV_FWD __device__ __forceinline__
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short bf16_t;  // storage type of one bf16 element
// 16-byte chunk as a native vector: HIP's uint4 is a struct whose plain copies lower to
// memcpy through a private alloca (scratch); an ext_vector stays in VGPRs.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
PCS_DEV u32x4 mk_u32x4(unsigned a, unsigned b, unsigned c, unsigned d) {
  u32x4 v = {a, b, c, d};
  return v;
}

#ifndef PCS_NT_STORE
#define PCS_NT_STORE 1   // streamed GEMM outputs stored non-temporal (nt): they outgrow L2 / MALL
#endif
// one 16-B store of a streamed activation / gradient row chunk (read back only by a later kernel)
PCS_DEV void st16(void *p, u32x4 v) {
#if PCS_NT_STORE
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
#else
  *reinterpret_cast<u32x4 *>(p) = v;
#endif
}


// ---------------------------------------------------------------------------------------
// element traits: T = float (parity path, f32 MFMA) or bf16_t (bench path, bf16 MFMA)
// EPC = elements per 16-byte chunk
// ---------------------------------------------------------------------------------------
template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int EPC = 4;
  static constexpr int SIZE = 4;
};
template <> struct Elem<bf16_t> {
  static constexpr int EPC = 8;
  static constexpr int SIZE = 2;
};

PCS_DEV float bf2f(uint32_t u16) { return __uint_as_float(u16 << 16); }

PCS_DEV uint32_t pack2bf(float a, float b) {
  f32x2 v = {a, b};
  bf16x2 h = __builtin_convertvector(v, bf16x2);
  return __builtin_bit_cast(uint32_t, h);
}

// 16-byte chunk <-> float[EPC]
PCS_DEV void unpack_chunk(const u32x4 &c, float (&v)[4]) {
  v[0] = __uint_as_float(c.x); v[1] = __uint_as_float(c.y);
  v[2] = __uint_as_float(c.z); v[3] = __uint_as_float(c.w);
}
PCS_DEV void unpack_chunk(const u32x4 &c, float (&v)[8]) {
  v[0] = bf2f(c.x & 0xffffu); v[1] = bf2f(c.x >> 16);
  v[2] = bf2f(c.y & 0xffffu); v[3] = bf2f(c.y >> 16);
  v[4] = bf2f(c.z & 0xffffu); v[5] = bf2f(c.z >> 16);
  v[6] = bf2f(c.w & 0xffffu); v[7] = bf2f(c.w >> 16);
}
PCS_DEV u32x4 pack_chunk(const float (&v)[4]) {
  return mk_u32x4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                    __float_as_uint(v[3]));
}
PCS_DEV u32x4 pack_chunk(const float (&v)[8]) {
  return mk_u32x4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]),
                    pack2bf(v[6], v[7]));
}

PCS_DEV float load_elem(const float *p, int64_t i) { return p[i]; }
PCS_DEV float load_elem(const bf16_t *p, int64_t i) { return bf2f(p[i]); }

// fp8 e4m3 (OCP e4m3fn on gfx950): one storage byte
typedef unsigned char fp8_t;
PCS_DEV float fp82f(uint32_t byte) { return __builtin_amdgcn_cvt_f32_fp8((int)byte, 0); }
PCS_DEV float load_elem(const fp8_t *p, int64_t i) { return fp82f(p[i]); }
// four floats -> four e4m3 bytes (round to nearest even; the hardware conversion saturates)
PCS_DEV uint32_t pack4fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

// load EPC floats of a small per-channel coefficient vector (L1/L2 resident)
template <int EPC>
PCS_DEV void load_vec(const float *__restrict__ p, int k, float (&v)[EPC]) {
#pragma unroll
  for (int e = 0; e < EPC; e += 4) {
    const float4 q = *reinterpret_cast<const float4 *>(p + k + e);
    v[e] = q.x; v[e + 1] = q.y; v[e + 2] = q.z; v[e + 3] = q.w;
  }
}

// dropout keep bit of element (row, k): bits packed 8 per byte along k.
PCS_DEV uint32_t mask_bits(const uint8_t *__restrict__ bits, int64_t row, int K, int k, int n) {
  // returns n (4 or 8) consecutive keep bits starting at k (k % n == 0)
  const uint32_t byte = bits[row * (K >> 3) + (k >> 3)];
  return n == 8 ? byte : ((byte >> (k & 7)) & 0xFu);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, then
// s_barrier.  Unlike __syncthreads() (a workgroup-scope fence) it never waits on vmcnt, so
// global loads issued for a later pipeline stage stay in flight across it (spill stores
// would otherwise make the fence drain them).  One asm statement with a "memory" clobber:
// the compiler moves no memory access across it.
PCS_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// wave-level helpers (wave64)
PCS_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Chan's parallel merge of (n, mean, M2) triples.
PCS_DEV void chan_merge(float &n, float &mean, float &m2, float nb, float meanb, float m2b) {
  const float nn = n + nb;
  if (nb == 0.f) return;
  if (n == 0.f) { n = nb; mean = meanb; m2 = m2b; return; }
  const float d = meanb - mean;
  const float f = nb / nn;
  mean += d * f;
  m2 += m2b + d * d * n * f;
  n = nn;
}

// ReLU as torch.relu: a NaN propagates.  __builtin_elementwise_maximum (IEEE 754-2019 maximum)
// lowers to v_maximum3_f32 on gfx950, issued at the v_max_f32 rate (4.6 against 4.5 cycles per
// wave-instruction, tools/probes/probe_maximum3.hip); fmaxf's maxNum would turn a NaN into 0, so a
// diverged run would report a finite loss where the reference reports NaN
PCS_DEV float relu(float x) { return __builtin_elementwise_maximum(x, 0.f); }

// x where the mask m is all ones, +0 where it is 0 (m = a sign-extended keep bit, v_bfe_i32):
// one v_and_b32.  In asm so that it stays a bitwise AND: hipcc rewrites x & sext(bit) into
// v_cmp + v_cndmask, whose SGPR hand-off also costs wait states (s_nop) -- 3-4 issue slots per
// element instead of 1 (r06: 128 v_cmp + 159 v_cndmask + 121 s_nop in the global_feat input
// gradient's epilogue per tile and wave)
PCS_DEV float and_mask(float x, uint32_t m) {
  float r;
  asm("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(m));
  return r;
}

// Max-pool candidate order of torch.max / torch.min over a dim (P:114): a NaN beats every
// number (torch propagates it), and among equal values -- or among NaNs -- the smaller row
// wins (the first one in row order).  (v, vi) is the candidate, (cur, ci) the running pick.
// (Bitwise on bools, so the selects stay branch-free: an ordered compare with a NaN operand
// is false, so the last two terms only ever hold between two numbers.)
PCS_DEV bool pool_max_wins(float v, int vi, float cur, int ci) {
  return ((v != v) & ((cur == cur) | (vi < ci))) | (v > cur) | ((v == cur) & (vi < ci));
}
PCS_DEV bool pool_min_wins(float v, int vi, float cur, int ci) {
  return ((v != v) & ((cur == cur) | (vi < ci))) | (v < cur) | ((v == cur) & (vi < ci));
}
// per-element running pick over ascending rows: a later row replaces the pick only when it is
// strictly greater (smaller) or the first NaN; the first row always makes a pick (ci is the
// 0x7fffffff "none yet" sentinel until then), so a column of -inf still gets its first row
constexpr int PCS_POOL_NONE = 0x7fffffff;
PCS_DEV bool pool_max_step(float v, float cur, int ci) {
  return (v > cur) | ((v != v) & (cur == cur)) | (ci == PCS_POOL_NONE);
}
PCS_DEV bool pool_min_step(float v, float cur, int ci) {
  return (v < cur) | ((v != v) & (cur == cur)) | (ci == PCS_POOL_NONE);
}

// row-tile geometry of one scene-aware chunk (rows never straddle scenes)
struct ChunkGeo {
  int64_t scene_rows;   // N: rows per scene (padded cloud length)
  int tiles_per_scene;  // ceil(N / BM)
  int tiles_per_chunk;
  int chunks_per_scene;
};

__host__ __device__ inline int64_t pcs_min64(int64_t a, int64_t b) { return a < b ? a : b; }
__host__ __device__ inline int64_t pcs_max64(int64_t a, int64_t b) { return a > b ? a : b; }

// Scene-aligned chunk geometry: fills a->chunks_per_scene (auto when <= 0, aiming at
// ~target workgroups over ncb column blocks) and returns rows per chunk.
inline int64_t pcs_fill_geometry(pcs_gemm_args *a, int64_t tile, int64_t target, int64_t ncb) {
  const int64_t tps = (a->scene_rows + tile - 1) / tile;
  int64_t cps = a->chunks_per_scene;
  if (cps <= 0) cps = (target + a->num_scenes * ncb - 1) / (a->num_scenes * ncb);
  if (cps > tps) cps = tps;
  if (cps < 1) cps = 1;
  const int64_t tpc = (tps + cps - 1) / cps;
  cps = (tps + tpc - 1) / tpc;  // no empty chunks
  a->chunks_per_scene = (int32_t)cps;
  return tpc * tile;
}

// wide-layer bf16 kernel (gemm_big.hip)
bool pcs_gemm_big_applicable(const pcs_gemm_args &a);
int pcs_gemm_big_launch(const pcs_gemm_args &a, int tiles_per_scene, int tiles_per_chunk,
                        hipStream_t s);
constexpr int PCS_BIG_BM = 256;
// LDS-DMA 256x256 kernel for the RAW-operand global_feat GEMMs (gemm_glds.hip)
bool pcs_gemm_glds_applicable(const pcs_gemm_args &a);
// gemm_wres.hip: W-resident LDS-DMA stream for conv5's BN+ReLU pass with an fp8 store (K = 128)
bool pcs_gemm_wres_applicable(const pcs_gemm_args &a);
int pcs_gemm_wres_launch(const pcs_gemm_args &g, int64_t rows_per_chunk, hipStream_t s);
int pcs_gemm_glds_launch(const pcs_gemm_args &a, int tiles_per_scene, int tiles_per_chunk,
                         hipStream_t s);
// fused seg_conv2 / seg_conv3 input + weight gradient (fused_seg4.hip)
bool pcs_seg4_applicable(const pcs_gemm_args &a);
int64_t pcs_seg4_geometry(pcs_gemm_args *a);
int pcs_seg4_launch(const pcs_gemm_args &a, float *wpart, hipStream_t s);
// conv5's folded input gradient as one LDS-DMA stream (fused_c5.hip)
bool pcs_c5_dgrad_class(const pcs_gemm_args &a);
bool pcs_c5_dgrad_applicable(const pcs_gemm_args &a);
int pcs_c5_dgrad_launch(const pcs_gemm_args &a, int64_t rows_per_chunk, hipStream_t s);
// streaming forward of the narrow-K BN+ReLU layers (fwd_stream.hip): output columns per
// workgroup (0 = not this kernel's class; shapes only, the chunk geometry), applicability, launch
int pcs_fwd_stream_nb(const pcs_gemm_args &a, int *target_workgroups);
bool pcs_fwd_stream_applicable(const pcs_gemm_args &a);
int pcs_fwd_stream_launch(const pcs_gemm_args &a, int64_t rows_per_chunk, hipStream_t s);
// the streamed CE head (head_stream.hip; pcs_head): class (shapes / modes), grid target, launch
bool pcs_head_stream_class(const pcs_head_args &a);
int pcs_head_stream_target();
int pcs_head_stream_launch(const pcs_head_args &a, int64_t rows_per_chunk, hipStream_t s);
// the Gram of relu(bn(Y)) at C = 128 in one pass over Y (wgrad_c5.hip; pcs_gram)
bool pcs_gram128_class(const pcs_wgrad_args &a);
bool pcs_gram128_applicable(const pcs_wgrad_args &a);
int pcs_gram128_splits(const pcs_wgrad_args &a);
int pcs_gram128_launch(const pcs_wgrad_args &a, hipStream_t s);
// conv5's R = dz5^T relu(bn4(y4)) as an LDS-DMA stream (wgrad_c5.hip)
bool pcs_wgrad_c5_class(const pcs_wgrad_args &a);
bool pcs_wgrad_c5_applicable(const pcs_wgrad_args &a);
int pcs_wgrad_c5_splits(const pcs_wgrad_args &a);
int pcs_wgrad_c5_launch(const pcs_wgrad_args &a, int64_t rows_per_split, hipStream_t s);
// wide-layer bf16 weight-gradient kernel (gemm_big_tn.hip)
bool pcs_wgrad_big_applicable(const pcs_wgrad_args &a);
int pcs_wgrad_big_splits(const pcs_wgrad_args &a);
int pcs_wgrad_big_launch(const pcs_wgrad_args &a, hipStream_t s);

#define PCS_CHECK_LAUNCH()                                     \
  do {                                                         \
    hipError_t _e = hipGetLastError();                         \
    if (_e != hipSuccess) return pcs_set_error(_e, __func__);  \
  } while (0)

int pcs_set_error(hipError_t e, const char *where);
int pcs_set_einval(const char *where, const char *msg);

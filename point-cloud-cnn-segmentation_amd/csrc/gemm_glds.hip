// bf16 256x256 points-major GEMM with LDS-DMA staging (global_load_lds_dwordx4) and an
// 8-phase software pipeline, for the two 1024-deep GEMMs of global_feat, whose operand is
// the materialised a5 = relu(bn5(y5)) (no prologue transform, so the operand goes
// HBM -> LDS without passing through registers):
//   forward   y_g = a5 Wg^T            epilogue: max-pool partials (P:113-114), optionally BN
//             statistics (the bf16 / fp8 training path takes them from the Gram of a5 instead
//             and passes W's rows pre-multiplied by sign(gamma_g), PCS_FLAG_POOL_SIGNED_W)
//   backward  dA5 = a5 H + c  with H = Wg^T diag(gamma_g) Wg, c = Wg^T beta_g (pcs_bn_fold),
//             the ReLU mask of bn5 read from the operand itself, S1 = sum dz per column
//             (autograd of P:110-114, P:254); the max-pool rows' sparse term is added after
//             the kernel by pcs_pool_rows_add: an ordinary global load in this epilogue makes
//             hipcc wait vmcnt(0), draining the LDS-DMA prefetch at every tile
//
// Structure (cdna_hip_programming.md §5, "The 256² 8-phase template"):
// * 8 waves as 2 (M) x 4 (N); each wave owns 128 x 64 outputs = 8 x 4 accumulators of
//   v_mfma_f32_16x16x32_bf16.  One K-tile (64 deep) is four phases of 16 MFMAs, one output
//   quadrant each: (rows lo, cols lo), (lo, hi), (hi, lo), (hi, hi).
// * LDS holds two K-tiles, each as four 16 KB regions (A-lo, A-hi, B-lo, B-hi: the lower /
//   upper halves of every wave's rows and columns), so a region is free as soon as its last
//   quadrant has read it: A-lo and B-lo after phase 1, B-hi after phase 2, A-hi after
//   phase 3.  One region is restaged per phase, about four phases ahead of its use, by two
//   glds per thread; waits are counted (vmcnt(10): five regions stay in flight, fewer on the
//   chunk's last two K-tiles, where nothing more is issued) and the
//   barriers are raw s_barriers, so the loads stay in flight across them.  The 16-B chunks
//   of a 128-B LDS row are XOR-swizzled by (row >> 1) & 7; glds writes LDS linearly, so the
//   swizzle is applied to the SOURCE address and again on the ds_read_b128 side (rule 21).
// * The pipeline runs across the row tiles of a workgroup's chunk without draining: the
//   epilogue works on the accumulators (DPP row reductions, per-wave running statistics in
//   LDS outside the staging area), so the next tile's first K-tiles load while it runs.
#include "common.h"

#include <type_traits>

namespace {

constexpr int THREADS = 512;
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int REG = 128 * BK * 2;                  // one region: 128 rows x 128 B
constexpr int KBUF = 4 * REG;                      // A-lo | A-hi | B-lo | B-hi
constexpr int STAGE_BYTES = 2 * KBUF;              // 128 KB
constexpr int OFF_RUN = STAGE_BYTES;               // [2 wm][256] float2: (mean, m2) | (S1, 0)
constexpr int OFF_BIAS = OFF_RUN + 2 * 256 * 8;    // [256] f32
constexpr int OFF_RUNN = OFF_BIAS + 256 * 4;       // [2] f32: rows merged per wave half
constexpr int OFF_UNI = OFF_RUNN + 16;             // 16 KB, per mode:
constexpr int OFF_POOL = OFF_UNI;                  //   FWD: [2][256] float4 max, argmax, min, argmin
constexpr int OFF_SGN = OFF_UNI + 2 * 256 * 16;    //        [256] f32 +1 / -1 (pool keeps max / min)
constexpr int OFF_CUR = OFF_SGN + 256 * 4;         //        [2][256] f32 running max of sgn * y
constexpr int OFF_MASK = OFF_UNI;                  //   DGRAD: 2 x [256 rows][8 words] ReLU mask bits
constexpr int LDS_BYTES = OFF_UNI + 2 * 256 * 8 * 4;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

enum { MODE_FWD = 0, MODE_DGRAD = 1 };

typedef __attribute__((address_space(3))) void lds_void_t;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

PCS_DEV void sbar() { __builtin_amdgcn_sched_barrier(0); }
// One LDS-DMA piece: 64 lanes x 16 B from sbase + voff (per lane) to lds_dst + 16*lane.  Inline
// asm (the §5.7 recipe) so that the compiler's own wait insertion neither drains these loads
// before unrelated LDS reads nor spills their 64-bit addresses: the kernel counts them itself.
PCS_DEV void glds16(const char *sbase, uint32_t voff, char *lds_dst) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(lds_void_t *)lds_dst;
  // (M0 not restored: hipcc never reads M0 in this file's kernels -- tests/test_asm_audit.py)
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0v)
               : "memory");
}
PCS_DEV void barrier_raw() {
  sbar();
  asm volatile("s_barrier" ::: "memory");
  sbar();
}
template <int N> PCS_DEV void wait_vm() {
  sbar();
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  sbar();
}
PCS_DEV void wait_lgkm0() {
  sbar();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  sbar();
}

// Butterfly over the 16 lanes of a DPP row (quad xor 1, quad xor 2, half-row mirror, row
// mirror): every lane of the row ends with the row's result.
template <int CTRL> PCS_DEV float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL> PCS_DEV int dppi(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
PCS_DEV float row_sum(float v) {
  v += dppf<0xB1>(v); v += dppf<0x4E>(v); v += dppf<0x141>(v);
  return v + dppf<0x140>(v);
}
PCS_DEV float row_max(float v) {   // maxNum: only for NaN-free operands
  v = fmaxf(v, dppf<0xB1>(v)); v = fmaxf(v, dppf<0x4E>(v)); v = fmaxf(v, dppf<0x141>(v));
  return fmaxf(v, dppf<0x140>(v));
}
PCS_DEV float row_min(float v) {
  v = fminf(v, dppf<0xB1>(v)); v = fminf(v, dppf<0x4E>(v)); v = fminf(v, dppf<0x141>(v));
  return fminf(v, dppf<0x140>(v));
}
// The pool's maxima propagate NaN, as torch.max does (P:114): v_maximum3_f32 (IEEE 754-2019
// maximum, gfx950) rather than v_max3_f32, whose maxNum drops a NaN operand.  Single
// instructions in asm: on MFMA results hipcc otherwise inserts a canonicalising v_max before
// each fmaxf (MI355X_MICROARCH 'Per-instruction cycle constants')
PCS_DEV float max3f(float a, float b, float c) {
  float r;
  asm volatile("v_maximum3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
PCS_DEV float max2f(float a, float b) {
  float r;
  asm volatile("v_maximum3_f32 %0, %1, %2, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
PCS_DEV float maxp(float a, float b) { return __builtin_elementwise_maximum(a, b); }
// 0 / 1 per 16-bit half: bf16 x > 0 <=> x > 0 as a signed 16-bit integer (-0 = 0x8000 is not)
PCS_DEV uint32_t pos01(uint32_t x, uint32_t one2) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0\n\tv_pk_min_i16 %0, %0, %2" : "=&v"(r) : "v"(x), "v"(one2));
  return r;
}
PCS_DEV int row_mini(int v) {
  v = min(v, dppi<0xB1>(v)); v = min(v, dppi<0x4E>(v)); v = min(v, dppi<0x141>(v));
  return min(v, dppi<0x140>(v));
}

// region row q (0..127) -> tile row (A regions) / weight row (B regions)
PCS_DEV int a_row(int hi, int q) { return (q & 63) + ((q >> 6) << 7) + (hi ? 64 : 0); }
PCS_DEV int b_row(int hi, int q) { return (q & 31) + ((q >> 5) << 6) + (hi ? 32 : 0); }
PCS_DEV int swz(int q, int chunk) { return chunk ^ ((q >> 1) & 7); }

// FP8 (PCS_FLAG_AW_FP8): A and W are e4m3 bytes, a K-tile is 128 elements (the same 128-B
// rows), one v_mfma_scale_f32_16x16x128_f8f6f4 replaces the two bf16 16x16x32 of a (i, j)
// pair (2x the MFMA rate); each weight row's E8M0 scale is replicated into the four scale
// bytes of every lane holding that row (the MX blocks of a row share it), A is unscaled.
// Both operands use the same lane -> k map (32 consecutive bytes at k = 32 (lane >> 4)), which
// is all a dot product over k needs.
template <int MODE, bool FP8>
__global__ __launch_bounds__(THREADS) void gemm_glds_kernel(pcs_gemm_args a, int tiles_per_scene,
                                                            int tiles_per_chunk, int ncb) {
  constexpr int ESZ = FP8 ? 1 : 2;
  constexpr int KT = 128 / ESZ;                    // K per K-tile (128-byte LDS rows)
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float2 *run = reinterpret_cast<float2 *>(lds + OFF_RUN);
  float4 *runp = reinterpret_cast<float4 *>(lds + OFF_POOL);
  float *lbias = reinterpret_cast<float *>(lds + OFF_BIAS);
  float *runn = reinterpret_cast<float *>(lds + OFF_RUNN);
  float *lsgn = reinterpret_cast<float *>(lds + OFF_SGN);
  float *lcur = reinterpret_cast<float *>(lds + OFF_CUR);
  uint32_t *mbits = reinterpret_cast<uint32_t *>(lds + OFF_MASK);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = L / ncb, cb = L % ncb;
  const int cps = a.chunks_per_scene;
  const int scene = chunk / cps, cis = chunk % cps;
  const int n0 = cb * BN;
  const int K = a.K, Ncols = a.Ncols;
  const int64_t N = a.scene_rows;
  const int t_begin = cis * tiles_per_chunk;
  const int t_end = min(t_begin + tiles_per_chunk, tiles_per_scene);
  if (t_begin >= t_end) return;   // uniform across the workgroup
  const int nks = K / KT;
  const int total = (t_end - t_begin) * nks;
  // FWD: the chunk's row tiles are visited in the order t -> (t * P) mod n (P prime, not dividing
  // n): spatially ordered clouds make a column's running maximum grow tile after tile, which
  // sends the pool epilogue down its slow path on most tiles; a strided order samples the whole
  // chunk early, so the running maxima settle after a few tiles.  DGRAD keeps the identity.
  const int ntl = t_end - t_begin;
  int P = 1;
  if (MODE == MODE_FWD && ntl > 8) {
    constexpr int primes[6] = {97, 89, 83, 79, 73, 71};
#pragma unroll
    for (int i = 5; i >= 0; --i)
      if (primes[i] < ntl && ntl % primes[i] != 0) P = primes[i];
    P = __builtin_amdgcn_readfirstlane(P);
  }
  auto pnext = [&](int pt) { return pt + P >= ntl ? pt + P - ntl : pt + P; };   // perm(t + 1) from perm(t)
  const int64_t row0 = (int64_t)scene * N + (int64_t)t_begin * BM;
  const int64_t scene_end = (int64_t)(scene + 1) * N;
  const char *Ab = reinterpret_cast<const char *>(a.A);
  const char *Wb = reinterpret_cast<const char *>(a.W) + (int64_t)n0 * K * ESZ;
  const int64_t rowbytes = (int64_t)K * ESZ;
  int wsc[4] = {0, 0, 0, 0};   // FP8: this lane's weight-row scales (rows wn*64 + j*16 + lr)
  if constexpr (FP8) {
#pragma unroll
    for (int j = 0; j < 4; ++j) wsc[j] = (int)a.w_scale[n0 + wn * 64 + j * 16 + lr] * 0x01010101;
  }

  // ---- per-workgroup constants -> LDS (ordinary loads, all retired before the first glds)
  const bool do_stats = a.stats != nullptr;
  const bool do_pool = MODE == MODE_FWD && a.pool != nullptr;
  const bool signed_w = (a.flags & PCS_FLAG_POOL_SIGNED_W) != 0;   // acc is already sgn * y
  if (tid < BN) {
    lbias[tid] = a.bias ? a.bias[n0 + tid] : 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) run[h * BN + tid] = make_float2(0.f, 0.f);
    if constexpr (MODE == MODE_FWD) {
      lsgn[tid] = (a.es && a.es[n0 + tid] < 0.f) ? -1.f : 1.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        runp[h * BN + tid] = make_float4(-__builtin_huge_valf(), __int_as_float(0x7fffffff),
                                         __builtin_huge_valf(), __int_as_float(0x7fffffff));
        lcur[h * BN + tid] = -__builtin_huge_valf();
      }
    }
  }
  if (tid < 2) runn[tid] = 0.f;
  __syncthreads();

  // ---- glds: piece g of wave w covers region rows (2w+g)*8 .. +8; lane -> row +lane/8,
  // LDS slot lane%8, which holds the logical 16-B chunk swz(row, lane%8) of the source row.
  // Addresses are a uniform (SGPR) base per K-tile plus a 32-bit per-lane byte offset.
  int qrow[2];
  uint32_t cbyte[2], boff[2][2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    qrow[g] = (2 * wid + g) * 8 + (lane >> 3);
    cbyte[g] = (uint32_t)swz(qrow[g], lane & 7) * 16u;
#pragma unroll
    for (int h = 0; h < 2; ++h) boff[h][g] = (uint32_t)b_row(h, qrow[g]) * (uint32_t)rowbytes + cbyte[g];
  }
  // (qseq, tl, kt): K-tile sequence number and its (row tile, K-tile) -- the loop keeps the
  // latter as counters, so the scalar path has no divisions
  auto issue = [&](int qseq, int tl, int kt, int region) {
    if (qseq >= total) return;   // nothing left to prefetch: the loop's tail waits shrink
                                 // to match (see the phase waits below)
    char *dst = lds + (qseq & 1) * KBUF + region * REG;
    if (region < 2) {
      const int64_t rb = row0 + (int64_t)tl * BM;
      const int valid = (int)pcs_min64(BM, scene_end - rb);
      const char *sb = Ab + rb * rowbytes + kt * 128;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const uint32_t tr = (uint32_t)min(a_row(region, qrow[g]), valid - 1);   // rows past the scene: clamped
        glds16(sb, tr * (uint32_t)rowbytes + cbyte[g], dst + (2 * wid + g) * 1024);
      }
    } else {
      const char *sb = Wb + kt * 128;
#pragma unroll
      for (int g = 0; g < 2; ++g)
        glds16(sb, boff[region - 2][g], dst + (2 * wid + g) * 1024);
    }
  };

  // ---- fragment reads (ds_read_b128 of the swizzled 16-B chunks): bf16 16x16x32 takes
  // chunk kk*4 + lg for k-step kk; fp8 16x16x128 takes chunks 2 lg, 2 lg + 1 (32 bytes)
  // bf16: two 4-dword fragments per (i) / (j), one per k-step; fp8: one 8-dword fragment
  typedef int v8i __attribute__((ext_vector_type(8)));
  u32x4 af[4][2], bfr[4][2];
  v8i af8[4], bf8[4];
  auto frag8 = [&](const char *p0, const char *p1) {
    const u32x4 lo = *reinterpret_cast<const u32x4 *>(p0), hi = *reinterpret_cast<const u32x4 *>(p1);
    return v8i{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  auto chunk_of = [&](int kk) { return FP8 ? 2 * lg + kk : kk * 4 + lg; };
  auto read_a = [&](int buf, int region) {
    const char *base = lds + buf * KBUF + region * REG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = wm * 64 + i * 16 + lr;
      if constexpr (FP8) {
        af8[i] = frag8(base + q * 128 + swz(q, chunk_of(0)) * 16, base + q * 128 + swz(q, chunk_of(1)) * 16);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          af[i][kk] = *reinterpret_cast<const u32x4 *>(base + q * 128 + swz(q, chunk_of(kk)) * 16);
      }
    }
  };
  auto read_b = [&](int buf, int region, int j0) {
    const char *base = lds + buf * KBUF + region * REG;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = wn * 32 + j * 16 + lr;
      if constexpr (FP8) {
        bf8[j0 + j] = frag8(base + q * 128 + swz(q, chunk_of(0)) * 16, base + q * 128 + swz(q, chunk_of(1)) * 16);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          bfr[j0 + j][kk] = *reinterpret_cast<const u32x4 *>(base + q * 128 + swz(q, chunk_of(kk)) * 16);
      }
    }
  };
  // DGRAD: the ReLU mask of bn5 comes from the operand (Yp == A, K == Ncols): the tile's
  // output columns n0 .. n0+255 are the k-columns of K-tiles (n0 >> 6) .. +3.  In phase 1 of
  // each of those K-tiles all 512 threads turn the staged a5 values into bits (thread: tile
  // row tid/2, 32 columns; bf16 x > 0 <=> sign clear and magnitude nonzero) in a per-tile-
  // parity LDS bitmap [256 rows][8 words] that the epilogue reads: the work is spread evenly
  // over all waves instead of stalling one wave column at the phase barriers.
  // region: 0 = A-lo (phase 1), 1 = A-hi (phase 4); thread: region row tid/4, 16 columns.  (r06:
  // reading A-hi with phase 3's fragment reads and forming the bits of each region one phase
  // later made the input gradient 0.4 ms slower, profiles/ab_r06/; they stay in one phase.)
  auto mask_load = [&](int buf, int region, u32x4 &v0, u32x4 &v1) {
    const int q = tid >> 2, h = tid & 3;
    const char *base = lds + buf * KBUF + region * REG + q * 128;
    v0 = *reinterpret_cast<const u32x4 *>(base + swz(q, h * 2) * 16);
    v1 = *reinterpret_cast<const u32x4 *>(base + swz(q, h * 2 + 1) * 16);
  };
  auto mask_bits = [&](int region, int kq, int par, const u32x4 &v0, const u32x4 &v1) {
    const int q = tid >> 2, h = tid & 3;
    const int t = a_row(region, q);
    uint32_t w = 0;
    if constexpr (FP8) {   // 32 columns (bytes) per thread: x > 0 <=> sign clear, 7 low bits nonzero
      // word d (columns 4d .. 4d + 3) flags each byte in its bit 7; shifting word d right by
      // 7 - d and OR-ing the 8 words puts column 4d + k at bit 8k + d (the epilogue's order)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const u32x4 &v = c ? v1 : v0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t x = v[d];
          const uint32_t pos = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) & ~x & 0x80808080u;
          w |= pos >> (7 - (4 * c + d));
        }
      }
      mbits[par * 2048 + t * 8 + kq * 4 + h] = w;
      return;
    }
    // bf16: two packed 16-bit ops per word give 0 / 1 per element (bit 0: element 2d, bit 16:
    // element 2d + 1); a chunk's 8 elements fold to one byte with the even elements in bits 0-3
    // and the odd ones in bits 4-7 (the epilogue reads that order)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const u32x4 &v = c ? v1 : v0;
      const uint32_t tb = pos01(v[0], 0x10001u) | (pos01(v[1], 0x10001u) << 1) | (pos01(v[2], 0x10001u) << 2) |
                         (pos01(v[3], 0x10001u) << 3);
      w |= ((tb | (tb >> 12)) & 0xffu) << (8 * c);
    }
    reinterpret_cast<uint16_t *>(mbits + par * 2048 + t * 8 + kq * 2)[h] = (uint16_t)w;
  };

  // accumulators start at the bias (zero without one): the epilogue needs no bias pass
  // (re-read from LDS at each reset rather than held in 16 VGPRs)
  auto bias_init = [&](f32x4 (&ac)[8][4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 bb = *reinterpret_cast<const f32x4 *>(lbias + wn * 64 + j * 16 + 4 * lg);
#pragma unroll
      for (int i = 0; i < 8; ++i) ac[i][j] = bb;
    }
  };
  f32x4 acc[8][4];
  bias_init(acc);
  auto mfma_quad = [&](int i0, int j0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (FP8) {
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              bf8[j0 + j], af8[i], acc[i0 + i][j0 + j], 0, 0, 0, wsc[j0 + j], 0, 0x7f7f7f7f);
        } else {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, bfr[j0 + j][kk]), __builtin_bit_cast(bf16x8, af[i][kk]),
                acc[i0 + i][j0 + j], 0, 0, 0);
        }
      }
  };

  // ---- prologue: K-tile 0 landed; A-lo, B-lo, B-hi of K-tile 1 in flight
  const int tl1 = nks == 1 ? pnext(0) : 0, kt1 = nks == 1 ? 0 : 1;   // K-tile 1 (row tile permuted)
  issue(0, 0, 0, 0); issue(0, 0, 0, 1); issue(0, 0, 0, 2); issue(0, 0, 0, 3);
  issue(1, tl1, kt1, 0); issue(1, tl1, kt1, 2); issue(1, tl1, kt1, 3);
  wait_vm<6>();
  barrier_raw();

  const int kq0 = n0 / KT;          // DGRAD: first K-tile holding this tile's mask columns
  constexpr unsigned NKQ = 256 / KT;  // DGRAD: K-tiles holding them (4 bf16, 2 fp8)
  float run_n = 0.f;                // rows of this wave's half merged so far (uniform)
  // The two wave halves run one barrier apart (the template's stagger): while the waves of
  // one half issue their MFMAs, the other half's ds_reads / glds / waits proceed, so each
  // SIMD (one wave of each half) keeps its matrix pipe busy.  Each wave retires its own
  // fragment reads before arriving at a phase's first barrier, which keeps the restaging of
  // a region one phase after its last read safe across the stagger.
  if (wm == 1) barrier_raw();
  // (No s_setprio around the MFMA sections: with the epilogues aligned, raising the MFMA
  // sections' priority over the partner's preparation measured 0.1-0.2 ms slower per GEMM, and
  // raising the preparation's instead no better; profiles/ab_r06/priority.txt)

  // (row tile, K-tile) of qs and of qs + 1; pcur / pa: their row tiles in visiting order
  int kt = 0, tcur = 0, ta = 0, ka = 0, pcur = 0, pa = 0;
  for (int qs = 0; qs < total; ++qs, kt = ka, tcur = ta, pcur = pa) {
    const int buf = qs & 1;
    // (row tile, K-tile) of qs + 1 and qs + 2
    const bool w1 = kt + 1 == nks;
    ta = w1 ? tcur + 1 : tcur;
    pa = w1 ? pnext(pcur) : pcur;
    ka = w1 ? 0 : kt + 1;
    const bool w2 = ka + 1 == nks;
    const int kb = w2 ? 0 : ka + 1;
    const int pb = w2 ? pnext(pa) : pa;
    // phase 1: (rows lo, cols lo); restage A-hi of K-tile qs+1
    const bool xmask = MODE == MODE_DGRAD && (unsigned)(kt - kq0) < NKQ;   // uniform
    u32x4 mv0, mv1;
    read_a(buf, 0);
    read_b(buf, 2, 0);
    if (xmask) {
      mask_load(buf, 0, mv0, mv1);
      mask_bits(0, kt - kq0, tcur & 1, mv0, mv1);
    }
    issue(qs + 1, pa, ka, 1);
    // every counted wait assumes the five regions issued after the one it retires are in
    // flight; on a chunk's last two K-tiles issue() skips loads, so the counts shrink to the
    // regions actually issued (phase 1 retires B-hi(qs): newer are A-hi(qs) and, unless qs is
    // the last K-tile, the four regions of qs+1)
    if (qs + 1 < total) wait_vm<10>(); else wait_vm<2>();
    wait_lgkm0();
    barrier_raw();
    mfma_quad(0, 0);
    barrier_raw();
    // phase 2: (lo, hi); restage A-lo of K-tile qs+2
    read_b(buf, 3, 2);
    issue(qs + 2, pb, kb, 0);
    // retires A-hi(qs): newer are the four regions of qs+1 and A-lo(qs+2)
    if (qs + 2 < total) wait_vm<10>(); else if (qs + 1 < total) wait_vm<8>(); else wait_vm<0>();
    wait_lgkm0();
    barrier_raw();
    mfma_quad(0, 2);
    barrier_raw();
    // phase 3: (hi, lo); restage B-lo of K-tile qs+2
    read_a(buf, 1);
    issue(qs + 2, pb, kb, 2);
    wait_lgkm0();
    barrier_raw();
    mfma_quad(4, 0);
    barrier_raw();
    // phase 4: (hi, hi); restage B-hi of K-tile qs+2.  A-hi's mask bits are taken here, not
    // in phase 3: B-lo's fragments are dead by now, which keeps the extraction's registers
    // out of the accumulators' way (A-hi(qs) is restaged only in phase 1 of qs+1)
    if (xmask) {
      mask_load(buf, 1, mv0, mv1);
      mask_bits(1, kt - kq0, tcur & 1, mv0, mv1);
    }
    issue(qs + 2, pb, kb, 3);
    // retires A-lo(qs+1), B-lo(qs+1): newer are B-hi(qs+1), A-hi(qs+1) and three of qs+2
    if (qs + 2 < total) wait_vm<10>(); else if (qs + 1 < total) wait_vm<4>(); else wait_vm<0>();
    barrier_raw();
    mfma_quad(4, 2);
    barrier_raw();

    if (kt != nks - 1) continue;

    // The halves meet for the epilogue (r06): staggered, half 1's epilogue would start only when
    // half 0's was done and its next MFMA phase began, so the two ran one after the other with
    // the SIMD's matrix pipe idle; aligned they run together and hide each other's latencies.
    // The stagger comes back after it (half 1 takes the extra barrier).
    if (wm == 0) barrier_raw();

    // ===================== epilogue of row tile tcur (rows of tile pcur) =====================
    const int64_t rb = row0 + (int64_t)pcur * BM;
    const int valid = (int)pcs_min64(BM, scene_end - rb);
    const int nvw = max(0, min(128, valid - wm * 128));   // valid rows of this wave's half
    // lane's columns c(j, r) = wn*64 + j*16 + 4*lg + r; rows m(i) = wm*128 + i*16 + lr
    uint32_t rowok = 0;   // bit i: row m(i) is a row of the scene
#pragma unroll
    for (int i = 0; i < 8; ++i) rowok |= (uint32_t)(wm * 128 + i * 16 + lr < valid) << i;
    const bool tile_full = valid == BM;   // uniform: only a scene's last tile is partial

    // after the 16-lane row reductions every lane of a row group holds its group's 16 column
    // results; lane lr then owns column e = lr of its group for the LDS bookkeeping
    const int cme = wm * BN + wn * 64 + (lr >> 2) * 16 + 4 * lg + (lr & 3);
    if constexpr (MODE == MODE_FWD) {
      if (nvw > 0) {
        if (do_stats) {
          // sums shifted by the half's running column mean, one Chan merge per column;
          // processed 4 columns (one j) at a time to keep registers for the accumulators
          float S1 = 0.f, S2 = 0.f, SH = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float sh[4], s1[4], s2[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              sh[r] = run[wm * BN + wn * 64 + j * 16 + 4 * lg + r].x;
              s1[r] = 0.f;
              s2[r] = 0.f;
            }
            if (tile_full) {
#pragma unroll
              for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const float d = acc[i][j][r] - sh[r];
                  s1[r] += d;
                  s2[r] = fmaf(d, d, s2[r]);
                }
            } else {
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                if ((rowok >> i) & 1u) {
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const float d = acc[i][j][r] - sh[r];
                    s1[r] += d;
                    s2[r] = fmaf(d, d, s2[r]);
                  }
                }
              }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              s1[r] = row_sum(s1[r]);
              s2[r] = row_sum(s2[r]);
              if (lr == j * 4 + r) { S1 = s1[r]; S2 = s2[r]; SH = sh[r]; }
            }
          }
          const float nt = (float)nvw, d1 = S1 / nt;
          float n = run_n, mean = run[cme].x, m2 = run[cme].y;
          chan_merge(n, mean, m2, nt, SH + d1, relu(S2 - S1 * d1));
          run[cme] = make_float2(mean, m2);
        }
        if (do_pool) {
          // only the extremum pool_finalize will use: max where es >= 0 (bn scale > 0), min
          // where es < 0, as the max of sgn * y.  Fast path: each lane compares its own 8-row
          // maxima with the half's running maxima (lcur, read 4 columns per ds_read_b128) and
          // the wave moves on unless some lane beats one -- after the first tiles of a chunk
          // that is rare, so the 16-lane reductions and the argmax search below (the slow
          // path) run on few tiles.
          const float *cur4 = lcur + wm * BN + wn * 64 + 4 * lg;
          const float *sgn4 = lsgn + wn * 64 + 4 * lg;
          uint32_t beat = 0;   // bit 4 j + r: this lane beats the running max of column (j, r)
          if (signed_w && tile_full) {
            // PCS_FLAG_POOL_SIGNED_W: acc = sgn * y, 4 max3/max per column and a compare
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float4 c4 = *reinterpret_cast<const float4 *>(cur4 + j * 16);
              const float cc[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float t0 = max3f(acc[0][j][r], acc[1][j][r], acc[2][j][r]);
                const float t1 = max3f(acc[3][j][r], acc[4][j][r], acc[5][j][r]);
                const float t2 = max3f(acc[6][j][r], acc[7][j][r], t0);
                // not <: an equal value may sit on an earlier row, and a NaN always beats
                beat |= (uint32_t)!(max2f(t1, t2) < cc[r]) << (4 * j + r);
              }
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float4 c4 = *reinterpret_cast<const float4 *>(cur4 + j * 16);
              const float4 g4 = *reinterpret_cast<const float4 *>(sgn4 + j * 16);
              const float cc[4] = {c4.x, c4.y, c4.z, c4.w};
              const float gg[4] = {signed_w ? 1.f : g4.x, signed_w ? 1.f : g4.y, signed_w ? 1.f : g4.z,
                                   signed_w ? 1.f : g4.w};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                float mx = -__builtin_huge_valf();
#pragma unroll
                for (int i = 0; i < 8; ++i)
                  if (tile_full || ((rowok >> i) & 1u)) mx = maxp(mx, gg[r] * acc[i][j][r]);
                beat |= (uint32_t)!(mx < cc[r]) << (4 * j + r);
              }
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (__builtin_amdgcn_ballot_w64((beat >> (4 * j)) & 0xFu) == 0) continue;   // uniform
            const float4 q = runp[cme];
            const float sgl = lsgn[cme - wm * BN];
            const float cur = sgl > 0.f ? q.x : -q.z;
            const int curix = __float_as_int(sgl > 0.f ? q.y : q.w);
            float vx[4], sg[4];
            float mine = -__builtin_huge_valf();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              sg[r] = signed_w ? 1.f : sgn4[j * 16 + r];
              vx[r] = -__builtin_huge_valf();
              // only the columns some lane beats (late in a chunk usually one of the four)
              if (__builtin_amdgcn_ballot_w64((beat >> (4 * j + r)) & 1u) == 0) continue;   // uniform
              float mx = -__builtin_huge_valf();
#pragma unroll
              for (int i = 0; i < 8; ++i)
                if (tile_full || ((rowok >> i) & 1u)) mx = maxp(mx, sg[r] * acc[i][j][r]);
              if (__builtin_amdgcn_ballot_w64(mx != mx) != 0) {   // uniform; rare (a diverged input)
                // a NaN in this column of the tile: torch.max's pick is the first NaN row; it
                // replaces a running number, or a running NaN on a later row (the tiles are not
                // visited in row order).  The running NaN makes every later tile take this slow
                // path, where a number never replaces it (mine >= NaN is false below).
                int ix = 0x7fffffff;
#pragma unroll
                for (int i = 7; i >= 0; --i)
                  if (((rowok >> i) & 1u) && acc[i][j][r] != acc[i][j][r]) ix = (int)(rb + wm * 128 + i * 16 + lr);
                ix = row_mini(ix);
                if (lr == j * 4 + r && (cur == cur || ix < curix)) {
                  float4 u = q;
                  if (sgl > 0.f) { u.x = __builtin_nanf(""); u.y = __int_as_float(ix); }
                  else { u.z = __builtin_nanf(""); u.w = __int_as_float(ix); }
                  runp[cme] = u;
                  lcur[cme] = __builtin_nanf("");
                }
                continue;
              }
              vx[r] = row_max(mx);
              if (lr == j * 4 + r) mine = vx[r];
            }
            // tiles are not visited in row order: an equal value replaces the running one when
            // its row is smaller (the first maximum, as in row order)
            const bool upd = (lr >> 2) == j && mine >= cur;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (__builtin_amdgcn_ballot_w64(upd && (lr & 3) == r) == 0) continue;
              int ix = 0x7fffffff;
#pragma unroll
              for (int i = 7; i >= 0; --i) {
                const float v = sg[r] > 0.f ? acc[i][j][r] : -acc[i][j][r];
                if (((rowok >> i) & 1u) && v == vx[r]) ix = (int)(rb + wm * 128 + i * 16 + lr);
              }
              ix = row_mini(ix);
              if (upd && (lr & 3) == r && (mine > cur || ix < curix)) {
                float4 u = q;
                if (sgl > 0.f) { u.x = vx[r]; u.y = __int_as_float(ix); }
                else { u.z = -vx[r]; u.w = __int_as_float(ix); }
                runp[cme] = u;
                lcur[cme] = vx[r];
              }
            }
          }
        }
        run_n += (float)nvw;
      }
    } else {   // MODE_DGRAD
      bf16_t *Cg = reinterpret_cast<bf16_t *>(a.C);
      const uint32_t *mrow = mbits + (tcur & 1) * 2048 + wn * 2;
      const bool full = valid == BM;   // uniform: only a scene's last tile is partial
      f32x2 s1[4][2] = {};   // columns (j, 2 h), (j, 2 h + 1) as a packed pair: v_pk_add_f32
      // Stores widened to 16 B (cdna_hip_programming.md T21 with v_permlane16_swap): a lane
      // holds 4 columns (8 B) of tile j; swapping tile j with tile j+1 between lane groups
      // 2h and 2h+1 leaves each lane 8 consecutive columns of tile j + (lg & 1), so every
      // store instruction writes 16 rows x 64 contiguous bytes instead of 16 x 32.
      const int scol = n0 + wn * 64 + 16 * (lg & 1) + 8 * (lg >> 1);
      // masking: v = acc & (0 - bit) (v_bfe_i32 sign-extends the keep bit to a full mask)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bool ok = full || ((rowok >> i) & 1u);
        const uint2 mw = *reinterpret_cast<const uint2 *>(mrow + (wm * 128 + i * 16 + lr) * 8);
        uint32_t pk[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // rows past the scene (a partial tile) get an all-zero mask word: their v is 0, so S1
          // sums v unconditionally (one select per word, not one per element); they are not stored
          // bf16 bitmap bytes: columns 8b + 2d at bit d, 8b + 2d + 1 at bit 4 + d (extract_mask);
          // the lane's columns 4 lg + r, r = 0..3, sit at bits {0, 4, 1, 5} after the shift
          // fp8 bitmap words: column e of the word's 32 at bit 8 (e % 4) + e / 4 (extract_mask);
          // the lane's columns 16 (j & 1) + 4 lg + r sit at bits 8 r after the shift
          const int word = ok ? (int)((j < 2 ? mw.x : mw.y) >> (FP8 ? 4 * (j & 1) + lg : (j & 1) * 16 + 8 * (lg >> 1) + 2 * (lg & 1))) : 0;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe(word, FP8 ? 8 * r : (r >> 1) + 4 * (r & 1), 1);
            v[r] = and_mask(acc[i][j][r], keep);
          }
          s1[j][0] += f32x2{v[0], v[1]};
          s1[j][1] += f32x2{v[2], v[3]};
          pk[j][0] = pack2bf(v[0], v[1]);
          pk[j][1] = pack2bf(v[2], v[3]);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const auto sw = __builtin_amdgcn_permlane16_swap(pk[2 * q][h], pk[2 * q + 1][h], false, false);
            pk[2 * q][h] = sw[0];
            pk[2 * q + 1][h] = sw[1];
          }
          if (ok)
            // plain store: dz5 is re-read right away by conv5's backward (nt measured 1 ms slower)
            *reinterpret_cast<u32x4 *>(Cg + (rb + wm * 128 + i * 16 + lr) * Ncols + scol + 32 * q) =
                mk_u32x4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);
        }
      }
      float S1 = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t = row_sum(s1[j][r >> 1][r & 1]);
          if (lr == j * 4 + r) S1 = t;
        }
      if (do_stats) run[cme].x += S1;
      // The stores count in vmcnt but are not waited for here: the next counted wait
      // (vmcnt(10), phase 1) only relies on the LOADS completing in order among themselves
      // (pending stores make it wait longer).  Counting the 16 stores in the next four waits
      // instead (so the loads need not wait for them) measured 0.15-0.25 ms SLOWER per call.
    }

    bias_init(acc);
    if (wm == 1) barrier_raw();   // the stagger again (see the epilogue's first barrier)
  }

  if (wm == 0) barrier_raw();   // re-align the halves (matching the stagger above)

  // ---- chunk end: merge the two wave halves and write this workgroup's partials
  if (wn == 0 && lane == 0) runn[wm] = run_n;
  __syncthreads();
  if (tid < BN) {
    const int64_t o = (int64_t)chunk * Ncols + n0 + tid;
    if (do_stats) {
      const float2 h0 = run[tid], h1 = run[BN + tid];
      if constexpr (MODE == MODE_FWD) {
        float n = runn[0], mean = h0.x, m2 = h0.y;
        chan_merge(n, mean, m2, runn[1], h1.x, h1.y);
        *reinterpret_cast<float2 *>(a.stats + o * 2) = make_float2(mean, m2);
      } else {
        *reinterpret_cast<float2 *>(a.stats + o * 2) = make_float2(h0.x + h1.x, 0.f);
      }
    }
    if (do_pool) {
      float4 p = runp[tid];
      const float4 q = runp[BN + tid];
      const int pi = __float_as_int(p.y), qi = __float_as_int(q.y);
      const int pj = __float_as_int(p.w), qj = __float_as_int(q.w);
      if (pool_max_wins(q.x, qi, p.x, pi)) { p.x = q.x; p.y = q.y; }
      if (pool_min_wins(q.z, qj, p.z, pj)) { p.z = q.z; p.w = q.w; }
      *reinterpret_cast<float4 *>(a.pool + o * 4) = p;
    }
  }
}

}  // namespace

bool pcs_gemm_glds_applicable(const pcs_gemm_args &a) {
  if (a.dtype != PCS_BF16 || (a.flags & (PCS_FLAG_GENERIC | PCS_FLAG_NO_GLDS))) return false;
  const bool fp8 = a.flags & PCS_FLAG_AW_FP8;
  if (fp8 && !a.w_scale) return false;
  if (a.prologue != PCS_PRO_RAW || a.K % (fp8 ? 256 : 2 * BK) != 0 || a.Ncols % BN != 0) return false;
  // forward: statistics / max-pool only (nothing stored); the pool keeps one extremum per
  // column, chosen by sign(es), so a pool needs es
  if (a.epilogue == PCS_EPI_FWD)
    return a.C == nullptr && a.scene_bias == nullptr && (!a.pool || a.es) &&
           (!(a.flags & PCS_FLAG_POOL_SIGNED_W) || (a.pool && !a.stats));
  if (a.epilogue == PCS_EPI_DGRAD)   // mask read from the operand itself, no S2, no addend
    return a.Yp == a.A && a.K == a.Ncols && !a.es && !a.et && !a.erstd && !a.addend && !a.c_mask &&
           !a.pool_w;
  return false;
}

int pcs_gemm_glds_launch(const pcs_gemm_args &g, int tps, int tpc, hipStream_t s) {
  const int ncb = g.Ncols / BN;
  const int nb = ncb * (int)(g.num_scenes * g.chunks_per_scene);
  const bool fp8 = g.flags & PCS_FLAG_AW_FP8;
#define PCS_GL(M, F) hipLaunchKernelGGL((gemm_glds_kernel<M, F>), dim3(nb), dim3(THREADS), 0, s, g, tps, tpc, ncb)
  if (g.epilogue == PCS_EPI_FWD) {
    if (fp8) PCS_GL(MODE_FWD, true); else PCS_GL(MODE_FWD, false);
  } else {
    if (fp8) PCS_GL(MODE_DGRAD, true); else PCS_GL(MODE_DGRAD, false);
  }
#undef PCS_GL
  PCS_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// pcs_pool_rows_add: the max-pool rows' term of global_feat's folded input gradient, after
// the LDS-DMA kernel (which leaves it out, see the top of this file):
//   dz[m, n] += (Yp[m, n] > 0) * sum_{c : idx[b, c] == m} coef[b, c] * Wp[c, n]
// for every distinct argmax row m of scene b, and the same term summed into S1.  Block
// (256 columns, scene, part): thread = column; the scene's (row, channel) pairs are rank-sorted
// in LDS so equal rows are applied once, in a fixed order, and the sorted list is cut into
// `parts` ranges at row boundaries (a row's pairs never straddle two blocks), so 1024 pairs
// are not one 1024-long dependent load chain per thread.  Part j adds its S1 share into chunk
// j's partial (j < chunks_per_scene): the partials are summed over chunks later, so no two
// threads update one value and the result is deterministic.
// ---------------------------------------------------------------------------------------
namespace {

constexpr int PR_MAXC = 1024;
constexpr int PR_PARTS = 16;

template <typename T, typename TY>
__global__ __launch_bounds__(256) void pool_rows_add_kernel(T *__restrict__ dz, const TY *__restrict__ Yp, int64_t N,
                                                            int Ncols, const int32_t *__restrict__ idx,
                                                            const float *__restrict__ coef, const float *__restrict__ Wp,
                                                            int64_t ldw, int P, float *__restrict__ stats, int cps) {
  // (row, channel) pairs sorted by row, then channel, as 64-bit keys row << 11 | channel:
  // a bitonic sort in LDS (55 compare-exchange passes; the O(P^2) rank sort it replaces was
  // most of this kernel's time)
  __shared__ unsigned long long keys[PR_MAXC];
  const int b = blockIdx.y, part = blockIdx.z, parts = gridDim.z, tid = threadIdx.x;
  const int n = blockIdx.x * 256 + tid;
  int Pp = 1;
  while (Pp < P) Pp <<= 1;
  for (int c = tid; c < Pp; c += 256)
    keys[c] = c < P ? ((unsigned long long)(uint32_t)idx[(int64_t)b * P + c] << 11) | (unsigned)c : ~0ull;
  __syncthreads();
  for (int k = 2; k <= Pp; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < Pp; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long x = keys[i], y = keys[ixj];
          if ((x > y) == ((i & k) == 0)) { keys[i] = y; keys[ixj] = x; }
        }
      }
      __syncthreads();
    }
  }
  auto srow_at = [&](int q) { return (int)(keys[q] >> 11); };
  auto sch_at = [&](int q) { return (int)(keys[q] & 2047u); };
  // this part's range [p0, p1): the nominal cut points moved forward to a row boundary
  auto cut = [&](int j) {
    int p = (int)((int64_t)j * P / parts);
    while (p > 0 && p < P && srow_at(p) == srow_at(p - 1)) ++p;
    return p;
  };
  const int p0 = cut(part), p1 = cut(part + 1);
  if (n >= Ncols || p0 >= p1) return;
  float ds1 = 0.f, v = 0.f;
  // 8 pairs' coefficients and W entries are loaded together (a 64-pair range walked one load
  // at a time made this kernel latency-bound); the sums still run in pair order
  constexpr int U = 8;
  for (int p = p0; p < p1; p += U) {
    float cf[U], wv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cf[u] = 0.f;
      wv[u] = 0.f;
      if (p + u < p1) {
        const int c = sch_at(p + u);
        cf[u] = coef[(int64_t)b * P + c];
        wv[u] = Wp[(int64_t)c * ldw + n];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = p + u;
      if (q >= p1) break;
      v = fmaf(cf[u], wv[u], v);
      if (q + 1 == p1 || srow_at(q + 1) != srow_at(q)) {   // last pair of this row: apply
        const int64_t m = (int64_t)srow_at(q);
        const int64_t o = m * Ncols + n;
        // rows outside scene b are skipped (pcs_pool_finalize emits none; a caller's index array
        // may): the row is a memory address here
        if (m >= (int64_t)b * N && m < (int64_t)(b + 1) * N && load_elem(Yp, o) > 0.f) {
          const float d = load_elem(dz, o) + v;
          if constexpr (sizeof(T) == 2) dz[o] = (T)(pack2bf(d, 0.f) & 0xffffu);
          else dz[o] = d;
          ds1 += v;
        }
        v = 0.f;
      }
    }
  }
  if (stats) stats[(((int64_t)b * cps + part) * Ncols + n) * 2] += ds1;
}

}  // namespace

extern "C" int pcs_pool_rows_add(void *dz, int32_t dz_dtype, const void *Yp, int32_t yp_dtype, int64_t num_scenes,
                                 int64_t scene_rows, int32_t Ncols, const int32_t *pool_idx, const float *pool_coef,
                                 const float *pool_w, int64_t pool_ldw, int32_t pool_c, float *stats,
                                 int32_t chunks_per_scene, pcs_stream_t stream) {
  if (!dz || !Yp || !pool_idx || !pool_coef || !pool_w || num_scenes <= 0 || scene_rows <= 0 || Ncols <= 0 ||
      pool_c <= 0 || pool_c > PR_MAXC || pool_ldw < Ncols || (stats && chunks_per_scene <= 0))
    return pcs_set_einval("pcs_pool_rows_add", "bad arguments (0 < pool_c <= 1024, pool_ldw >= Ncols)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int parts = stats ? (chunks_per_scene < PR_PARTS ? chunks_per_scene : PR_PARTS) : PR_PARTS;
  const dim3 grid((Ncols + 255) / 256, (unsigned)num_scenes, (unsigned)parts);
#define PCS_PRA(T, TY)                                                                                          \
  hipLaunchKernelGGL((pool_rows_add_kernel<T, TY>), grid, dim3(256), 0, s, static_cast<T *>(dz),                 \
                     static_cast<const TY *>(Yp), scene_rows, (int)Ncols, pool_idx, pool_coef, pool_w, pool_ldw, \
                     (int)pool_c, stats, (int)chunks_per_scene)
  if (dz_dtype == PCS_BF16 && yp_dtype == PCS_BF16) PCS_PRA(bf16_t, bf16_t);
  else if (dz_dtype == PCS_BF16 && yp_dtype == PCS_FP8) PCS_PRA(bf16_t, fp8_t);
  else if (dz_dtype == PCS_F32 && yp_dtype == PCS_F32) PCS_PRA(float, float);
  else return pcs_set_einval("pcs_pool_rows_add", "dtypes: (bf16, bf16), (bf16, fp8) or (f32, f32)");
#undef PCS_PRA
  PCS_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// pcs_quant_fp8_rows: per-row E8M0-scaled e4m3 copy of a weight matrix (one block per row)
// ---------------------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const float *__restrict__ W, int64_t cols, int64_t ldw,
                                                             fp8_t *__restrict__ Wq, uint8_t *__restrict__ scale,
                                                             float *__restrict__ deq) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  const float *w = W + r * ldw;
  float mx = 0.f;
  for (int64_t k = threadIdx.x; k < cols; k += 256) mx = fmaxf(mx, fabsf(w[k]));
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int e = 0;
  if (mx > 0.f) {
    e = (int)ceilf(log2f(mx / 448.f));
    e = e < -126 ? -126 : (e > 127 ? 127 : e);
  }
  if (threadIdx.x == 0) scale[r] = (uint8_t)(127 + e);
  const float inv = ldexpf(1.f, -e);
  for (int64_t k = threadIdx.x * 4; k < cols; k += 1024) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = k + q < cols ? w[k + q] * inv : 0.f;
    const uint32_t b = pack4fp8(v[0], v[1], v[2], v[3]);
    for (int q = 0; q < 4 && k + q < cols; ++q) {
      Wq[r * cols + k + q] = (fp8_t)(b >> (8 * q));
      if (deq) deq[r * cols + k + q] = ldexpf(fp82f((b >> (8 * q)) & 255u), e);
    }
  }
}
}  // namespace

extern "C" int pcs_quant_fp8_rows(const float *W, int64_t rows, int64_t cols, int64_t ldw, uint8_t *Wq, uint8_t *scale,
                                  float *deq, pcs_stream_t stream) {
  if (!W || !Wq || !scale || rows <= 0 || cols <= 0 || ldw < cols) return pcs_set_einval("pcs_quant_fp8_rows", "bad arguments");
  hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3((unsigned)rows), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), W,
                     cols, ldw, Wq, scale, deq);
  PCS_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// pcs_sign_rows: W's rows with the sign bit flipped where sign_of[r] < 0 (PCS_FLAG_POOL_SIGNED_W)
// ---------------------------------------------------------------------------------------
namespace {
template <typename T>
__global__ __launch_bounds__(256) void sign_rows_kernel(const T *__restrict__ W, int64_t cols,
                                                        const float *__restrict__ sign_of, T *__restrict__ out) {
  const int64_t r = blockIdx.y;
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= cols) return;
  constexpr uint32_t SB = 1u << (8 * sizeof(T) - 1);
  out[r * cols + k] = sign_of[r] < 0.f ? (T)(W[r * cols + k] ^ SB) : W[r * cols + k];
}
}  // namespace

extern "C" int pcs_sign_rows(const void *W, int32_t dtype, int64_t rows, int64_t cols, const float *sign_of, void *out,
                             pcs_stream_t stream) {
  if (!W || !sign_of || !out || rows <= 0 || rows > 65535 || cols <= 0)
    return pcs_set_einval("pcs_sign_rows", "bad arguments (0 < rows <= 65535)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((cols + 255) / 256), (unsigned)rows);
  if (dtype == PCS_F32)
    hipLaunchKernelGGL(sign_rows_kernel<uint32_t>, grid, dim3(256), 0, s, static_cast<const uint32_t *>(W), cols,
                       sign_of, static_cast<uint32_t *>(out));
  else if (dtype == PCS_BF16)
    hipLaunchKernelGGL(sign_rows_kernel<uint16_t>, grid, dim3(256), 0, s, static_cast<const uint16_t *>(W), cols,
                       sign_of, static_cast<uint16_t *>(out));
  else if (dtype == PCS_FP8)
    hipLaunchKernelGGL(sign_rows_kernel<uint8_t>, grid, dim3(256), 0, s, static_cast<const uint8_t *>(W), cols,
                       sign_of, static_cast<uint8_t *>(out));
  else
    return pcs_set_einval("pcs_sign_rows", "bad dtype");
  PCS_CHECK_LAUNCH();
  return 0;
}

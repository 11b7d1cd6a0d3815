// Gram G = a^T a of the stored bf16 activation a5 = relu(bn5(y5)) [M, C] (C = 1024) on the
// LDS-DMA pipeline: the weight gradient of global_feat (autograd of P:113 at P:254) in its
// Gram form (gram.hip: dW = beta (x) S + diag(gamma) W G + pool rows).
//
// * Only the C/256 x (C/256 + 1) / 2 upper 256-tiles of the symmetric G are computed
//   (10 for C = 1024); pcs_gram_raw mirrors the lower ones.
// * Grid = tiles x row splits, splits = floor(CUs / tiles) (25 for 10 tiles on 256 CUs): one
//   wave of workgroups, every CU busy but a few, each workgroup one tile over one contiguous
//   range of 64-row steps.  The tiles of a split are consecutive workgroups, which the XCD
//   remap places on one XCD, so the split's rows are read from HBM once and served to its
//   ten tiles from that XCD's L2.  Each workgroup writes one fp32 partial tile; pcs_gram_raw
//   sums them per tile in a fixed order.
// * The K-loop is the gemm_glds.hip 8-phase schedule with K = rows: a K-step stages 64 rows
//   x 256 columns of each operand HBM -> LDS by DMA (global_load_lds_dwordx4) as four 16 KB
//   regions (A-lo, A-hi: the n columns of wave rows i < 4 / i >= 4; B-lo, B-hi: the k
//   columns j < 2 / j >= 2), restaged one region per phase with counted vmcnt waits (shrunk
//   on the range's last two steps, where nothing more is issued) and raw barriers; the wave
//   halves run one barrier apart.
// * MFMA operands need 8 consecutive rows of one column per lane: ds_read_b64_tr_b16 reads
//   the [row][col] LDS image transposed.  Rows are 256 B; the 32-B granules of row r are
//   XOR-swizzled by f(r) = (r & 3) | ((r >> 3) & 1) << 2 (applied to the DMA source address,
//   since the DMA writes LDS linearly), so the 8 rows each half-wave reads land in 8 distinct
//   bank groups.
// * The final M % 64 rows are left to pcs_gram_raw's tail kernel.
// * fp8 (the cfg5 path, a5 stored as e4m3 by conv5's epilogue): a K-step is 128 rows of 128-B
//   region rows (the same 16 KB regions), one unit-scaled v_mfma_scale_f32_16x16x128_f8f6f4
//   per (i, j) pair.  A lane's 32 k-values of one column are four ds_read_b64_tr_b8 of 8 rows
//   (rows 32 t + 8 (lane >> 4) .. + 8, t = 0..3), the same lane -> k map for both operands;
//   the 16-B granules of row r are XOR-swizzled by (r >> 1) & 7, so the 16 rows a half-wave
//   reads fill all 64 banks.  Products of e4m3 values are exact in the fp32 accumulators: G is
//   the Gram of the stored activation, as in bf16.
#include "common.h"

#ifndef GG_PRIO
#define GG_PRIO 1   // base wave priority: above the dropout draw that shares its CUs (step -0.36 ms)
#endif

namespace {

constexpr int THREADS = 512;
constexpr int TN = 256;
constexpr int REG = 16384;                    // region: 64 rows x 256 B (bf16) | 128 x 128 B (fp8)
constexpr int KBUF = 4 * REG;                 // A-lo | A-hi | B-lo | B-hi
constexpr int LDS_BYTES = 2 * KBUF;           // 128 KB
template <bool FP8> struct GCfg {
  static constexpr int ESZ = FP8 ? 1 : 2;
  static constexpr int MS = FP8 ? 128 : 64;   // rows per K-step
  static constexpr int ROWB = 128 * ESZ;      // region row: 128 columns
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v2i lds_v2i;
typedef __attribute__((address_space(3))) void lds_void_t;

PCS_DEV void sbar() { __builtin_amdgcn_sched_barrier(0); }
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

PCS_DEV int gsw(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }   // bf16: 32-B granule swizzle of row r
PCS_DEV int gsw8(int r) { return (r >> 1) & 7; }                     // fp8: 16-B granule swizzle
// byte offset of (row, byte-in-row) in a region
PCS_DEV int roff(int r, int byte) { return r * 256 + ((((byte >> 5) ^ gsw(r)) << 5) | (byte & 31)); }
PCS_DEV int roff8(int r, int byte) { return r * 128 + ((((byte >> 4) ^ gsw8(r)) << 4) | (byte & 15)); }

// tile index t (0 .. nt(nt+1)/2 - 1) -> (block row, block col) of the upper triangle
PCS_DEV void tile_rc(int t, int nt, int &br, int &bc) {
  br = 0;
  while (t >= nt - br) { t -= nt - br; ++br; }
  bc = br + t;
}

// fp8: 32 k-values (rows 32 t + r0 .. + 8, t = 0..3) of one column per lane
PCS_DEV v8i tr_frag8(const char *region, int r0, int byte) {
  v8i v;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const v2i x = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i *)(region + roff8(32 * t + r0, byte)));
    v[2 * t] = x[0];
    v[2 * t + 1] = x[1];
  }
  return v;
}
PCS_DEV bf16x8 tr_frag(const char *region, int r0, int r1, int byte) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(region + roff(r0, byte)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(region + roff(r1, byte)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// Workgroup L = split * ntile + tile: steps [split * steps / nsplit, (split + 1) * steps / nsplit)
// of tile `tile`, partial slot L.
template <bool FP8>
__global__ __launch_bounds__(THREADS) void gram_glds_kernel(const void *__restrict__ A, int C, int64_t steps,
                                                            int ntile, float *__restrict__ part) {
  typedef GCfg<FP8> CF;
  constexpr int MS = CF::MS;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int nsplit = gridDim.x / ntile;
  const int split = L / ntile, tile = L % ntile;
  const int64_t s0 = (int64_t)split * steps / nsplit, s1 = (int64_t)(split + 1) * steps / nsplit;
  float *out = part + (int64_t)L * TN * TN;
  const int total = (int)(s1 - s0);
  const int nt = C / TN;
  int br, bc;
  tile_rc(tile, nt, br, bc);
  const int64_t rowbytes = (int64_t)C * CF::ESZ;
  const char *Ab = reinterpret_cast<const char *>(A);

  // ---- DMA, bf16: piece g (0, 1) of wave w covers region rows (2w + g) * 4 .. + 4; lane ->
  // row + lane / 16, LDS slot lane % 16 (16 B), which holds logical chunk c of the row:
  // granule (slot / 2) ^ f(row), half slot % 2.
  //   A regions (n columns): chunk c -> tile column (c & 7) * 8 + (c >> 3) * 128 + hi * 64
  //   B regions (k columns): chunk c -> tile column (c >> 2) * 64 + (c & 3) * 8 + hi * 32
  // fp8: rows (2w + g) * 8 + lane / 8, slot lane % 8 holds granule c = slot ^ f8(row) (16 columns)
  //   A: c -> (c & 3) * 16 + (c >> 2) * 128 + hi * 64;  B: c -> (c >> 1) * 64 + (c & 1) * 16 + hi * 32
  int prow[2];
  uint32_t acol[2][2], bcol[2][2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    if constexpr (FP8) {
      prow[g] = (2 * wid + g) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ gsw8(prow[g]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acol[h][g] = (uint32_t)((c & 3) * 16 + (c >> 2) * 128 + h * 64);
        bcol[h][g] = (uint32_t)((c >> 1) * 64 + (c & 1) * 16 + h * 32);
      }
    } else {
      prow[g] = (2 * wid + g) * 4 + (lane >> 4);
      const int slot = lane & 15;
      const int c = ((((slot >> 1) ^ gsw(prow[g])) << 1) | (slot & 1));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acol[h][g] = (uint32_t)(((c & 7) * 8 + (c >> 3) * 128 + h * 64) * 2);
        bcol[h][g] = (uint32_t)(((c >> 2) * 64 + (c & 3) * 8 + h * 32) * 2);
      }
    }
  }

  auto issue = [&](int qseq, int region) {
    if (qseq >= total) return;   // nothing left: the tail waits below shrink to match
    const int hi = region & 1;
    const int col0 = (region < 2 ? br : bc) * TN;
    const char *sb = Ab + (s0 + qseq) * MS * rowbytes + (int64_t)col0 * CF::ESZ;
    char *dst = lds + (qseq & 1) * KBUF + region * REG;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const uint32_t col = region < 2 ? acol[hi][g] : bcol[hi][g];
      glds16(sb, (uint32_t)prow[g] * (uint32_t)rowbytes + col, dst + (2 * wid + g) * 1024);
    }
  };

  // fragments, bf16: lane (q = (lane >> 2) & 3, p = lane & 3, g = lane >> 4) reads rows
  // 32 kk + 8 g + q (+4) of column base + 4 p, transposed.  fp8: in each 16-lane group lane i
  // reads row 8 g + i / 2 (+ 32 t), bytes 8 (i & 1) .. of the group's 16 columns, and ends
  // with column i of the 8 rows
  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int r8 = 8 * fg + ((lane & 15) >> 1), c8 = 8 * (lane & 1);
  bf16x8 af[4][2], bfr[4][2];
  v8i af8[4], bf8[4];
  auto read_a = [&](int buf, int hi) {   // n columns wm*128 + (hi*4 + i)*16 .. -> region col wm*64 + i*16
    const char *base = lds + buf * KBUF + hi * REG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (FP8) {
        af8[i] = tr_frag8(base, r8, wm * 64 + i * 16 + c8);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int r0 = 32 * kk + 8 * fg + fq;
          af[i][kk] = tr_frag(base, r0, r0 + 4, (wm * 64 + i * 16 + 4 * fp) * 2);
        }
      }
    }
  };
  auto read_b = [&](int buf, int hi, int j0) {   // k columns wn*64 + (hi*2 + j)*16 -> region col wn*32 + j*16
    const char *base = lds + buf * KBUF + (2 + hi) * REG;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (FP8) {
        bf8[j0 + j] = tr_frag8(base, r8, wn * 32 + j * 16 + c8);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int r0 = 32 * kk + 8 * fg + fq;
          bfr[j0 + j][kk] = tr_frag(base, r0, r0 + 4, (wn * 32 + j * 16 + 4 * fp) * 2);
        }
      }
    }
  };

  f32x4 acc[8][4];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  auto mfma_quad = [&](int i0, int j0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (FP8) {
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              bf8[j0 + j], af8[i], acc[i0 + i][j0 + j], 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
        } else {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j0 + j][kk], af[i][kk],
                                                                           acc[i0 + i][j0 + j], 0, 0, 0);
        }
      }
  };

  // ---- prologue: step 0 landed; A-lo, B-lo, B-hi of step 1 in flight
  if (total <= 0) {   // uniform: an empty range still owns its (zero) partial slot
    for (int e = tid; e < TN * TN / 4; e += THREADS) reinterpret_cast<f32x4 *>(out)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  issue(0, 0); issue(0, 1); issue(0, 2); issue(0, 3);
  issue(1, 0); issue(1, 2); issue(1, 3);
  if (total > 1) wait_vm<6>(); else wait_vm<0>();
  barrier_raw();
  if (wm == 1) barrier_raw();   // wave halves one barrier apart

  for (int qs = 0; qs < total; ++qs) {
    const int buf = qs & 1;
    // phase 1: (n lo, k lo); restage A-hi of step qs+1
    read_a(buf, 0);
    read_b(buf, 0, 0);
    issue(qs + 1, 1);
    if (qs + 1 < total) wait_vm<10>(); else wait_vm<2>();      // retires B-hi(qs)
    wait_lgkm0();
    barrier_raw();
    __builtin_amdgcn_s_setprio(1 + GG_PRIO);
    mfma_quad(0, 0);
    __builtin_amdgcn_s_setprio(GG_PRIO);
    barrier_raw();
    // phase 2: (lo, hi); restage A-lo of step qs+2
    read_b(buf, 1, 2);
    issue(qs + 2, 0);
    if (qs + 2 < total) wait_vm<10>(); else if (qs + 1 < total) wait_vm<8>(); else wait_vm<0>();   // A-hi(qs)
    wait_lgkm0();
    barrier_raw();
    __builtin_amdgcn_s_setprio(1 + GG_PRIO);
    mfma_quad(0, 2);
    __builtin_amdgcn_s_setprio(GG_PRIO);
    barrier_raw();
    // phase 3: (hi, lo); restage B-lo of step qs+2
    read_a(buf, 1);
    issue(qs + 2, 2);
    wait_lgkm0();
    barrier_raw();
    __builtin_amdgcn_s_setprio(1 + GG_PRIO);
    mfma_quad(4, 0);
    __builtin_amdgcn_s_setprio(GG_PRIO);
    barrier_raw();
    // phase 4: (hi, hi); restage B-hi of step qs+2
    issue(qs + 2, 3);
    if (qs + 2 < total) wait_vm<10>(); else if (qs + 1 < total) wait_vm<4>(); else wait_vm<0>();   // A-lo, B-lo(qs+1)
    barrier_raw();
    __builtin_amdgcn_s_setprio(1 + GG_PRIO);
    mfma_quad(4, 2);
    __builtin_amdgcn_s_setprio(GG_PRIO);
    barrier_raw();

  }
  // lane holds G[n = wm*128 + i*16 + (lane & 15)][k = wn*64 + j*16 + 4*(lane >> 4) + r]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = wm * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = wn * 64 + j * 16 + 4 * (lane >> 4);
      *reinterpret_cast<f32x4 *>(out + n * TN + k) = acc[i][j];
    }
  }
  if (wm == 0) barrier_raw();   // re-align the halves
}

// sum the nsplit partial slots of each upper tile into G (fixed order) and add the Gram of
// the tail rows [m_tail, M) (fewer than one K-step); mirror into the lower tiles
template <typename T>
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float *__restrict__ part, const T *__restrict__ A,
                                                          int64_t M, int64_t m_tail, int C, int ntile, int nsplit,
                                                          float *__restrict__ G) {
  const int t = blockIdx.y;
  const int nt = C / TN;
  int br, bc;
  tile_rc(t, nt, br, bc);
  const int e = blockIdx.x * 256 + threadIdx.x;   // element of the 256 x 256 tile
  const int n = e >> 8, k = e & 255;
  float s = 0.f;
  for (int sp = 0; sp < nsplit; ++sp) s += part[((int64_t)sp * ntile + t) * TN * TN + e];
  const int gn = br * TN + n, gk = bc * TN + k;
  for (int64_t m = m_tail; m < M; ++m)
    s = fmaf(load_elem(A, m * C + gn), load_elem(A, m * C + gk), s);
  G[(int64_t)gn * C + gk] = s;
  if (br != bc) G[(int64_t)gk * C + gn] = s;
}

}  // namespace

namespace {
int gram_splits(int C) {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const int nt = C / TN, ntile = nt * (nt + 1) / 2;
  return ncu / ntile > 0 ? ncu / ntile : 1;
}
}  // namespace

extern "C" int64_t pcs_gram_raw_workspace(int64_t M, int32_t C) {
  if (M <= 0 || C <= 0 || C % TN) return pcs_set_einval("pcs_gram_raw_workspace", "C must be a multiple of 256");
  const int nt = C / TN, ntile = nt * (nt + 1) / 2;
  return (int64_t)gram_splits(C) * ntile * TN * TN * 4;
}

extern "C" int pcs_gram_raw(const void *A, int64_t M, int32_t C, int32_t dtype, float *workspace,
                            int64_t workspace_bytes, float *G, pcs_stream_t stream) {
  if (!A || !workspace || !G || M <= 0 || C <= 0 || C % TN)
    return pcs_set_einval("pcs_gram_raw", "A, workspace, G, M > 0 and C % 256 == 0 required");
  if (dtype != PCS_BF16 && dtype != PCS_FP8) return pcs_set_einval("pcs_gram_raw", "dtype must be PCS_BF16 or PCS_FP8");
  if (M >= ((int64_t)1 << 31)) return pcs_set_einval("pcs_gram_raw", "M must be < 2^31");
  const int64_t need = pcs_gram_raw_workspace(M, C);
  if (need < 0) return (int)need;
  if (workspace_bytes < need) return pcs_set_einval("pcs_gram_raw", "workspace too small (pcs_gram_raw_workspace)");
  const int nt = C / TN, ntile = nt * (nt + 1) / 2;
  const int nsplit = gram_splits(C);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 rgrid(TN * TN / 256, ntile);
  if (dtype == PCS_FP8) {
    const int64_t steps = M / GCfg<true>::MS;
    hipLaunchKernelGGL(gram_glds_kernel<true>, dim3(nsplit * ntile), dim3(THREADS), 0, s, A, (int)C, steps, ntile,
                       workspace);
    PCS_CHECK_LAUNCH();
    hipLaunchKernelGGL(gram_reduce_kernel<fp8_t>, rgrid, dim3(256), 0, s, workspace, static_cast<const fp8_t *>(A), M,
                       steps * GCfg<true>::MS, (int)C, ntile, nsplit, G);
  } else {
    const int64_t steps = M / GCfg<false>::MS;
    hipLaunchKernelGGL(gram_glds_kernel<false>, dim3(nsplit * ntile), dim3(THREADS), 0, s, A, (int)C, steps, ntile,
                       workspace);
    PCS_CHECK_LAUNCH();
    hipLaunchKernelGGL(gram_reduce_kernel<bf16_t>, rgrid, dim3(256), 0, s, workspace, static_cast<const bf16_t *>(A),
                       M, steps * GCfg<false>::MS, (int)C, ntile, nsplit, G);
  }
  PCS_CHECK_LAUNCH();
  return 0;
}

// bf16 256x256x64 points-major GEMM for the wide layers (global_feat forward and dgrad:
// M x 1024 x 1024, 75 % of the model's MACs; P:113 and its autograd at P:254).
//
// Same contract as gemm_nt.hip (pcs_gemm_args, scene-aligned row chunks, prologue and
// epilogue fusion) with a tile sized for MFMA throughput instead of generality:
// * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns 128 x 64 outputs =
//   8 x 4 v_mfma_f32_16x16x32_bf16 accumulators; 64 MFMAs per wave per 64-deep k-step.
// * operands staged global -> VGPR (BN+ReLU / BN-backward prologue) -> LDS, 128-B rows,
//   16-B slots XOR-swizzled with (row>>1)&7 so the ds_read_b128 fragment reads are
//   bank-conflict free; two LDS stages, one barrier per k-step; the next k-step's global
//   loads are issued before the current MFMAs.
// * forward epilogue: bias, tile staged through LDS for 16-B coalesced stores (BN
//   statistics and max-pool partials come from one streaming pass, pcs_colstats: fused
//   here as cross-lane reductions they cost ~1/3 of the kernel).
// * dgrad: raw store (PCS_EPI_RAW); the ReLU / BN-backward stage of the previous layer runs
//   as one streaming pass (pcs_bnrelu_bwd).
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int KMAX = 1024;                   // per-channel coefficient arrays live in LDS
constexpr int ROWB = BK * 2;                 // 128 B per LDS row
constexpr int STAGE = (BM + BN) * ROWB;      // 64 KB
constexpr int CROW = BN * 2 + 16;            // epilogue tile row stride
constexpr int CTILE = BM * CROW;             // 132 KB
constexpr int CPR = BN * 2 / 16;             // 32 chunks per output row
constexpr int RPP = THREADS / CPR;           // 16 rows per pass
constexpr int LDS_MAIN = (2 * STAGE > CTILE) ? 2 * STAGE : CTILE;
constexpr int COEF = 4 * KMAX * 4;           // up to 4 per-channel arrays (16 KB)
constexpr int LDS_BYTES = LDS_MAIN + COEF + 32;   // + per-tile argmax-row bitmap (256 bits)

PCS_DEV int swz8(int row, int slot) { return slot ^ ((row >> 1) & 7); }

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

PCS_DEV void lds_vec8(const float *p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4 *>(p);
  const float4 b = *reinterpret_cast<const float4 *>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// Pipeline (one LDS double buffer, one register stage, one barrier per 64-deep k-step):
//   compute(ks) from LDS[ks&1]  ->  transform + write the registers (k-step ks+1) into
//   LDS[(ks+1)&1]  ->  issue the global loads of k-step ks+2  ->  barrier.
// Each load has a full MFMA block to land; the per-channel prologue coefficients come from
// LDS (staged once per workgroup: a workgroup's row chunk never leaves its scene), and rows
// past the end of a scene are clamped rather than branched around (their outputs are never
// stored), so the k-loop carries no exec-mask branches and no early vmcnt(0).
template <int PRO, int EPI, bool MASK>
__global__ __launch_bounds__(THREADS) void gemm_big_kernel(pcs_gemm_args a, int tiles_per_scene,
                                                           int tiles_per_chunk, int ncb) {
  constexpr int EPC = 8;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float *cf = reinterpret_cast<float *>(lds + LDS_MAIN);
  uint32_t *tbits = reinterpret_cast<uint32_t *>(lds + LDS_MAIN + COEF);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = L / ncb, cb = L % ncb;
  const int cps = a.chunks_per_scene;
  const int scene = chunk / cps, cis = chunk % cps;
  const int n0 = cb * BN;
  const int K = a.K, Ncols = a.Ncols;
  const int64_t N = a.scene_rows;
  const int t_begin = cis * tiles_per_chunk;
  const int t_end = min(t_begin + tiles_per_chunk, tiles_per_scene);
  const int nks = K / BK;
  if (t_begin >= t_end) return;

  const bf16_t *__restrict__ Ag = reinterpret_cast<const bf16_t *>(a.A);
  const bf16_t *__restrict__ A2g = reinterpret_cast<const bf16_t *>(a.A2);
  const bf16_t *__restrict__ Wg = reinterpret_cast<const bf16_t *>(a.W);
  bf16_t *__restrict__ Cg = reinterpret_cast<bf16_t *>(a.C);

  // per-channel prologue coefficients -> LDS: c0 | c1 | c2 | pool argmax rows
  for (int k = tid; k < K; k += THREADS) {
    if constexpr (PRO == PCS_PRO_BNRELU) {
      cf[k] = a.pa[k]; cf[KMAX + k] = a.pb[k];
    } else if constexpr (PRO == PCS_PRO_BWD) {
      cf[k] = a.pa[k]; cf[KMAX + k] = a.pb[k]; cf[2 * KMAX + k] = a.pc[k];
    } else if constexpr (PRO == PCS_PRO_BWD_POOL) {
      cf[k] = a.pool_coef[(int64_t)scene * K + k]; cf[KMAX + k] = a.pb[k];
      cf[2 * KMAX + k] = a.pc[k];
      reinterpret_cast<int *>(cf)[3 * KMAX + k] = a.pool_idx[(int64_t)scene * K + k];
    }
  }

  const int slot = tid & 7, srow = tid >> 3;  // staging: rows srow + 64*i, fixed k-slot
  const int ecc = tid % CPR, er0 = tid / CPR, ecol = n0 + ecc * EPC;
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);

  u32x4 ra[4], ra2[4], rb[4];
  uint32_t mk[4];
  uint32_t hits = 0;   // POOL: bit i set if staging row srow + 64 i is an argmax row of the tile
  auto load_stage = [&](int64_t row_base, int valid, int ks) {
    const int k0 = ks * BK + slot * EPC;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = min(srow + 64 * i, valid - 1);
      const int64_t off = (row_base + r) * K + k0;
      ra[i] = *reinterpret_cast<const u32x4 *>(Ag + off);
      if constexpr (PRO == PCS_PRO_BWD) ra2[i] = *reinterpret_cast<const u32x4 *>(A2g + off);
      if constexpr (MASK) mk[i] = a.a_mask[off >> 3];
      rb[i] = *reinterpret_cast<const u32x4 *>(Wg + (int64_t)(n0 + srow + 64 * i) * K + k0);
    }
  };
  auto store_stage = [&](int64_t row_base, int ks, int buf) {
    char *tA = lds + buf * STAGE;
    char *tB = tA + BM * ROWB;
    const int k0 = ks * BK + slot * EPC;
    float c0[EPC], c1[EPC], c2[EPC];
    if constexpr (PRO == PCS_PRO_BNRELU) {
      lds_vec8(cf + k0, c0); lds_vec8(cf + KMAX + k0, c1);
    } else if constexpr (PRO == PCS_PRO_BWD) {
      lds_vec8(cf + k0, c0); lds_vec8(cf + KMAX + k0, c1); lds_vec8(cf + 2 * KMAX + k0, c2);
    } else if constexpr (PRO == PCS_PRO_BWD_POOL) {
      lds_vec8(cf + KMAX + k0, c1); lds_vec8(cf + 2 * KMAX + k0, c2);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = srow + 64 * i;
      float v[EPC];
      unpack_chunk(ra[i], v);
      if constexpr (PRO == PCS_PRO_BNRELU) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          float x = fmaxf(fmaf(v[e], c0[e], c1[e]), 0.f);
          if constexpr (MASK) x *= ((mk[i] >> e) & 1u) ? a.a_keep_scale : 0.f;
          v[e] = x;
        }
      } else if constexpr (PRO == PCS_PRO_BWD) {
        float y[EPC];
        unpack_chunk(ra2[i], y);
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = fmaf(c0[e], v[e], fmaf(c2[e], y[e], c1[e]));
      } else if constexpr (PRO == PCS_PRO_BWD_POOL) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = fmaf(c2[e], v[e], c1[e]);
        if ((hits >> i) & 1u) {   // rare: this row is the max-pool argmax of some channel
          const int grow = (int)(row_base + r);
          const int *am = reinterpret_cast<const int *>(cf + 3 * KMAX);
#pragma unroll
          for (int e = 0; e < EPC; ++e) v[e] += am[k0 + e] == grow ? cf[k0 + e] : 0.f;
        }
      }
      const u32x4 out = (PRO == PCS_PRO_RAW) ? ra[i] : pack_chunk(v);
      *reinterpret_cast<u32x4 *>(tA + r * ROWB + swz8(r, slot) * 16) = out;
      *reinterpret_cast<u32x4 *>(tB + r * ROWB + swz8(r, slot) * 16) = rb[i];
    }
  };

  auto tile_rows = [&](int tile) { return (int)pcs_min64(BM, N - (int64_t)tile * BM); };

  int64_t row_base = scene * N + (int64_t)t_begin * BM;
  int valid = tile_rows(t_begin);
  load_stage(row_base, valid, 0);
  __syncthreads();   // coefficients visible

  for (int tile = t_begin; tile < t_end; ++tile) {
    if constexpr (PRO == PCS_PRO_BWD_POOL) {   // bitmap of the tile's argmax rows
      if (tid < BM / 32) tbits[tid] = 0u;
      __syncthreads();
      const int *am = reinterpret_cast<const int *>(cf + 3 * KMAX);
      for (int c = tid; c < K; c += THREADS) {
        const int64_t m = (int64_t)am[c] - row_base;
        if (m >= 0 && m < valid) atomicOr(&tbits[m >> 5], 1u << (m & 31));
      }
      __syncthreads();
      hits = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = srow + 64 * i;
        hits |= ((tbits[r >> 5] >> (r & 31)) & 1u) << i;
      }
    }
    store_stage(row_base, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    load_stage(row_base, valid, 1);   // nks >= 8 (K >= 512)
    lds_barrier();

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int64_t next_base = row_base + BM;
    const int next_valid = (tile + 1 < t_end) ? tile_rows(tile + 1) : 0;
    for (int ks = 0; ks < nks; ++ks) {
      const int buf = ks & 1;
      const char *tA = lds + buf * STAGE;
      const char *tB = tA + BM * ROWB;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int sl = (lane >> 4) + 4 * kk;
        bf16x8 bfr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = wn * 64 + j * 16 + (lane & 15);
          bfr[j] = *reinterpret_cast<const bf16x8 *>(tB + r * ROWB + swz8(r, sl) * 16);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int r = wm * 128 + i * 16 + (lane & 15);
          const bf16x8 af = *reinterpret_cast<const bf16x8 *>(tA + r * ROWB + swz8(r, sl) * 16);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af, acc[i][j], 0, 0, 0);
        }
      }
      if (ks + 1 < nks) {
        store_stage(row_base, ks + 1, buf ^ 1);
        __builtin_amdgcn_sched_barrier(0);   // keep one staging register set live, not two
        // ONE load site (two sites make the compiler merge their registers with copies that
        // wait for the loads): k-step ks+2 of this tile, else step 0 of the next tile, else
        // a harmless in-bounds reload that is never consumed.
        const bool tail = ks + 2 >= nks;
        const bool has_next = next_valid > 0;
        load_stage(tail && has_next ? next_base : row_base, tail && has_next ? next_valid : valid,
                   tail ? 0 : ks + 2);
      }
      lds_barrier();
    }

    // lane owns rows m = wm*128 + i*16 + (lane&15), cols n = wn*64 + j*16 + 4*(lane>>4) + r
    if constexpr (EPI == PCS_EPI_FWD) {
      if (a.bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 bb = *reinterpret_cast<const float4 *>(a.bias + n0 + wn * 64 + j * 16 + lcol);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            acc[i][j][0] += bb.x; acc[i][j][1] += bb.y; acc[i][j][2] += bb.z; acc[i][j][3] += bb.w;
          }
        }
      }
    }

    // phase 1: tile -> LDS (bf16), phase 2: coalesced row chunks
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = wm * 128 + i * 16 + lrow;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = wn * 64 + j * 16 + lcol;
        *reinterpret_cast<uint2 *>(lds + m * CROW + n * 2) =
            make_uint2(pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3]));
      }
    }
    __syncthreads();
    if (Cg) {
#pragma unroll 4
      for (int rr = er0; rr < valid; rr += RPP)
        *reinterpret_cast<u32x4 *>(Cg + (row_base + rr) * Ncols + ecol) =
            *reinterpret_cast<const u32x4 *>(lds + rr * CROW + ecc * 16);
    }
    __syncthreads();
    row_base = next_base;
    valid = next_valid;
  }
}

template <int PRO, int EPI, bool MASK>
int launch(const pcs_gemm_args &a, int tps, int tpc, hipStream_t s) {
  const int ncb = a.Ncols / BN;
  const int nb = ncb * (int)(a.num_scenes * a.chunks_per_scene);
  hipLaunchKernelGGL((gemm_big_kernel<PRO, EPI, MASK>), dim3(nb), dim3(THREADS), 0, s, a, tps, tpc, ncb);
  PCS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

bool pcs_gemm_big_applicable(const pcs_gemm_args &a) {
  if (a.dtype != PCS_BF16 || a.K % BK != 0 || a.Ncols % BN != 0 || a.K < 512 || a.K > KMAX) return false;
  if (a.a_mask && a.prologue != PCS_PRO_BNRELU) return false;
  if (a.flags & PCS_FLAG_GENERIC) return false;
  if (a.epilogue == PCS_EPI_FWD)   // statistics / pool: pcs_colstats on the stored output
    return a.prologue == PCS_PRO_BNRELU && !a.stats && !a.pool && !a.scene_bias;
  if (a.epilogue == PCS_EPI_RAW) return a.prologue != PCS_PRO_RAW;   // dgrad: pcs_bnrelu_bwd after
  return false;
}

int pcs_gemm_big_launch(const pcs_gemm_args &g, int tps, int tpc, hipStream_t s) {
  if (g.epilogue == PCS_EPI_FWD)
    return g.a_mask ? launch<PCS_PRO_BNRELU, PCS_EPI_FWD, true>(g, tps, tpc, s)
                    : launch<PCS_PRO_BNRELU, PCS_EPI_FWD, false>(g, tps, tpc, s);
  if (g.prologue == PCS_PRO_BWD_POOL) return launch<PCS_PRO_BWD_POOL, PCS_EPI_RAW, false>(g, tps, tpc, s);
  if (g.prologue == PCS_PRO_BNRELU)
    return g.a_mask ? launch<PCS_PRO_BNRELU, PCS_EPI_RAW, true>(g, tps, tpc, s)
                    : launch<PCS_PRO_BNRELU, PCS_EPI_RAW, false>(g, tps, tpc, s);
  return launch<PCS_PRO_BWD, PCS_EPI_RAW, false>(g, tps, tpc, s);
}

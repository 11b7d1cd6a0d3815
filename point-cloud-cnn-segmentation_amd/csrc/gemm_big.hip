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
constexpr int ROWB = BK * 2;                 // 128 B per LDS row
constexpr int STAGE = (BM + BN) * ROWB;      // 64 KB
constexpr int CROW = BN * 2 + 16;            // epilogue tile row stride
constexpr int CTILE = BM * CROW;             // 135 KB
constexpr int CPR = BN * 2 / 16;             // 32 chunks per output row
constexpr int RPP = THREADS / CPR;           // 16 rows per pass
constexpr int LDS_MAIN = (2 * STAGE > CTILE) ? 2 * STAGE : CTILE;
constexpr int SRED = 4 * 2 * BN * 4;         // small cross-wave reduction area (16 KB)
constexpr int LDS_BYTES = LDS_MAIN + SRED;

PCS_DEV int swz8(int row, int slot) { return slot ^ ((row >> 1) & 7); }

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

PCS_DEV float round_bf16(float v) { return bf2f(pack2bf(v, 0.f) & 0xffffu); }

template <int PRO, int EPI, bool POOL>
__global__ __launch_bounds__(THREADS) void gemm_big_kernel(pcs_gemm_args a, int tiles_per_scene,
                                                           int tiles_per_chunk, int ncb) {
  constexpr int EPC = 8;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float *sred = reinterpret_cast<float *>(lds + LDS_MAIN);

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

  const bf16_t *__restrict__ Ag = reinterpret_cast<const bf16_t *>(a.A);
  const bf16_t *__restrict__ A2g = reinterpret_cast<const bf16_t *>(a.A2);
  const bf16_t *__restrict__ Wg = reinterpret_cast<const bf16_t *>(a.W);
  bf16_t *__restrict__ Cg = reinterpret_cast<bf16_t *>(a.C);

  const int slot = tid & 7, srow = tid >> 3;  // staging: rows srow + 64*i, fixed k-slot

  const int ecc = tid % CPR, er0 = tid / CPR, ecol = n0 + ecc * EPC;

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int64_t row_base = scene * N + (int64_t)tile * BM;
    const int valid = (int)pcs_min64(BM, N - (int64_t)tile * BM);

    u32x4 ra[4], ra2[4], rb[4];
    auto load_stage = [&](int ks) {
      const int k0 = ks * BK + slot * EPC;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = srow + 64 * i;
        if (r < valid) {
          const int64_t off = (row_base + r) * K + k0;
          ra[i] = *reinterpret_cast<const u32x4 *>(Ag + off);
          if constexpr (PRO == PCS_PRO_BWD) ra2[i] = *reinterpret_cast<const u32x4 *>(A2g + off);
        }
        rb[i] = *reinterpret_cast<const u32x4 *>(Wg + (int64_t)(n0 + r) * K + k0);
      }
    };
    auto store_stage = [&](int ks, int buf) {
      char *tA = lds + buf * STAGE;
      char *tB = tA + BM * ROWB;
      const int k0 = ks * BK + slot * EPC;
      float c0[EPC], c1[EPC], c2[EPC];
      int am[EPC];
      if constexpr (PRO == PCS_PRO_BNRELU) {
        load_vec<EPC>(a.pa, k0, c0); load_vec<EPC>(a.pb, k0, c1);
      } else if constexpr (PRO == PCS_PRO_BWD) {
        load_vec<EPC>(a.pa, k0, c0); load_vec<EPC>(a.pb, k0, c1); load_vec<EPC>(a.pc, k0, c2);
      } else if constexpr (PRO == PCS_PRO_BWD_POOL) {
        load_vec<EPC>(a.pb, k0, c1); load_vec<EPC>(a.pc, k0, c2);
        load_vec<EPC>(a.pool_coef + scene * K, k0, c0);
        const int4 i0 = *reinterpret_cast<const int4 *>(a.pool_idx + scene * K + k0);
        const int4 i1 = *reinterpret_cast<const int4 *>(a.pool_idx + scene * K + k0 + 4);
        am[0] = i0.x; am[1] = i0.y; am[2] = i0.z; am[3] = i0.w;
        am[4] = i1.x; am[5] = i1.y; am[6] = i1.z; am[7] = i1.w;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = srow + 64 * i;
        u32x4 out = mk_u32x4(0, 0, 0, 0);
        if (r < valid) {
          float v[EPC];
          unpack_chunk(ra[i], v);
          if constexpr (PRO == PCS_PRO_BNRELU) {
            uint32_t bits = 0xffu;
            if (a.a_mask) bits = mask_bits(a.a_mask, row_base + r, K, k0, EPC);
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
              float x = fmaxf(fmaf(v[e], c0[e], c1[e]), 0.f);
              if (a.a_mask) x *= ((bits >> e) & 1u) ? a.a_keep_scale : 0.f;
              v[e] = x;
            }
          } else if constexpr (PRO == PCS_PRO_BWD) {
            float y[EPC];
            unpack_chunk(ra2[i], y);
#pragma unroll
            for (int e = 0; e < EPC; ++e) v[e] = fmaf(c0[e], v[e], fmaf(c2[e], y[e], c1[e]));
          } else if constexpr (PRO == PCS_PRO_BWD_POOL) {
            const int grow = (int)(row_base + r);
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
              float x = fmaf(c2[e], v[e], c1[e]);
              if (am[e] == grow) x += c0[e];
              v[e] = x;
            }
          }
          out = pack_chunk(v);
        }
        *reinterpret_cast<u32x4 *>(tA + r * ROWB + swz8(r, slot) * 16) = out;
        *reinterpret_cast<u32x4 *>(tB + r * ROWB + swz8(r, slot) * 16) = rb[i];
      }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    load_stage(0);
    store_stage(0, 0);
    __syncthreads();
    for (int ks = 0; ks < nks; ++ks) {
      const int buf = ks & 1;
      if (ks + 1 < nks) load_stage(ks + 1);
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
      if (ks + 1 < nks) store_stage(ks + 1, buf ^ 1);
      __syncthreads();
    }

    // lane owns rows m = wm*128 + i*16 + (lane&15), cols n = wn*64 + j*16 + 4*(lane>>4) + r
    const int lrow = lane & 15, lcol = 4 * (lane >> 4);
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
  }

}

template <int PRO, int EPI, bool POOL>
int launch(const pcs_gemm_args &a, int tps, int tpc, hipStream_t s) {
  const int ncb = a.Ncols / BN;
  const int nb = ncb * (int)(a.num_scenes * a.chunks_per_scene);
  hipLaunchKernelGGL((gemm_big_kernel<PRO, EPI, POOL>), dim3(nb), dim3(THREADS), 0, s, a, tps, tpc, ncb);
  PCS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

bool pcs_gemm_big_applicable(const pcs_gemm_args &a) {
  if (a.dtype != PCS_BF16 || a.K % BK != 0 || a.Ncols % BN != 0 || a.K < 512) return false;
  if (a.flags & PCS_FLAG_GENERIC) return false;
  if (a.epilogue == PCS_EPI_FWD)   // statistics / pool: pcs_colstats on the stored output
    return a.prologue == PCS_PRO_BNRELU && !a.stats && !a.pool && !a.scene_bias;
  if (a.epilogue == PCS_EPI_RAW) return a.prologue != PCS_PRO_RAW;   // dgrad: pcs_bnrelu_bwd after
  return false;
}

int pcs_gemm_big_launch(const pcs_gemm_args &g, int tps, int tpc, hipStream_t s) {
  if (g.epilogue == PCS_EPI_FWD) return launch<PCS_PRO_BNRELU, PCS_EPI_FWD, false>(g, tps, tpc, s);
  if (g.prologue == PCS_PRO_BWD_POOL) return launch<PCS_PRO_BWD_POOL, PCS_EPI_RAW, false>(g, tps, tpc, s);
  if (g.prologue == PCS_PRO_BNRELU) return launch<PCS_PRO_BNRELU, PCS_EPI_RAW, false>(g, tps, tpc, s);
  return launch<PCS_PRO_BWD, PCS_EPI_RAW, false>(g, tps, tpc, s);
}

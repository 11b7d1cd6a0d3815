// Points-major fused GEMM for the 1x1 Conv1d chain of PointNetSegmentation.
//
//   C[m, n] = sum_k pro(A)[m, k] * W[n, k]        (forward: P:106-128; dgrad: P:254)
//
// * pro(): BN-apply + ReLU (+ dropout keep bits) of the previous layer, or the BatchNorm
//   backward affine dy = alpha*dz + beta + gamma*y, applied while the tile is staged
//   global -> registers -> LDS, so activations are read once per tile and never written
//   back in transformed form.
// * epilogue: bias / per-scene bias, store, and per-chunk BatchNorm statistics (Welford
//   per thread, Chan merge across threads) plus max/min+arg for the global max-pool; or,
//   for dgrad, the ReLU/dropout mask of the previous layer and its BN-backward sums.
// * MFMA: v_mfma_f32_16x16x32_bf16 (bf16 path) or v_mfma_f32_16x16x4_f32 (fp32 parity
//   path: exact f32 products, one rounding per FMA).  Operands are swapped (W as the
//   MFMA A operand) so each lane owns 4 consecutive output channels of one point.
// * LDS operand tiles are 64 B per row (one k-step) with a 16-B-slot XOR swizzle that
//   makes the ds_read_b128 fragment reads bank-conflict free.
// * A workgroup walks a scene-aligned chunk of row tiles for one column block; blocks
//   that share a chunk are mapped onto one XCD (round-robin dispatch, speed only).
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int ROWB = 64;  // bytes per LDS operand row (one k-step)

PCS_DEV int swz(int row, int slot) { return slot ^ ((-(row >> 2)) & 3); }

template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  static constexpr int KSTEP = 32;  // elements per k-step (64 B)
  static constexpr int KK = 1;      // MFMA k-iterations per k-step
  typedef bf16x8 frag;
  static PCS_DEV frag load(const char *tile, int row, int lane, int kk) {
    (void)kk;
    return *reinterpret_cast<const frag *>(tile + row * ROWB + swz(row, lane >> 4) * 16);
  }
  static PCS_DEV f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  static constexpr int KSTEP = 16;
  static constexpr int KK = 4;
  typedef float frag;
  static PCS_DEV frag load(const char *tile, int row, int lane, int kk) {
    return *reinterpret_cast<const float *>(tile + row * ROWB + swz(row, kk) * 16 +
                                            (lane >> 4) * 4);
  }
  static PCS_DEV f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

// bijective XCD-grouping remap of the linear block id (cdna_hip_programming.md §5)
PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

constexpr int KMAX = 1024;   // prologue coefficient arrays staged in LDS (K <= KMAX)

template <int PRO> struct Coef {   // per-channel prologue arrays kept in LDS
  static constexpr int N = (PRO == PCS_PRO_BNRELU || PRO == PCS_PRO_CAT) ? 2 : PRO == PCS_PRO_BWD ? 3
                           : PRO == PCS_PRO_BWD_POOL ? 4 : 0;
};

template <int EPC>
PCS_DEV void lds_vec(const float *p, float (&v)[EPC]) {
#pragma unroll
  for (int e = 0; e < EPC; e += 4) {
    const float4 q = *reinterpret_cast<const float4 *>(p + e);
    v[e] = q.x; v[e + 1] = q.y; v[e + 2] = q.z; v[e + 3] = q.w;
  }
}

// Staging of one k-step: global -> registers (issued one k-step ahead) ...
template <typename T, int BM, int BN, int PRO, bool MASK>
PCS_DEV void nt_load(const pcs_gemm_args &a, const T *__restrict__ Ag, const T *__restrict__ A2g,
                     const T *__restrict__ Wg, int64_t row_base, int valid, int K, int n0, int k0,
                     int srow, u32x4 (&ra)[BM / 64], u32x4 (&ra2)[BM / 64], u32x4 (&rb)[BN / 64],
                     uint32_t (&mk)[BM / 64]) {
  constexpr int EPC = Elem<T>::EPC;
  if constexpr (PRO == PCS_PRO_CAT) {   // k-steps never straddle K1 (a multiple of the k-step)
    const int K1 = a.K1, K2 = K - K1;
    const bool first = k0 < K1;
#pragma unroll
    for (int i = 0; i < BM / 64; ++i) {
      const int r = min(srow + 64 * i, valid - 1);
      ra[i] = first ? *reinterpret_cast<const u32x4 *>(Ag + (row_base + r) * K1 + k0)
                    : *reinterpret_cast<const u32x4 *>(A2g + (row_base + r) * K2 + (k0 - K1));
    }
    const T *W2g = reinterpret_cast<const T *>(a.W2);
#pragma unroll
    for (int i = 0; i < BN / 64; ++i) {
      const int64_t n = n0 + srow + 64 * i;
      rb[i] = first ? *reinterpret_cast<const u32x4 *>(Wg + n * K1 + k0)
                    : *reinterpret_cast<const u32x4 *>(W2g + n * K2 + (k0 - K1));
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < BM / 64; ++i) {
    const int r = min(srow + 64 * i, valid - 1);   // clamped: rows >= valid are zeroed later
    const int64_t off = (row_base + r) * K + k0;
    ra[i] = *reinterpret_cast<const u32x4 *>(Ag + off);
    if constexpr (PRO == PCS_PRO_BWD) ra2[i] = *reinterpret_cast<const u32x4 *>(A2g + off);
    if constexpr (MASK) {
      const uint32_t byte = a.a_mask[off >> 3];
      mk[i] = EPC == 8 ? byte : (byte >> (k0 & 7)) & 0xFu;
    }
  }
#pragma unroll
  for (int i = 0; i < BN / 64; ++i)
    rb[i] = *reinterpret_cast<const u32x4 *>(Wg + (int64_t)(n0 + srow + 64 * i) * K + k0);
}

// ... then prologue transform (coefficients from LDS) and registers -> LDS
template <typename T, int BM, int BN, int PRO, bool MASK>
PCS_DEV void nt_store(const pcs_gemm_args &a, char *tA, const float *cf, int64_t row_base, int valid,
                      int k0, int slot, int srow, const u32x4 (&ra)[BM / 64],
                      const u32x4 (&ra2)[BM / 64], const u32x4 (&rb)[BN / 64],
                      const uint32_t (&mk)[BM / 64]) {
  constexpr int EPC = Elem<T>::EPC;
  char *tB = tA + BM * ROWB;
  float c0[EPC], c1[EPC], c2[EPC];
  const bool cat2 = PRO == PCS_PRO_CAT && k0 >= a.K1;   // the BN+ReLU part of a CAT operand
  if constexpr (PRO == PCS_PRO_BNRELU) {
    lds_vec<EPC>(cf + k0, c0); lds_vec<EPC>(cf + KMAX + k0, c1);
  } else if constexpr (PRO == PCS_PRO_CAT) {
    if (cat2) { lds_vec<EPC>(cf + (k0 - a.K1), c0); lds_vec<EPC>(cf + KMAX + (k0 - a.K1), c1); }
  } else if constexpr (PRO == PCS_PRO_BWD || PRO == PCS_PRO_BWD_POOL) {
    lds_vec<EPC>(cf + k0, c0); lds_vec<EPC>(cf + KMAX + k0, c1); lds_vec<EPC>(cf + 2 * KMAX + k0, c2);
  }
#pragma unroll
  for (int i = 0; i < BM / 64; ++i) {
    const int r = srow + 64 * i;
    float v[EPC];
    unpack_chunk(ra[i], v);
    if constexpr (PRO == PCS_PRO_BNRELU) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        float x = relu(fmaf(v[e], c0[e], c1[e]));
        if constexpr (MASK) x *= ((mk[i] >> e) & 1u) ? a.a_keep_scale : 0.f;
        v[e] = x;
      }
    } else if constexpr (PRO == PCS_PRO_CAT) {
      if (cat2) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = relu(fmaf(v[e], c0[e], c1[e]));
      }
    } else if constexpr (PRO == PCS_PRO_BWD) {
      float y[EPC];
      unpack_chunk(ra2[i], y);
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] = fmaf(c0[e], v[e], fmaf(c2[e], y[e], c1[e]));
    } else if constexpr (PRO == PCS_PRO_BWD_POOL) {
      const int grow = (int)(row_base + r);
      const int *am = reinterpret_cast<const int *>(cf + 3 * KMAX) + k0;
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] = fmaf(c2[e], v[e], c1[e]) + (am[e] == grow ? c0[e] : 0.f);
    }
    u32x4 out = (PRO == PCS_PRO_RAW || (PRO == PCS_PRO_CAT && !cat2)) ? ra[i] : pack_chunk(v);
    if (r >= valid) out = mk_u32x4(0, 0, 0, 0);
    *reinterpret_cast<u32x4 *>(tA + r * ROWB + swz(r, slot) * 16) = out;
  }
#pragma unroll
  for (int i = 0; i < BN / 64; ++i) {
    const int r = srow + 64 * i;
    *reinterpret_cast<u32x4 *>(tB + r * ROWB + swz(r, slot) * 16) = rb[i];
  }
}

template <typename T, int BM, int BN, int PRO, int EPI, bool POOL, bool MASK, bool SPARSE>
__global__ __launch_bounds__(THREADS, 2) void gemm_nt_kernel(pcs_gemm_args a, int tiles_per_scene,
                                                          int tiles_per_chunk, int ncb) {
  constexpr int EPC = Elem<T>::EPC;
  constexpr int SZ = Elem<T>::SIZE;
  constexpr int KSTEP = Mfma<T>::KSTEP;
  constexpr int WTM = BM / 2, WTN = BN / 2;  // 2x2 waves
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int ACH = BM / 64, BCH = BN / 64;  // 16-B chunks per thread per k-step
  constexpr int STAGE_BYTES = 2 * (BM + BN) * ROWB;
  constexpr int CROW = BN * SZ + 16;           // epilogue tile row stride (bytes)
  constexpr int CTILE_BYTES = BM * CROW;
  constexpr int CPR = BN * SZ / 16;            // chunks per output row
  constexpr int RPP = THREADS / CPR;           // rows per epilogue pass
  constexpr int RED_BYTES = RPP * BN * 16;
  constexpr int MAIN_BYTES = STAGE_BYTES > CTILE_BYTES
                                 ? (STAGE_BYTES > RED_BYTES ? STAGE_BYTES : RED_BYTES)
                                 : (CTILE_BYTES > RED_BYTES ? CTILE_BYTES : RED_BYTES);
  constexpr int PCOEF = Coef<PRO>::N * KMAX;            // floats
  constexpr int ECOEF = EPI == PCS_EPI_DGRAD ? 4 * BN : 0;
  constexpr int SPMAX = 1024;                            // sparse rows: [pool_c] idx | coef | bitmap
  constexpr int SP_BYTES = SPARSE ? 2 * SPMAX * 4 + BM / 8 : 0;
  constexpr int LDS_BYTES = MAIN_BYTES + 4 * (PCOEF + ECOEF) + SP_BYTES;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float *cf = reinterpret_cast<float *>(lds + MAIN_BYTES);
  float *ecf = cf + PCOEF;
  int *spi = reinterpret_cast<int *>(ecf + ECOEF);
  float *spc = reinterpret_cast<float *>(spi + SPMAX);
  uint32_t *tbits = reinterpret_cast<uint32_t *>(spc + SPMAX);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = L / ncb, cb = L % ncb;
  const int cps = a.chunks_per_scene;
  const int scene = chunk / cps, cis = chunk % cps;
  const int n0 = cb * BN;
  const int K = a.K, Ncols = a.Ncols;
  const int64_t N = a.scene_rows;
  const int t_begin = cis * tiles_per_chunk;
  const int t_end = min(t_begin + tiles_per_chunk, tiles_per_scene);
  const int nks = K / KSTEP;
  if (t_begin >= t_end) return;  // uniform across the block

  const T *__restrict__ Ag = reinterpret_cast<const T *>(a.A);
  const T *__restrict__ A2g = reinterpret_cast<const T *>(a.A2);
  const T *__restrict__ Wg = reinterpret_cast<const T *>(a.W);
  T *__restrict__ Cg = reinterpret_cast<T *>(a.C);

  // per-channel coefficients -> LDS (a workgroup's rows never leave its scene)
  for (int k = tid; k < (PRO == PCS_PRO_CAT ? K - a.K1 : K); k += THREADS) {
    if constexpr (PRO == PCS_PRO_BNRELU || PRO == PCS_PRO_CAT) {
      cf[k] = a.pa[k]; cf[KMAX + k] = a.pb[k];
    } else if constexpr (PRO == PCS_PRO_BWD) {
      cf[k] = a.pa[k]; cf[KMAX + k] = a.pb[k]; cf[2 * KMAX + k] = a.pc[k];
    } else if constexpr (PRO == PCS_PRO_BWD_POOL) {
      cf[k] = a.pool_coef[(int64_t)scene * K + k]; cf[KMAX + k] = a.pb[k]; cf[2 * KMAX + k] = a.pc[k];
      reinterpret_cast<int *>(cf)[3 * KMAX + k] = a.pool_idx[(int64_t)scene * K + k];
    }
  }
  if constexpr (EPI == PCS_EPI_DGRAD) {   // NULL es/et: mask Yp > 0; NULL erstd: no S2
    for (int c = tid; c < BN; c += THREADS) {
      ecf[c] = a.es ? a.es[n0 + c] : 1.f; ecf[BN + c] = a.et ? a.et[n0 + c] : 0.f;
      ecf[2 * BN + c] = a.emean ? a.emean[n0 + c] : 0.f; ecf[3 * BN + c] = a.erstd ? a.erstd[n0 + c] : 0.f;
    }
  }
  if constexpr (SPARSE) {
    for (int c = tid; c < a.pool_c; c += THREADS) {
      spi[c] = a.pool_idx[(int64_t)scene * a.pool_c + c];
      spc[c] = a.pool_coef[(int64_t)scene * a.pool_c + c];
    }
  }

  const int slot = tid & 3;           // staging: fixed k-slot per thread
  const int srow = tid >> 2;          // staging: row (+64*i)

  // epilogue thread mapping (fixed columns per thread)
  const int ecc = tid % CPR, er0 = tid / CPR;
  const int ecol = n0 + ecc * EPC;

  // per-thread epilogue accumulators
  float st_mean[EPC], st_m2[EPC], st_cnt = 0.f;
  float pmax[EPC], pmin[EPC];
  int pmaxi[EPC], pmini[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    st_mean[e] = 0.f; st_m2[e] = 0.f;
    pmax[e] = -__builtin_huge_valf(); pmin[e] = __builtin_huge_valf();
    pmaxi[e] = 0x7fffffff; pmini[e] = 0x7fffffff;
  }

  auto tile_rows = [&](int tile) { return (int)pcs_min64(BM, N - (int64_t)tile * BM); };
  u32x4 ra[ACH], ra2[ACH], rb[BCH];
  uint32_t mk[ACH];
  int64_t row_base = scene * N + (int64_t)t_begin * BM;
  int valid = tile_rows(t_begin);
  nt_load<T, BM, BN, PRO, MASK>(a, Ag, A2g, Wg, row_base, valid, K, n0, slot * EPC, srow, ra, ra2, rb, mk);
  __syncthreads();   // coefficients visible

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int64_t next_base = row_base + BM;
    const int next_valid = tile + 1 < t_end ? tile_rows(tile + 1) : 0;
    // ONE load site per k-step (see gemm_big.hip): step ks+1 of this tile, else step 0 of
    // the next tile, else an in-bounds reload that is never consumed
    auto prefetch = [&](int ks_next) {
      const bool tail = ks_next >= nks;
      const bool nxt = tail && next_valid > 0;
      nt_load<T, BM, BN, PRO, MASK>(a, Ag, A2g, Wg, nxt ? next_base : row_base, nxt ? next_valid : valid,
                                    K, n0, (tail ? 0 : ks_next) * KSTEP + slot * EPC, srow, ra, ra2, rb, mk);
    };

    if constexpr (SPARSE) {   // bitmap of the tile's rows that carry sparse terms
      __syncthreads();
      if (tid < BM / 32) tbits[tid] = 0u;
      __syncthreads();
      for (int c = tid; c < a.pool_c; c += THREADS) {
        const int64_t m = (int64_t)spi[c] - row_base;
        if (m >= 0 && m < valid) atomicOr(&tbits[m >> 5], 1u << (m & 31));
      }
      __syncthreads();
    }

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    nt_store<T, BM, BN, PRO, MASK>(a, lds, cf, row_base, valid, slot * EPC, slot, srow, ra, ra2, rb, mk);
    __builtin_amdgcn_sched_barrier(0);
    prefetch(1);
    lds_barrier();
    for (int ks = 0; ks < nks; ++ks) {
      const int buf = ks & 1;
      const char *tA = lds + buf * (BM + BN) * ROWB;
      const char *tB = tA + BM * ROWB;
#pragma unroll
      for (int kk = 0; kk < Mfma<T>::KK; ++kk) {
        typename Mfma<T>::frag af[FM], bf[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = Mfma<T>::load(tA, wm * WTM + i * 16 + (lane & 15), lane, kk);
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[j] = Mfma<T>::load(tB, wn * WTN + j * 16 + (lane & 15), lane, kk);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = Mfma<T>::mma(bf[j], af[i], acc[i][j]);
      }
      if (ks + 1 < nks) {
        nt_store<T, BM, BN, PRO, MASK>(a, lds + (buf ^ 1) * (BM + BN) * ROWB, cf, row_base, valid,
                                       (ks + 1) * KSTEP + slot * EPC, slot, srow, ra, ra2, rb, mk);
        __builtin_amdgcn_sched_barrier(0);
        prefetch(ks + 2);
      }
      lds_barrier();
    }

    // ---- epilogue phase 1: accumulators (+bias) -> LDS tile [BM][BN] in T ----
    {
      const float *bias = nullptr;
      if constexpr (EPI == PCS_EPI_FWD || EPI == PCS_EPI_BNRELU)
        bias = a.scene_bias ? a.scene_bias + scene * Ncols : a.bias;
      else if constexpr (EPI == PCS_EPI_DGRAD)
        bias = a.bias;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = wm * WTM + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = wn * WTN + j * 16 + 4 * (lane >> 4);
          float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
          if (bias) {
            const float4 bb = *reinterpret_cast<const float4 *>(bias + n0 + n);
            v0 += bb.x; v1 += bb.y; v2 += bb.z; v3 += bb.w;
          }
          if constexpr (EPI == PCS_EPI_BNRELU) {   // this layer's BN + ReLU on the way out
            const float4 s4 = *reinterpret_cast<const float4 *>(a.es + n0 + n);
            const float4 t4 = *reinterpret_cast<const float4 *>(a.et + n0 + n);
            v0 = relu(fmaf(v0, s4.x, t4.x)); v1 = relu(fmaf(v1, s4.y, t4.y));
            v2 = relu(fmaf(v2, s4.z, t4.z)); v3 = relu(fmaf(v3, s4.w, t4.w));
          }
          char *dst = lds + m * CROW + n * SZ;
          if constexpr (SZ == 4) {
            *reinterpret_cast<float4 *>(dst) = make_float4(v0, v1, v2, v3);
          } else {
            *reinterpret_cast<uint2 *>(dst) = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
          }
        }
      }
    }
    __syncthreads();

    // ---- epilogue phase 2: coalesced row chunks ----
    {
      float es[EPC], et[EPC], em[EPC], er[EPC];
      if constexpr (EPI == PCS_EPI_DGRAD) {
        const int lc = ecc * EPC;
        lds_vec<EPC>(ecf + lc, es); lds_vec<EPC>(ecf + BN + lc, et);
        lds_vec<EPC>(ecf + 2 * BN + lc, em); lds_vec<EPC>(ecf + 3 * BN + lc, er);
      }
      const T *Ypg = reinterpret_cast<const T *>(a.Yp);
      const T *Addg = reinterpret_cast<const T *>(a.addend);
      // BM/RPP rows per thread; the global loads of each batch are issued together so the
      // epilogue is bandwidth- rather than latency-bound (accumulators are dead here)
      constexpr int NP = BM / RPP;
      constexpr int BATCH = NP < 4 ? NP : 4;
#pragma unroll
      for (int p0 = 0; p0 < NP; p0 += BATCH) {
        u32x4 yv[BATCH], adv[BATCH];
        uint32_t mb[BATCH];
        if constexpr (EPI == PCS_EPI_DGRAD) {
#pragma unroll
          for (int q = 0; q < BATCH; ++q) {
            const int rr = min(er0 + RPP * (p0 + q), valid - 1);
            const int64_t goff = (row_base + rr) * Ncols + ecol;
            yv[q] = *reinterpret_cast<const u32x4 *>(Ypg + goff);
            adv[q] = Addg ? *reinterpret_cast<const u32x4 *>(Addg + goff) : mk_u32x4(0, 0, 0, 0);
            mb[q] = a.c_mask ? mask_bits(a.c_mask, row_base + rr, Ncols, ecol, EPC) : 0xffu;
          }
        }
#pragma unroll
        for (int q = 0; q < BATCH; ++q) {
          const int rr = er0 + RPP * (p0 + q);
          if (rr < valid) {
            const int64_t grow = row_base + rr;
            const int64_t goff = grow * Ncols + ecol;
            const u32x4 raw = *reinterpret_cast<const u32x4 *>(lds + rr * CROW + ecc * 16);
            float v[EPC];
            unpack_chunk(raw, v);
            if constexpr (EPI == PCS_EPI_FWD) {
              if (Cg) st16(Cg + goff, raw);
              if (a.stats) {
                st_cnt += 1.f;
                const float rn = 1.f / st_cnt;
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                  const float d = v[e] - st_mean[e];
                  st_mean[e] = fmaf(d, rn, st_mean[e]);
                  st_m2[e] = fmaf(d, v[e] - st_mean[e], st_m2[e]);
                }
              }
              if constexpr (POOL) {
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                  if (pool_max_step(v[e], pmax[e], pmaxi[e])) { pmax[e] = v[e]; pmaxi[e] = (int)grow; }
                  if (pool_min_step(v[e], pmin[e], pmini[e])) { pmin[e] = v[e]; pmini[e] = (int)grow; }
                }
              }
            } else if constexpr (EPI == PCS_EPI_DGRAD) {
              if (Addg) {
                float ad[EPC];
                unpack_chunk(adv[q], ad);
#pragma unroll
                for (int e = 0; e < EPC; ++e) v[e] += ad[e];
              }
              if constexpr (SPARSE) {   // rare: rows carrying max-pool terms (pool_w)
                if ((tbits[rr >> 5] >> (rr & 31)) & 1u) {
                  for (int c = 0; c < a.pool_c; ++c) {
                    if (spi[c] != (int)grow) continue;
                    const float w = spc[c];
                    const float *wr = a.pool_w + (int64_t)c * a.pool_ldw + ecol;
#pragma unroll
                    for (int e = 0; e < EPC; ++e) v[e] = fmaf(w, wr[e], v[e]);
                  }
                }
              }
              if (a.c_mask) {
#pragma unroll
                for (int e = 0; e < EPC; ++e) v[e] *= ((mb[q] >> e) & 1u) ? a.c_keep_scale : 0.f;
              }
              float y[EPC];
              unpack_chunk(yv[q], y);
#pragma unroll
              for (int e = 0; e < EPC; ++e) {
                const float dz = fmaf(y[e], es[e], et[e]) > 0.f ? v[e] : 0.f;
                v[e] = dz;
                st_mean[e] += dz;                                        // S1
                st_m2[e] = fmaf(dz, (y[e] - em[e]) * er[e], st_m2[e]);   // S2
              }
              st16(Cg + goff, pack_chunk(v));
            } else {  // RAW
              st16(Cg + goff, raw);
            }
          }
        }
      }
    }
    __syncthreads();
    row_base = next_base;
    valid = next_valid;
  }

  // ---- chunk end: cross-thread reduction of the per-thread partials ----
  const int64_t chunk_id = (int64_t)scene * cps + cis;
  if constexpr (EPI == PCS_EPI_FWD || EPI == PCS_EPI_DGRAD) {
    if (a.stats) {
      float4 *red = reinterpret_cast<float4 *>(lds);  // [RPP][BN]
#pragma unroll
      for (int e = 0; e < EPC; ++e)
        red[er0 * BN + ecc * EPC + e] = make_float4(st_cnt, st_mean[e], st_m2[e], 0.f);
      __syncthreads();
      for (int c = tid; c < BN; c += THREADS) {
        float n = 0.f, mean = 0.f, m2 = 0.f;
        for (int j = 0; j < RPP; ++j) {
          const float4 q = red[j * BN + c];
          if constexpr (EPI == PCS_EPI_FWD) {
            chan_merge(n, mean, m2, q.x, q.y, q.z);
          } else {
            mean += q.y; m2 += q.z;
          }
        }
        *reinterpret_cast<float2 *>(a.stats + (chunk_id * Ncols + n0 + c) * 2) = make_float2(mean, m2);
      }
      __syncthreads();
    }
  }
  if constexpr (POOL) {
    float4 *red = reinterpret_cast<float4 *>(lds);
#pragma unroll
    for (int e = 0; e < EPC; ++e)
      red[er0 * BN + ecc * EPC + e] =
          make_float4(pmax[e], __int_as_float(pmaxi[e]), pmin[e], __int_as_float(pmini[e]));
    __syncthreads();
    for (int c = tid; c < BN; c += THREADS) {
      float mx = -__builtin_huge_valf(), mn = __builtin_huge_valf();
      int mxi = 0x7fffffff, mni = 0x7fffffff;
      for (int j = 0; j < RPP; ++j) {
        const float4 q = red[j * BN + c];
        const int qi = __float_as_int(q.y), qj = __float_as_int(q.w);
        if (pool_max_wins(q.x, qi, mx, mxi)) { mx = q.x; mxi = qi; }
        if (pool_min_wins(q.z, qj, mn, mni)) { mn = q.z; mni = qj; }
      }
      *reinterpret_cast<float4 *>(a.pool + (chunk_id * Ncols + n0 + c) * 4) =
          make_float4(mx, __int_as_float(mxi), mn, __int_as_float(mni));
    }
  }
}

template <typename T, int BM, int BN, int PRO, int EPI, bool POOL, bool SPARSE = false>
int launch_t(const pcs_gemm_args &a, int tps, int tpc, hipStream_t s) {
  const int ncb = a.Ncols / BN;
  const int nb = ncb * (int)(a.num_scenes * a.chunks_per_scene);
  if (PRO == PCS_PRO_BNRELU && a.a_mask)
    hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, PRO, EPI, POOL, PRO == PCS_PRO_BNRELU, SPARSE>), dim3(nb),
                       dim3(THREADS), 0, s, a, tps, tpc, ncb);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, PRO, EPI, POOL, false, SPARSE>), dim3(nb), dim3(THREADS), 0, s,
                       a, tps, tpc, ncb);
  PCS_CHECK_LAUNCH();
  return 0;
}

template <typename T, int BN>
int dispatch_pro_epi(const pcs_gemm_args &a, int tps, int tpc, hipStream_t s) {
  constexpr int BM = 128;
  const bool pool = a.pool != nullptr;
  switch (a.epilogue) {
    case PCS_EPI_FWD:
      switch (a.prologue) {
        case PCS_PRO_BNRELU:
          return pool ? launch_t<T, BM, BN, PCS_PRO_BNRELU, PCS_EPI_FWD, true>(a, tps, tpc, s)
                      : launch_t<T, BM, BN, PCS_PRO_BNRELU, PCS_EPI_FWD, false>(a, tps, tpc, s);
        case PCS_PRO_RAW:
          return pool ? launch_t<T, BM, BN, PCS_PRO_RAW, PCS_EPI_FWD, true>(a, tps, tpc, s)
                      : launch_t<T, BM, BN, PCS_PRO_RAW, PCS_EPI_FWD, false>(a, tps, tpc, s);
        default: break;
      }
      break;
    case PCS_EPI_DGRAD:
      switch (a.prologue) {
        case PCS_PRO_BWD: return launch_t<T, BM, BN, PCS_PRO_BWD, PCS_EPI_DGRAD, false>(a, tps, tpc, s);
        case PCS_PRO_BWD_POOL:
          return launch_t<T, BM, BN, PCS_PRO_BWD_POOL, PCS_EPI_DGRAD, false>(a, tps, tpc, s);
        case PCS_PRO_BNRELU:   // a_{l-1} H (folded BN backward of a wide layer, see pcs_bn_fold)
          return launch_t<T, BM, BN, PCS_PRO_BNRELU, PCS_EPI_DGRAD, false>(a, tps, tpc, s);
        case PCS_PRO_CAT:      // dz5 (diag alpha W5) + a4 H4 + c (conv5, folded, one pass)
          return launch_t<T, BM, BN, PCS_PRO_CAT, PCS_EPI_DGRAD, false>(a, tps, tpc, s);
        case PCS_PRO_RAW:      // a5 H + c + max-pool rows (global_feat, folded)
          return a.pool_w ? launch_t<T, BM, BN, PCS_PRO_RAW, PCS_EPI_DGRAD, false, true>(a, tps, tpc, s)
                          : launch_t<T, BM, BN, PCS_PRO_RAW, PCS_EPI_DGRAD, false>(a, tps, tpc, s);
        default: break;
      }
      break;
    case PCS_EPI_BNRELU:
      switch (a.prologue) {
        case PCS_PRO_BNRELU: return launch_t<T, BM, BN, PCS_PRO_BNRELU, PCS_EPI_BNRELU, false>(a, tps, tpc, s);
        case PCS_PRO_RAW: return launch_t<T, BM, BN, PCS_PRO_RAW, PCS_EPI_BNRELU, false>(a, tps, tpc, s);
        default: break;
      }
      break;
    case PCS_EPI_RAW:
      switch (a.prologue) {
        case PCS_PRO_BWD: return launch_t<T, BM, BN, PCS_PRO_BWD, PCS_EPI_RAW, false>(a, tps, tpc, s);
        case PCS_PRO_BWD_POOL:
          return launch_t<T, BM, BN, PCS_PRO_BWD_POOL, PCS_EPI_RAW, false>(a, tps, tpc, s);
        case PCS_PRO_BNRELU:
          return launch_t<T, BM, BN, PCS_PRO_BNRELU, PCS_EPI_RAW, false>(a, tps, tpc, s);
        default: break;
      }
      break;
  }
  return pcs_set_einval("pcs_gemm", "unsupported prologue/epilogue combination");
}

}  // namespace

static constexpr int GEMM_BM = 128;

// The row-chunk geometry depends only on shapes, dtype and flags, never on which optional
// operands are set: callers size their partial buffers from pcs_gemm_geometry() before the
// pointers exist.  Shapes the 256x256 kernels can take use 256-row-multiple chunks; if a call
// of that class ends up on the generic kernel (an operand combination the wide kernels do not
// implement), that kernel walks the same chunks in 128-row tiles.
static bool wide_class(const pcs_gemm_args &a) {
  if (a.prologue == PCS_PRO_CAT) return false;   // generic kernel only
  // seg_conv3's input gradient (K 128 -> 256 columns, DGRAD epilogue): the 128-row kernel
  // measured faster at cfg2 (3.13 vs 3.38 ms, tools/bench_bwd_shapes.py)
  if (a.K == 128 && a.Ncols == 256 && a.epilogue == PCS_EPI_DGRAD) return false;
  return a.dtype == PCS_BF16 && !(a.flags & PCS_FLAG_GENERIC) && a.K % 64 == 0 && a.Ncols % 256 == 0 &&
         a.K >= 128 && a.K <= 1024;
}

extern "C" int64_t pcs_gemm_geometry(pcs_gemm_args *a) {
  if (!a || a->num_scenes <= 0 || a->scene_rows <= 0 || a->Ncols <= 0)
    return pcs_set_einval("pcs_gemm_geometry", "empty geometry");
  int fs_target = 256;
  if (const int nbc = pcs_fwd_stream_nb(*a, &fs_target))   // streaming forward
    return pcs_fill_geometry(a, 256, fs_target, a->Ncols / nbc);
  if (wide_class(*a))
    return pcs_fill_geometry(a, PCS_BIG_BM, 256, a->Ncols / 256);   // one 512-thread WG per CU
  if (pcs_c5_dgrad_class(*a))   // conv5's folded input gradient: one 512-thread WG per CU
    return pcs_fill_geometry(a, GEMM_BM, 256, 1);
  const int64_t ncb = a->Ncols >= 128 ? a->Ncols / 128 : 1;
  return pcs_fill_geometry(a, GEMM_BM, 2048, ncb);                 // ~8 WGs per CU
}

extern "C" int pcs_gemm(const pcs_gemm_args *ap, pcs_stream_t stream) {
  if (!ap) return pcs_set_einval("pcs_gemm", "null args");
  pcs_gemm_args a = *ap;
  if (a.K <= 0 || a.Ncols <= 0) return pcs_set_einval("pcs_gemm", "K/Ncols must be positive");
  if (a.Ncols % 64 != 0) return pcs_set_einval("pcs_gemm", "Ncols must be a multiple of 64");
  const int kstep = a.dtype == PCS_BF16 ? 32 : 16;
  if (a.K % kstep != 0) return pcs_set_einval("pcs_gemm", "K must be a multiple of the k-step");
  if (!a.A || !a.W) return pcs_set_einval("pcs_gemm", "A and W are required");
  if (a.prologue == PCS_PRO_BWD && (!a.A2 || !a.pa || !a.pb || !a.pc))
    return pcs_set_einval("pcs_gemm", "PRO_BWD needs A2 (=Y_l), alpha, beta, gamma");
  if (a.prologue == PCS_PRO_BWD_POOL && (!a.pb || !a.pc || !a.pool_idx || !a.pool_coef))
    return pcs_set_einval("pcs_gemm", "PRO_BWD_POOL needs beta, gamma, pool_idx, pool_coef");
  if (a.prologue == PCS_PRO_BNRELU && (!a.pa || !a.pb))
    return pcs_set_einval("pcs_gemm", "PRO_BNRELU needs s and t");
  if (a.epilogue < PCS_EPI_FWD || a.epilogue > PCS_EPI_BNRELU) return pcs_set_einval("pcs_gemm", "bad epilogue");
  if (a.epilogue == PCS_EPI_DGRAD && (!a.Yp || !a.C || !a.es != !a.et || (a.erstd && !a.emean)))
    return pcs_set_einval("pcs_gemm", "EPI_DGRAD needs Yp and C (es/et both or neither, emean with erstd)");
  if (a.epilogue == PCS_EPI_BNRELU && (!a.es || !a.et || !a.C || a.pool))
    return pcs_set_einval("pcs_gemm", "EPI_BNRELU needs es, et and C (no pool)");
  // EPI_BNRELU statistics = per-chunk column sums of the stored output (bf16 256-wide kernel)
  if (a.epilogue == PCS_EPI_BNRELU && a.stats &&
      !(wide_class(a) && (pcs_gemm_wres_applicable(a) || pcs_gemm_big_applicable(a))))
    return pcs_set_einval("pcs_gemm", "EPI_BNRELU column sums need the bf16 256-wide kernel (Ncols % 256 == 0)");
  if (a.pool && a.epilogue != PCS_EPI_FWD) return pcs_set_einval("pcs_gemm", "pool needs EPI_FWD");
  if (a.pool_w && (a.epilogue != PCS_EPI_DGRAD || a.prologue != PCS_PRO_RAW || !a.pool_idx || !a.pool_coef ||
                   a.pool_c <= 0 || a.pool_c > 1024 || a.pool_ldw < a.Ncols))
    return pcs_set_einval("pcs_gemm", "pool_w (sparse rows) needs EPI_DGRAD, PRO_RAW, pool_idx, pool_coef, "
                                      "0 < pool_c <= 1024, pool_ldw >= Ncols");
  if (a.scene_rows * a.num_scenes >= (int64_t)1 << 31)
    return pcs_set_einval("pcs_gemm", "M must be < 2^31 rows");
  if (a.prologue == PCS_PRO_CAT) {
    if (!a.A2 || !a.W2 || !a.pa || !a.pb || a.K1 <= 0 || a.K1 >= a.K || a.K1 % kstep || a.K - a.K1 > KMAX ||
        a.epilogue != PCS_EPI_DGRAD || a.a_mask)
      return pcs_set_einval("pcs_gemm", "PRO_CAT needs A2, W2, pa, pb, 0 < K1 < K (a k-step multiple), "
                                        "K - K1 <= 1024, EPI_DGRAD, no a_mask");
  } else if (a.K > KMAX) {
    return pcs_set_einval("pcs_gemm", "K must be <= 1024");
  }
  if ((a.flags & PCS_FLAG_AW_FP8) && !(wide_class(a) && pcs_gemm_glds_applicable(a)))
    return pcs_set_einval("pcs_gemm", "fp8 operands (PCS_FLAG_AW_FP8) need the LDS-DMA kernel: bf16 C, RAW prologue, "
                                      "K % 256 == 0, Ncols % 256 == 0, w_scale, FWD (no C) or folded DGRAD");
  if ((a.flags & PCS_FLAG_C_FP8) && !(a.epilogue == PCS_EPI_BNRELU &&
                                      (a.prologue == PCS_PRO_BNRELU || a.prologue == PCS_PRO_RAW) && !a.a_mask &&
                                      wide_class(a) && (pcs_gemm_wres_applicable(a) || pcs_gemm_big_applicable(a))))
    return pcs_set_einval("pcs_gemm", "fp8 output (PCS_FLAG_C_FP8) needs PRO_BNRELU (no dropout) or PRO_RAW + EPI_BNRELU "
                                      "on the bf16 256-wide kernel");
  if ((a.flags & PCS_FLAG_POOL_SIGNED_W) && !(a.epilogue == PCS_EPI_FWD && a.pool && a.es && !a.stats &&
                                             wide_class(a) && pcs_gemm_glds_applicable(a)))
    return pcs_set_einval("pcs_gemm", "PCS_FLAG_POOL_SIGNED_W needs EPI_FWD with pool and es, no statistics, on the "
                                      "LDS-DMA kernel");
  if (a.a_mask && a.prologue != PCS_PRO_BNRELU)
    return pcs_set_einval("pcs_gemm", "a_mask applies to the BNRELU prologue only");
  const int64_t rpc = pcs_gemm_geometry(&a);
  if (rpc < 0) return (int)rpc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a.gram && !(a.K == 64 && a.Ncols == 64 && a.epilogue == PCS_EPI_FWD && !a.a_mask && !a.scene_bias &&
                  pcs_fwd_stream_applicable(a)))
    return pcs_set_einval("pcs_gemm", "gram (the operand's Gram) needs bf16 PRO_BNRELU + EPI_FWD, K = Ncols = 64, "
                                      "no dropout bits, on the streaming kernel");
  if (pcs_fwd_stream_applicable(a)) return pcs_fwd_stream_launch(a, rpc, s);
  if (wide_class(a) && pcs_gemm_wres_applicable(a)) return pcs_gemm_wres_launch(a, rpc, s);
  if (wide_class(a) && pcs_gemm_glds_applicable(a)) {
    const int tps = (int)((a.scene_rows + PCS_BIG_BM - 1) / PCS_BIG_BM);
    return pcs_gemm_glds_launch(a, tps, (int)(rpc / PCS_BIG_BM), s);
  }
  if (wide_class(a) && pcs_gemm_big_applicable(a)) {
    const int tps = (int)((a.scene_rows + PCS_BIG_BM - 1) / PCS_BIG_BM);
    return pcs_gemm_big_launch(a, tps, (int)(rpc / PCS_BIG_BM), s);
  }
  if (pcs_c5_dgrad_applicable(a)) return pcs_c5_dgrad_launch(a, rpc, s);
  const int tps = (int)((a.scene_rows + GEMM_BM - 1) / GEMM_BM);
  const int tpc = (int)(rpc / GEMM_BM);
  const bool bn128 = a.Ncols % 128 == 0;
  if (a.dtype == PCS_BF16)
    return bn128 ? dispatch_pro_epi<bf16_t, 128>(a, tps, tpc, s) : dispatch_pro_epi<bf16_t, 64>(a, tps, tpc, s);
  if (a.dtype == PCS_F32)
    return bn128 ? dispatch_pro_epi<float, 128>(a, tps, tpc, s) : dispatch_pro_epi<float, 64>(a, tps, tpc, s);
  return pcs_set_einval("pcs_gemm", "bad dtype");
}

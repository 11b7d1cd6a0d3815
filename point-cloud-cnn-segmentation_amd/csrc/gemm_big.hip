// bf16 256x256x64 points-major GEMM (pcs_gemm for bf16 with Ncols % 256 == 0, K >= 128):
// the wide layers' forward and input-gradient GEMMs (global_feat M x 1024 x 1024 is 75 % of
// the model's MACs; conv5, seg_conv1/2/3; P:106-128 and their autograd at P:254).
//
// Same contract as gemm_nt.hip (pcs_gemm_args, scene-aligned row chunks, prologue and
// epilogue fusion) with a tile sized for MFMA throughput instead of generality:
// * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns 128 x 64 outputs =
//   8 x 4 v_mfma_f32_16x16x32_bf16 accumulators; 64 MFMAs per wave per 64-deep k-step.
// * operands staged global -> VGPR (BN+ReLU / BN-backward prologue, coefficients from LDS)
//   -> LDS, 128-B rows, 16-B slots XOR-swizzled with (row>>1)&7 so the ds_read_b128
//   fragment reads are bank-conflict free; two LDS stages, one raw barrier per k-step; the
//   loads of step ks+2 are issued right after step ks+1 is written (one load site).
// * epilogue: the tile goes through LDS (phase 1) and is walked in coalesced row chunks
//   (phase 2): bias / per-scene bias + store, or the previous layer's ReLU / dropout /
//   addend backward (EPI_DGRAD).  Column statistics (Welford; or the BN-backward sums
//   S1/S2) and max-pool max/min+argmax are per-thread over 16 rows, merged per tile
//   through LDS into running per-column accumulators and written once per chunk in the
//   generic kernel's partial layout.
#include "common.h"

#ifndef PCS_DGRAD_BATCH
#define PCS_DGRAD_BATCH 16  // DGRAD epilogue: rows of Yp (and mask / addend) loaded per batch (all 16)
#endif

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
constexpr int NPASS = BM / RPP;              // 16 rows per thread in phase 2
constexpr int LDS_MAIN = (2 * STAGE > CTILE) ? 2 * STAGE : CTILE;

// LDS layout after the main area: prologue coefficients | argmax bitmap | epilogue
// coefficients (DGRAD) | running per-column accumulators
template <int PRO, int EPI> struct Lay {
  static constexpr int NC = PRO == PCS_PRO_BNRELU ? 2 : PRO == PCS_PRO_BWD ? 3 : PRO == PCS_PRO_BWD_POOL ? 4 : 0;
  static constexpr int COEF = LDS_MAIN;
  static constexpr int BITS = COEF + NC * KMAX * 4;
  static constexpr int ECOEF = BITS + (PRO == PCS_PRO_BWD_POOL ? 32 : 0);
  static constexpr int RUN = ECOEF + (EPI == PCS_EPI_DGRAD ? 4 * BN * 4 : 0);
  static constexpr int BYTES = RUN + (EPI == PCS_EPI_FWD ? 6 * BN * 4 : (EPI == PCS_EPI_DGRAD || EPI == PCS_EPI_BNRELU) ? 2 * BN * 4 : 0);
  static_assert(BYTES <= 160 * 1024, "LDS budget");
};

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
// MASK: dropout keep bits of A (FWD prologue) or of C (DGRAD epilogue); ADD: DGRAD addend,
// or (BNRELU epilogue) an fp8 e4m3 output (PCS_FLAG_C_FP8)
template <int PRO, int EPI, bool MASK, bool ADD>
__global__ __launch_bounds__(THREADS) void gemm_big_kernel(pcs_gemm_args a, int tiles_per_scene,
                                                           int tiles_per_chunk, int ncb) {
  constexpr int EPC = 8;
  constexpr bool AMASK = MASK && PRO == PCS_PRO_BNRELU;   // dropout bits of the A operand
  constexpr bool CMASK = MASK && EPI == PCS_EPI_DGRAD;    // dropout bits of the dgrad output
  constexpr bool C8 = ADD && EPI == PCS_EPI_BNRELU;       // fp8 activation store
  typedef Lay<PRO, EPI> LY;
  __shared__ __attribute__((aligned(16))) char lds[LY::BYTES];
  float *cf = reinterpret_cast<float *>(lds + LY::COEF);
  uint32_t *tbits = reinterpret_cast<uint32_t *>(lds + LY::BITS);
  float *ecf = reinterpret_cast<float *>(lds + LY::ECOEF);   // DGRAD: es | et | emean | erstd
  float *run = reinterpret_cast<float *>(lds + LY::RUN);     // mean|m2|max|maxi|min|mini, S1|S2 or colsum

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
  const bool do_stats = a.stats != nullptr, do_pool = EPI == PCS_EPI_FWD && a.pool != nullptr;
  if (tid < BN) {
    if constexpr (EPI == PCS_EPI_DGRAD) {
      ecf[tid] = a.es[n0 + tid]; ecf[BN + tid] = a.et[n0 + tid];
      ecf[2 * BN + tid] = a.emean[n0 + tid]; ecf[3 * BN + tid] = a.erstd[n0 + tid];
      run[tid] = 0.f; run[BN + tid] = 0.f;
    } else if constexpr (EPI == PCS_EPI_FWD) {
      run[tid] = 0.f; run[BN + tid] = 0.f;
      run[2 * BN + tid] = -__builtin_huge_valf(); run[3 * BN + tid] = __int_as_float(0x7fffffff);
      run[4 * BN + tid] = __builtin_huge_valf(); run[5 * BN + tid] = __int_as_float(0x7fffffff);
    } else if constexpr (EPI == PCS_EPI_BNRELU) {
      run[tid] = 0.f; run[BN + tid] = 0.f;
    }
  }
  float run_n = 0.f;   // rows merged into the running statistics so far (uniform)

  const int slot = tid & 7, srow = tid >> 3;  // staging: rows srow + 64*i, fixed k-slot
  const int ecc_ = tid % CPR, er0_ = tid / CPR;
  const int ecc = ecc_, er0 = er0_, ecol = n0 + ecc * EPC;
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);

  u32x4 ra[4], ra2[4], rb[4];
  uint32_t mk[4];
  uint32_t hits = 0;   // POOL: bit i set if staging row srow + 64 i is an argmax row of the tile
  // Staging addresses: a uniform (SGPR) base per tile and k-step plus per-thread 32-bit byte
  // offsets computed once per tile (rows clamped to the tile's valid rows), so the loads use
  // the saddr + voffset form instead of 64-bit VALU address arithmetic every k-step.
  uint32_t woff[4], aoff[4], aoff_next[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) woff[i] = (uint32_t)(((srow + 64 * i) * K + slot * EPC) * 2);
  const char *wbase0 = reinterpret_cast<const char *>(Wg + (int64_t)n0 * K);
  auto row_offs = [&](int valid_rows, uint32_t (&o)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (uint32_t)((min(srow + 64 * i, valid_rows - 1) * K + slot * EPC) * 2);
  };
  auto load_stage = [&](int64_t row_base, const uint32_t (&o)[4], int ks) {
    const int64_t e0 = row_base * K + (int64_t)ks * BK;   // element offset of (row_base, k-step)
    const char *ab = reinterpret_cast<const char *>(Ag + e0);
    const char *wb = wbase0 + ks * BK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *reinterpret_cast<const u32x4 *>(ab + o[i]);
      if constexpr (PRO == PCS_PRO_BWD)
        ra2[i] = *reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(A2g + e0) + o[i]);
      if constexpr (AMASK) mk[i] = (a.a_mask + (e0 >> 3))[o[i] >> 4];
      rb[i] = *reinterpret_cast<const u32x4 *>(wb + woff[i]);
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
          float x = relu(fmaf(v[e], c0[e], c1[e]));
          if constexpr (AMASK) x *= ((mk[i] >> e) & 1u) ? a.a_keep_scale : 0.f;
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
  row_offs(valid, aoff);
  load_stage(row_base, aoff, 0);
  __syncthreads();   // coefficients visible

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int64_t next_base = row_base + BM;
    const int next_valid = (tile + 1 < t_end) ? tile_rows(tile + 1) : 0;
    // ONE load site per k-step (two sites make the compiler merge their registers with
    // copies that wait for the loads): step ks_next of this tile, else step 0 of the next
    // tile, else a harmless in-bounds reload that is never consumed.
    row_offs(next_valid > 0 ? next_valid : 1, aoff_next);
    auto prefetch = [&](int ks_next) {
      const bool tail = ks_next >= nks;
      const bool nxt = tail && next_valid > 0;
      uint32_t o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = nxt ? aoff_next[i] : aoff[i];
      load_stage(nxt ? next_base : row_base, o, tail ? 0 : ks_next);
    };
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
    prefetch(1);
    lds_barrier();

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

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
        prefetch(ks + 2);
      }
      lds_barrier();
    }

    // lane owns rows m = wm*128 + i*16 + (lane&15), cols n = wn*64 + j*16 + 4*(lane>>4) + r
    if constexpr (EPI == PCS_EPI_FWD || EPI == PCS_EPI_BNRELU) {
      const float *bias = a.scene_bias ? a.scene_bias + (int64_t)scene * Ncols : a.bias;
      if (bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 bb = *reinterpret_cast<const float4 *>(bias + n0 + wn * 64 + j * 16 + lcol);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            acc[i][j][0] += bb.x; acc[i][j][1] += bb.y; acc[i][j][2] += bb.z; acc[i][j][3] += bb.w;
          }
        }
      }
    }

    if constexpr (EPI == PCS_EPI_BNRELU) {   // this layer's BN + ReLU on the way out
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 s4 = *reinterpret_cast<const float4 *>(a.es + n0 + wn * 64 + j * 16 + lcol);
        const float4 t4 = *reinterpret_cast<const float4 *>(a.et + n0 + wn * 64 + j * 16 + lcol);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[i][j][0] = relu(fmaf(acc[i][j][0], s4.x, t4.x));
          acc[i][j][1] = relu(fmaf(acc[i][j][1], s4.y, t4.y));
          acc[i][j][2] = relu(fmaf(acc[i][j][2], s4.z, t4.z));
          acc[i][j][3] = relu(fmaf(acc[i][j][3], s4.w, t4.w));
        }
      }
    }

    // phase 1: tile -> LDS (bf16; fp8 store: e4m3 bytes rounded once from fp32, in the first
    // half of each tile row)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = wm * 128 + i * 16 + lrow;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = wn * 64 + j * 16 + lcol;
        if constexpr (C8)
          *reinterpret_cast<uint32_t *>(lds + m * CROW + n) =
              pack4fp8(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        else
          *reinterpret_cast<uint2 *>(lds + m * CROW + n * 2) =
              make_uint2(pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3]));
      }
    }
    __syncthreads();

    // phase 2: coalesced row chunks (thread: 8 columns ecc*8.., rows er0 + 16 p)
    float sa[EPC], sb[EPC];                      // Welford mean/M2, or S1/S2
    float pmx[EPC], pmn[EPC];
    int pmxi[EPC], pmni[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      sa[e] = 0.f; sb[e] = 0.f;
      pmx[e] = -__builtin_huge_valf(); pmn[e] = __builtin_huge_valf();
      pmxi[e] = 0x7fffffff; pmni[e] = 0x7fffffff;
    }
    // tile statistics are shifted by the tile's first row (same shift for every thread of a
    // column): per-thread sums of d = v - K, plain adds across threads, one Chan merge per
    // column per tile
    float ksh[EPC];
    float kc = 0.f;   // merge thread tid < BN: the shift of column tid
    if constexpr (EPI == PCS_EPI_FWD) {
      unpack_chunk(*reinterpret_cast<const u32x4 *>(lds + ecc * 16), ksh);
      if (tid < BN) kc = bf2f(*reinterpret_cast<const unsigned short *>(lds + tid * 2));
#pragma unroll 4
      for (int p = 0; p < NPASS; ++p) {
        const int rr = er0 + RPP * p;
        if (rr < valid) {
          const u32x4 raw = *reinterpret_cast<const u32x4 *>(lds + rr * CROW + ecc * 16);
          if (Cg) st16(Cg + (row_base + rr) * Ncols + ecol, raw);
          if (do_stats || do_pool) {
            float v[EPC];
            unpack_chunk(raw, v);
            if (do_stats) {
#pragma unroll
              for (int e = 0; e < EPC; ++e) {
                const float d = v[e] - ksh[e];
                sa[e] += d;
                sb[e] = fmaf(d, d, sb[e]);
              }
            }
            if (do_pool) {
              const int grow = (int)(row_base + rr);
#pragma unroll
              for (int e = 0; e < EPC; ++e) {
                if (pool_max_step(v[e], pmx[e], pmxi[e])) { pmx[e] = v[e]; pmxi[e] = grow; }
                if (pool_min_step(v[e], pmn[e], pmni[e])) { pmn[e] = v[e]; pmni[e] = grow; }
              }
            }
          }
        }
      }
    } else if constexpr (EPI == PCS_EPI_DGRAD) {
      // per-thread indices made opaque per tile: addresses derived from them are recomputed
      // here instead of hoisted out of the tile loop and spilled across the k-loop
      int ecc = ecc_, er0 = er0_;
      asm volatile("" : "+v"(ecc), "+v"(er0));
      const int ecol = n0 + ecc * EPC;
      const bf16_t *Ypg = reinterpret_cast<const bf16_t *>(a.Yp);
      const bf16_t *Addg = reinterpret_cast<const bf16_t *>(a.addend);
      float es[EPC], et[EPC];
      const int lc = ecc * EPC;
      lds_vec8(ecf + lc, es); lds_vec8(ecf + BN + lc, et);
      const float ks = a.c_keep_scale;
      constexpr int BATCH = ADD ? (PCS_DGRAD_BATCH + 1) / 2 : PCS_DGRAD_BATCH;
#pragma unroll
      for (int p0 = 0; p0 < NPASS; p0 += BATCH) {
        u32x4 yv[BATCH], adv[BATCH];
        uint32_t mb[BATCH];
#pragma unroll
        for (int q = 0; q < BATCH; ++q) {   // clamped loads, issued together
          const int rr = min(er0 + RPP * (p0 + q), valid - 1);
          const int64_t goff = (row_base + rr) * Ncols + ecol;
          yv[q] = *reinterpret_cast<const u32x4 *>(Ypg + goff);
          if constexpr (ADD) adv[q] = *reinterpret_cast<const u32x4 *>(Addg + goff);
          if constexpr (CMASK) mb[q] = a.c_mask[goff >> 3];
        }
#pragma unroll
        for (int q = 0; q < BATCH; ++q) {
          const int rr = er0 + RPP * (p0 + q);
          if (rr < valid) {
            const u32x4 raw = *reinterpret_cast<const u32x4 *>(lds + rr * CROW + ecc * 16);
            float v[EPC], y[EPC];
            unpack_chunk(raw, v);
            unpack_chunk(yv[q], y);
            if constexpr (ADD) {
              float ad[EPC];
              unpack_chunk(adv[q], ad);
#pragma unroll
              for (int e = 0; e < EPC; ++e) v[e] += ad[e];
            }
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
              float g = v[e];
              if constexpr (CMASK) g = ((mb[q] >> e) & 1u) ? g * ks : 0.f;
              const float dz = fmaf(y[e], es[e], et[e]) > 0.f ? g : 0.f;
              v[e] = dz;
              sa[e] += dz;                  // S1
              sb[e] = fmaf(dz, y[e], sb[e]);  // sum dz*y; S2 = rstd*(sum dz*y - mean*S1)
            }
            st16(Cg + (row_base + rr) * Ncols + ecol, pack_chunk(v));
          }
        }
      }
    } else {  // RAW / BNRELU
#pragma unroll 4
      for (int p = 0; p < NPASS; ++p) {
        const int rr = er0 + RPP * p;
        if (rr < valid) {
          if constexpr (C8) {   // fp8 e4m3 activation (8 B)
            const uint2 w8 = *reinterpret_cast<const uint2 *>(lds + rr * CROW + ecc * 8);
            const uint32_t lo = w8.x, hi = w8.y;
            __builtin_nontemporal_store((uint64_t)hi << 32 | lo,
                                        reinterpret_cast<uint64_t *>(reinterpret_cast<fp8_t *>(a.C) +
                                                                     (row_base + rr) * Ncols + ecol));
            if (do_stats) {   // column sums of the stored (fp8-rounded) activation
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                sa[e] += fp82f((lo >> (8 * e)) & 255u);
                sa[4 + e] += fp82f((hi >> (8 * e)) & 255u);
              }
            }
          } else {
            const u32x4 raw = *reinterpret_cast<const u32x4 *>(lds + rr * CROW + ecc * 16);
            st16(Cg + (row_base + rr) * Ncols + ecol, raw);
            if constexpr (EPI == PCS_EPI_BNRELU) {
              if (do_stats) {   // column sums of the stored (bf16-rounded) activation
                float v[EPC];
                unpack_chunk(raw, v);
#pragma unroll
                for (int e = 0; e < EPC; ++e) sa[e] += v[e];
              }
            }
          }
        }
      }
    }
    __syncthreads();   // the C tile has been consumed

    // per-tile merge of the per-thread partials into the running per-column accumulators
    if ((EPI == PCS_EPI_FWD || EPI == PCS_EPI_DGRAD || EPI == PCS_EPI_BNRELU) && (do_stats || do_pool)) {
      float2 *ps = reinterpret_cast<float2 *>(lds);                 // [RPP][BN] stats / S1,S2 / colsum
      float4 *pp = reinterpret_cast<float4 *>(lds + RPP * BN * 8);  // [RPP][BN] pool
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        const int c = ecc * EPC + e;
        if (do_stats) ps[er0 * BN + c] = make_float2(sa[e], sb[e]);
        if (do_pool) pp[er0 * BN + c] = make_float4(pmx[e], __int_as_float(pmxi[e]), pmn[e], __int_as_float(pmni[e]));
      }
      __syncthreads();
      if (tid < BN) {
        const int c = tid;
        if (do_stats) {
          if constexpr (EPI == PCS_EPI_FWD) {
            float s1 = 0.f, s2 = 0.f;   // shifted sums of the tile's valid rows
#pragma unroll
            for (int j = 0; j < RPP; ++j) {
              const float2 q = ps[j * BN + c];
              s1 += q.x; s2 += q.y;
            }
            const float nt = (float)valid, d1 = s1 / nt;
            float n = run_n, mean = run[c], m2 = run[BN + c];
            chan_merge(n, mean, m2, nt, kc + d1, relu(s2 - s1 * d1));
            run[c] = mean; run[BN + c] = m2;
          } else {
            float s1 = run[c], s2 = run[BN + c];
            for (int j = 0; j < RPP; ++j) {
              const float2 q = ps[j * BN + c];
              s1 += q.x; s2 += q.y;
            }
            run[c] = s1; run[BN + c] = s2;
          }
        }
        if (do_pool) {
          float mx = run[2 * BN + c], mn = run[4 * BN + c];
          int mxi = __float_as_int(run[3 * BN + c]), mni = __float_as_int(run[5 * BN + c]);
          for (int j = 0; j < RPP; ++j) {
            const float4 q = pp[j * BN + c];
            const int qi = __float_as_int(q.y), qj = __float_as_int(q.w);
            if (pool_max_wins(q.x, qi, mx, mxi)) { mx = q.x; mxi = qi; }
            if (pool_min_wins(q.z, qj, mn, mni)) { mn = q.z; mni = qj; }
          }
          run[2 * BN + c] = mx; run[3 * BN + c] = __int_as_float(mxi);
          run[4 * BN + c] = mn; run[5 * BN + c] = __int_as_float(mni);
        }
      }
      __syncthreads();   // partial area reused by the next tile's staging
    }
    run_n += (float)valid;
    row_base = next_base;
    valid = next_valid;
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i] = aoff_next[i];
  }

  // chunk end: this workgroup's per-column partials (same layout as gemm_nt)
  if ((EPI == PCS_EPI_FWD || EPI == PCS_EPI_DGRAD || EPI == PCS_EPI_BNRELU) && tid < BN) {
    const int64_t o = (int64_t)chunk * Ncols + n0 + tid;
    if (do_stats) {
      float s2 = run[BN + tid];
      if constexpr (EPI == PCS_EPI_DGRAD) s2 = ecf[3 * BN + tid] * (s2 - ecf[2 * BN + tid] * run[tid]);
      *reinterpret_cast<float2 *>(a.stats + o * 2) = make_float2(run[tid], s2);
    }
    if (do_pool)
      *reinterpret_cast<float4 *>(a.pool + o * 4) =
          make_float4(run[2 * BN + tid], run[3 * BN + tid], run[4 * BN + tid], run[5 * BN + tid]);
  }
}

template <int PRO, int EPI, bool MASK, bool ADD = false>
int launch(const pcs_gemm_args &a, int tps, int tpc, hipStream_t s) {
  const int ncb = a.Ncols / BN;
  const int nb = ncb * (int)(a.num_scenes * a.chunks_per_scene);
  hipLaunchKernelGGL((gemm_big_kernel<PRO, EPI, MASK, ADD>), dim3(nb), dim3(THREADS), 0, s, a, tps, tpc, ncb);
  PCS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

bool pcs_gemm_big_applicable(const pcs_gemm_args &a) {
  if (a.dtype != PCS_BF16 || a.K % BK != 0 || a.Ncols % BN != 0 || a.K < 128 || a.K > KMAX) return false;
  if (a.flags & PCS_FLAG_GENERIC) return false;
  if (a.a_mask && a.prologue != PCS_PRO_BNRELU) return false;
  if (a.epilogue == PCS_EPI_FWD || a.epilogue == PCS_EPI_BNRELU)
    return a.prologue == PCS_PRO_BNRELU || a.prologue == PCS_PRO_RAW;
  if (a.epilogue == PCS_EPI_DGRAD && (!a.es || !a.erstd || a.bias || a.pool_w)) return false;
  if (a.epilogue == PCS_EPI_DGRAD)   // BWD_POOL (global_feat) has neither a mask nor an addend
    return a.prologue == PCS_PRO_BWD ? !(a.c_mask && a.addend)
                                     : a.prologue == PCS_PRO_BWD_POOL && !a.c_mask && !a.addend;
  if (a.epilogue == PCS_EPI_RAW) return a.prologue == PCS_PRO_BWD || a.prologue == PCS_PRO_BWD_POOL;
  return false;
}

int pcs_gemm_big_launch(const pcs_gemm_args &g, int tps, int tpc, hipStream_t s) {
  switch (g.epilogue) {
    case PCS_EPI_FWD:
      if (g.prologue == PCS_PRO_RAW) return launch<PCS_PRO_RAW, PCS_EPI_FWD, false>(g, tps, tpc, s);
      return g.a_mask ? launch<PCS_PRO_BNRELU, PCS_EPI_FWD, true>(g, tps, tpc, s)
                      : launch<PCS_PRO_BNRELU, PCS_EPI_FWD, false>(g, tps, tpc, s);
    case PCS_EPI_BNRELU:
      if (g.prologue == PCS_PRO_RAW)   // (fp8 store: the eval path's split a4, pcs_bnrelu_bf16)
        return (g.flags & PCS_FLAG_C_FP8) ? launch<PCS_PRO_RAW, PCS_EPI_BNRELU, false, true>(g, tps, tpc, s)
                                          : launch<PCS_PRO_RAW, PCS_EPI_BNRELU, false>(g, tps, tpc, s);
      if (g.flags & PCS_FLAG_C_FP8) return launch<PCS_PRO_BNRELU, PCS_EPI_BNRELU, false, true>(g, tps, tpc, s);
      return g.a_mask ? launch<PCS_PRO_BNRELU, PCS_EPI_BNRELU, true>(g, tps, tpc, s)
                      : launch<PCS_PRO_BNRELU, PCS_EPI_BNRELU, false>(g, tps, tpc, s);
    case PCS_EPI_DGRAD:
      if (g.prologue == PCS_PRO_BWD_POOL) return launch<PCS_PRO_BWD_POOL, PCS_EPI_DGRAD, false>(g, tps, tpc, s);
      if (g.c_mask) return launch<PCS_PRO_BWD, PCS_EPI_DGRAD, true>(g, tps, tpc, s);
      if (g.addend) return launch<PCS_PRO_BWD, PCS_EPI_DGRAD, false, true>(g, tps, tpc, s);
      return launch<PCS_PRO_BWD, PCS_EPI_DGRAD, false>(g, tps, tpc, s);
    default:
      return g.prologue == PCS_PRO_BWD_POOL ? launch<PCS_PRO_BWD_POOL, PCS_EPI_RAW, false>(g, tps, tpc, s)
                                            : launch<PCS_PRO_BWD, PCS_EPI_RAW, false>(g, tps, tpc, s);
  }
}

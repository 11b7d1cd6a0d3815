// bf16 256x256 weight-gradient kernel for the wide layer (global_feat, 1024 x 1024:
// dW = dy^T x summed over all M points; autograd of P:113 at P:254).
//
// * 512 threads = 8 waves as 2 (Cout) x 4 (Cin); each wave owns 128 x 64 outputs
//   (8 x 4 v_mfma_f32_16x16x32_bf16 accumulators), 64 MFMAs per 64-row step.
// * dy = beta + gamma*y_g (+ alpha*dz at the max-pool argmax rows) and x = relu(bn5(y5))
//   are formed while staging [64 rows x 256 cols] tiles global -> VGPR -> LDS; the MFMA
//   operands are read back transposed with ds_read_b64_tr_b16 (rows permuted + 32-B
//   padded: the 8 rows one transposed read touches hit 8 distinct bank groups).
// * the M reduction is split into scene-aligned row slices; each workgroup writes one
//   fp32 partial tile and pcs_reduce_partials sums them in a fixed order.
// * Gram mode (DYMODE = PCS_PRO_BNRELU, pcs_gram): both operands are a = relu(Y*s + t) of
//   the same activations, only the upper 256-tiles of the symmetric a^T a are computed,
//   and the diagonal tiles also sum their x columns (sum_m a[m, k]).
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int TM = 256, TN = 256, MS = 64;
constexpr int ROWB = TM * 2 + 32;          // 544 B: padded LDS row
constexpr int OPB = MS * ROWB;             // one operand tile (34 KB)
constexpr int STAGE = 2 * OPB;
constexpr int COEF = 6 * 256 * 4;          // alpha|beta|gamma|argmax (Cout cols), s|t (Cin cols)
constexpr int LDS_BYTES = 2 * STAGE + COEF;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PCS_DEV int prow(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

PCS_DEV bf16x8 tr_frag(const char *tile, int r0, int r1, int col) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tile + r0 * ROWB + col * 2));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tile + r1 * ROWB + col * 2));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int DYMODE, bool MASK>
PCS_DEV void tn_load(const bf16_t *__restrict__ dZ, const bf16_t *__restrict__ Yg,
                     const bf16_t *__restrict__ Xg, const uint8_t *__restrict__ xmask, int64_t rbase,
                     int64_t rlast, int Cout, int Cin, int an, int bk, int r0, u32x4 (&rz)[4],
                     u32x4 (&ry)[4], u32x4 (&rx)[4], uint32_t (&mk)[4]) {
  // uniform (SGPR) step bases + 32-bit per-thread offsets (saddr + voffset loads): 64-bit
  // per-row addresses for three operands cost 24 VGPRs and spilled at the k-loop's peak
  const int lim = (int)pcs_min64(rlast - 1 - rbase, MS - 1);   // last valid row of the step
  const char *zb = reinterpret_cast<const char *>(dZ + rbase * Cout);
  const char *yb = reinterpret_cast<const char *>(Yg + rbase * Cout);
  const char *xb = reinterpret_cast<const char *>(Xg + rbase * Cin);
  const uint8_t *mb = MASK ? xmask + ((rbase * Cin) >> 3) : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = min(r0 + 16 * i, lim);
    const uint32_t oy = (uint32_t)(rl * Cout + an), ox = (uint32_t)(rl * Cin + bk);
    if constexpr (DYMODE == PCS_PRO_BWD) rz[i] = *reinterpret_cast<const u32x4 *>(zb + 2 * oy);
    ry[i] = *reinterpret_cast<const u32x4 *>(yb + 2 * oy);
    rx[i] = *reinterpret_cast<const u32x4 *>(xb + 2 * ox);
    if constexpr (MASK) mk[i] = mb[ox >> 3];
  }
}

PCS_DEV void lds8(const float *p, float (&v)[8]) {
  const float4 x = *reinterpret_cast<const float4 *>(p);
  const float4 y = *reinterpret_cast<const float4 *>(p + 4);
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}

// Transform one staged 64-row step (dy and x) and write it to LDS.  Coefficients come from
// the workgroup's LDS copy (cf: [alpha|pool coef][beta][gamma][argmax] over its 256 Cout
// columns, [s][t] over its 256 Cin columns); rows past the slice end are written as zeros.
template <int DYMODE, bool MASK, bool RAWG = false>
PCS_DEV void tn_store(const pcs_wgrad_args &a, char *tA, const float *cf, int64_t rbase, int64_t rlast,
                      int bk, int cc, int r0, const u32x4 (&rz)[4], const u32x4 (&ry)[4],
                      const u32x4 (&rx)[4], const uint32_t (&mk)[4], bool diag, float (&csum)[8]) {
  char *tB = tA + OPB;
  if constexpr (RAWG) {   // Gram of stored activations (a5): no transform, straight to LDS
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = r0 + 16 * i;
      const bool ok = rbase + rl < rlast;
      const u32x4 z = mk_u32x4(0, 0, 0, 0);
      *reinterpret_cast<u32x4 *>(tA + prow(rl) * ROWB + cc * 16) = ok ? ry[i] : z;
      *reinterpret_cast<u32x4 *>(tB + prow(rl) * ROWB + cc * 16) = ok ? rx[i] : z;
      if (diag && ok) {
        float w[8];
        unpack_chunk(rx[i], w);
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += w[e];
      }
    }
    return;
  }
  // dy rows first, then x rows: only one operand's coefficients are live at a time (the
  // k-loop runs at the 256-VGPR limit)
  const int c8 = cc * 8;
  {
    float ca[8], cb[8], cg[8];
    int am[8];
    lds8(cf + c8, ca);
    lds8(cf + 256 + c8, cb);
    lds8(cf + 512 + c8, cg);
    if constexpr (DYMODE == PCS_PRO_BWD_POOL) {
      const int4 i0 = *reinterpret_cast<const int4 *>(cf + 768 + c8);
      const int4 i1 = *reinterpret_cast<const int4 *>(cf + 768 + c8 + 4);
      am[0] = i0.x; am[1] = i0.y; am[2] = i0.z; am[3] = i0.w;
      am[4] = i1.x; am[5] = i1.y; am[6] = i1.z; am[7] = i1.w;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = r0 + 16 * i;
      const int64_t r = rbase + rl;
      float y[8], v[8];
      unpack_chunk(ry[i], y);
      if constexpr (DYMODE == PCS_PRO_BWD) {
        unpack_chunk(rz[i], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(ca[e], v[e], fmaf(cg[e], y[e], cb[e]));
      } else if constexpr (DYMODE == PCS_PRO_BNRELU) {   // Gram: (beta, gamma) slots hold (s, t)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = relu(fmaf(y[e], cb[e], cg[e]));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = fmaf(cg[e], y[e], cb[e]);
          if (am[e] == (int)r) x += ca[e];
          v[e] = x;
        }
      }
      u32x4 o = pack_chunk(v);
      if (r >= rlast) o = mk_u32x4(0, 0, 0, 0);
      *reinterpret_cast<u32x4 *>(tA + prow(rl) * ROWB + cc * 16) = o;
    }
  }
  float xs[8], xt[8];
  lds8(cf + 1024 + c8, xs);
  lds8(cf + 1280 + c8, xt);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = r0 + 16 * i;
    const bool ok = rbase + rl < rlast;
    float w[8];
    unpack_chunk(rx[i], w);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = relu(fmaf(w[e], xs[e], xt[e]));
      if constexpr (MASK) x *= ((mk[i] >> e) & 1u) ? a.x_keep_scale : 0.f;
      w[e] = x;
    }
    if constexpr (DYMODE == PCS_PRO_BNRELU) {
      if (diag && ok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += w[e];
      }
    }
    u32x4 ox = pack_chunk(w);
    if (!ok) ox = mk_u32x4(0, 0, 0, 0);
    *reinterpret_cast<u32x4 *>(tB + prow(rl) * ROWB + cc * 16) = ox;
  }
}

template <int DYMODE, bool MASK, bool RAWG = false>
__global__ __launch_bounds__(THREADS) void wgrad_big_kernel(pcs_wgrad_args a, int64_t rows_per_split,
                                                            int ntn, int ntiles) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float *cf = reinterpret_cast<float *>(lds + 2 * STAGE);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / ntiles, tile = L % ntiles;
  int nt = tile / ntn, kt = tile % ntn;
  if constexpr (DYMODE == PCS_PRO_BNRELU) {   // upper triangle: tile -> (nt <= kt)
    int t = tile;
    nt = 0;
    while (t >= ntn - nt) { t -= ntn - nt; ++nt; }
    kt = nt + t;
  }
  const int n0 = nt * TM, k0 = kt * TN;
  const bool diag = nt == kt;
  const int sps = a.splits_per_scene;
  const int scene = split / sps, sis = split % sps;
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int64_t rlast = scene * N + hi;           // global row bound of this slice
  const int Cout = a.Cout, Cin = a.Cin;
  const bf16_t *dZ = reinterpret_cast<const bf16_t *>(a.dZ);
  const bf16_t *Yg = reinterpret_cast<const bf16_t *>(a.Y);
  const bf16_t *Xg = reinterpret_cast<const bf16_t *>(a.X);
  const int cc = tid & 31, r0 = tid >> 5;   // staging: fixed 8-column chunk, rows r0 + 16 i
  const int an = n0 + cc * 8, bk = k0 + cc * 8;
  for (int c = tid; c < 256; c += THREADS) {
    if constexpr (DYMODE == PCS_PRO_BWD) {
      cf[c] = a.alpha[n0 + c];
    } else if constexpr (DYMODE == PCS_PRO_BWD_POOL) {
      cf[c] = a.pool_coef[(int64_t)scene * Cout + n0 + c];
      reinterpret_cast<int *>(cf)[768 + c] = a.pool_idx[(int64_t)scene * Cout + n0 + c];
    }
    if constexpr (RAWG) continue;
    if constexpr (DYMODE == PCS_PRO_BNRELU) {
      cf[256 + c] = a.s[n0 + c];
      cf[512 + c] = a.t[n0 + c];
    } else {
      cf[256 + c] = a.beta[n0 + c];
      cf[512 + c] = a.gamma[n0 + c];
    }
    cf[1024 + c] = a.s[k0 + c];
    cf[1280 + c] = a.t[k0 + c];
  }
  __syncthreads();

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (int)((hi - lo + MS - 1) / MS);
  u32x4 rz[4], ry[4], rx[4];
  uint32_t mk[4] = {0xffu, 0xffu, 0xffu, 0xffu};
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (nsteps > 0) {
    const int64_t rb = scene * N + lo;
    tn_load<DYMODE, MASK>(dZ, Yg, Xg, a.x_mask, rb, rlast, Cout, Cin, an, bk, r0, rz, ry, rx, mk);
    tn_store<DYMODE, MASK, RAWG>(a, lds, cf, rb, rlast, bk, cc, r0, rz, ry, rx, mk, diag, csum);
    __syncthreads();
  }
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const int64_t rb = scene * N + lo + (int64_t)st * MS;
    if (st + 1 < nsteps)
      tn_load<DYMODE, MASK>(dZ, Yg, Xg, a.x_mask, rb + MS, rlast, Cout, Cin, an, bk, r0, rz, ry, rx, mk);
    const char *tA = lds + buf * STAGE;
    const char *tB = tA + OPB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ra = prow(32 * kk + 8 * g + q), rb1 = prow(32 * kk + 8 * g + 4 + q);
      bf16x8 xf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xf[j] = tr_frag(tB, ra, rb1, wn * 64 + j * 16 + 4 * p);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 yf = tr_frag(tA, ra, rb1, wm * 128 + i * 16 + 4 * p);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[j], yf, acc[i][j], 0, 0, 0);
      }
    }
    if (st + 1 < nsteps)
      tn_store<DYMODE, MASK, RAWG>(a, lds + (buf ^ 1) * STAGE, cf, rb + MS, rlast, bk, cc, r0, rz, ry, rx, mk,
                                   diag, csum);
    lds_barrier();
  }
  // lane holds dW[n = n0 + wm*128 + i*16 + (lane&15)][k = k0 + wn*64 + j*16 + 4*(lane>>4) + r]
  float *out = a.partial + (int64_t)split * Cout * Cin;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = n0 + wm * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      *reinterpret_cast<float4 *>(out + (int64_t)n * Cin + k) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
  if constexpr (DYMODE == PCS_PRO_BNRELU) {   // column sums of a over this slice (diagonal tiles)
    if (diag) {
      __syncthreads();
      float *red = reinterpret_cast<float *>(lds);   // [16 row groups][256 columns]
#pragma unroll
      for (int e = 0; e < 8; ++e) red[r0 * 256 + cc * 8 + e] = csum[e];
      __syncthreads();
      if (tid < 256) {
        float v = 0.f;
        for (int j = 0; j < THREADS / 32; ++j) v += red[j * 256 + tid];
        const int nsplit = gridDim.x / ntiles;
        a.partial[(int64_t)nsplit * Cout * Cin + (int64_t)split * Cin + k0 + tid] = v;
      }
    }
  }
}

}  // namespace

bool pcs_wgrad_big_applicable(const pcs_wgrad_args &a) {
  if (a.dy_mode == PCS_PRO_BNRELU && (a.Cout != a.Cin || a.x_mask)) return false;   // Gram: square
  return !(a.flags & PCS_FLAG_GENERIC) && a.dtype == PCS_BF16 && a.Cout % TM == 0 && a.Cin % TN == 0 &&
         a.x_mode == PCS_PRO_BNRELU &&
         (a.dy_mode == PCS_PRO_BWD || a.dy_mode == PCS_PRO_BWD_POOL || a.dy_mode == PCS_PRO_BNRELU);
}

int pcs_wgrad_big_tiles(const pcs_wgrad_args &a) {
  const int ntm = a.Cout / TM, ntn = a.Cin / TN;
  return a.dy_mode == PCS_PRO_BNRELU ? ntm * (ntm + 1) / 2 : ntm * ntn;
}

int pcs_wgrad_big_splits(const pcs_wgrad_args &a) {
  // one 512-thread workgroup per CU: pick the row splits per scene that minimise
  // (waves of 256 workgroups) / splits, i.e. the time of the slowest CU, with the fp32
  // partial slabs kept below 256 MB
  const int64_t per_split = a.num_scenes * pcs_wgrad_big_tiles(a);
  const int64_t slab = (int64_t)a.Cout * a.Cin * 4;
  const int64_t max_sps = pcs_max64(1, pcs_min64((a.scene_rows + 8 * MS - 1) / (8 * MS),
                                                 ((int64_t)256 << 20) / slab / a.num_scenes));
  int64_t best = 1;
  double best_cost = 1e30;
  for (int64_t sps = 1; sps <= max_sps; ++sps) {
    const double waves = (double)((per_split * sps + 255) / 256);
    const double cost = waves / (double)sps * (1.0 + 1e-3 * sps);   // tie-break: fewer slabs
    if (cost < best_cost) { best_cost = cost; best = sps; }
  }
  return (int)best;
}

int pcs_wgrad_big_launch(const pcs_wgrad_args &a, hipStream_t s) {
  int64_t rps = (a.scene_rows + a.splits_per_scene - 1) / a.splits_per_scene;
  rps = (rps + MS - 1) / MS * MS;
  const int ntn = a.Cin / TN, ntiles = pcs_wgrad_big_tiles(a);
  const int nb = ntiles * (int)(a.num_scenes * a.splits_per_scene);
  if (a.dy_mode == PCS_PRO_BNRELU) {
    if (!a.s)   // Gram of stored activations (pcs_gram with s = t = NULL)
      hipLaunchKernelGGL((wgrad_big_kernel<PCS_PRO_BNRELU, false, true>), dim3(nb), dim3(THREADS), 0, s, a, rps, ntn,
                         ntiles);
    else
      hipLaunchKernelGGL((wgrad_big_kernel<PCS_PRO_BNRELU, false>), dim3(nb), dim3(THREADS), 0, s, a, rps, ntn, ntiles);
  } else if (a.dy_mode == PCS_PRO_BWD_POOL) {
    if (a.x_mask) hipLaunchKernelGGL((wgrad_big_kernel<PCS_PRO_BWD_POOL, true>), dim3(nb), dim3(THREADS), 0, s, a, rps, ntn, ntiles);
    else hipLaunchKernelGGL((wgrad_big_kernel<PCS_PRO_BWD_POOL, false>), dim3(nb), dim3(THREADS), 0, s, a, rps, ntn, ntiles);
  } else {
    if (a.x_mask) hipLaunchKernelGGL((wgrad_big_kernel<PCS_PRO_BWD, true>), dim3(nb), dim3(THREADS), 0, s, a, rps, ntn, ntiles);
    else hipLaunchKernelGGL((wgrad_big_kernel<PCS_PRO_BWD, false>), dim3(nb), dim3(THREADS), 0, s, a, rps, ntn, ntiles);
  }
  PCS_CHECK_LAUNCH();
  return 0;
}

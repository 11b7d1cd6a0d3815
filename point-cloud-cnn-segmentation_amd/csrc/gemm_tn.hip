// Weight gradient of the 1x1 Conv1d chain (autograd of P:106-128 at P:254):
//
//   dW[n, k] = sum_m dy[m, n] * x[m, k]
//
// dy is formed on the fly from the stored BN-input Y_l and the ReLU-masked gradient dZ_l
// (dy = alpha*dz + beta + gamma*y, or the max-pool sparse form for bn_global) and x from
// the previous layer's stored Y_{l-1} (relu(bn(y)) * dropout keep bits), so neither dy
// nor x is ever materialised.  The M reduction is split into scene-aligned row slices,
// each workgroup writes an fp32 partial tile, and pcs_reduce_partials sums the slices in
// a fixed order (deterministic).
//
// LDS tiles are [m][col] images read with ds_read_b64_tr_b16 (bf16: the hardware
// transpose delivers 4 consecutive m of one column per lane) or ds_read_b32 (fp32 MFMA
// 16x16x4).  bf16 rows are permuted (bits 2<->3 of m swapped) and padded by 32 B so the
// eight rows one transposed read touches land on eight distinct bank groups.
#include "common.h"

namespace {

constexpr int THREADS = 256;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T> struct TnCfg;
template <> struct TnCfg<bf16_t> {
  static constexpr int MS = 64;    // rows (reduction) per step: 2 MFMA k-iterations
  static constexpr int PADB = 32;  // row padding in bytes
  static PCS_DEV int prow(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }
};
template <> struct TnCfg<float> {
  static constexpr int MS = 16;
  static constexpr int PADB = 64;
  static PCS_DEV int prow(int r) { return r; }
};

template <typename T, int COLS, int MODE>
struct Operand {
  // staging of one [MS x COLS] operand tile; a thread owns a fixed column chunk
  static constexpr int EPC = Elem<T>::EPC;
  static constexpr int MS = TnCfg<T>::MS;
  static constexpr int CPR = COLS / EPC;
  static constexpr int RP = THREADS / CPR;
  static constexpr int NCH = MS / RP;
  static constexpr int ROWB = COLS * Elem<T>::SIZE + TnCfg<T>::PADB;
  static constexpr int BYTES = MS * ROWB;
};

template <typename T, int TM, int TN, int DYMODE, int XMODE, bool MASK>
__global__ __launch_bounds__(THREADS, 2) void wgrad_kernel(pcs_wgrad_args a, int64_t rows_per_split,
                                                           int ntn, int ntiles) {
  constexpr int EPC = Elem<T>::EPC;
  constexpr int MS = TnCfg<T>::MS;
  typedef Operand<T, TM, DYMODE> OA;  // dy tile [MS][TM]
  typedef Operand<T, TN, XMODE> OB;   // x tile  [MS][TN]
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int FM = TM / 2 / 16, FN = TN / 2 / 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / ntiles, tile = L % ntiles;
  const int n0 = (tile / ntn) * TM, k0 = (tile % ntn) * TN;
  const int sps = a.splits_per_scene;
  const int scene = split / sps, sis = split % sps;
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int Cout = a.Cout, Cin = a.Cin;

  const T *__restrict__ dZ = reinterpret_cast<const T *>(a.dZ);
  const T *__restrict__ Yg = reinterpret_cast<const T *>(a.Y);
  const T *__restrict__ Xg = reinterpret_cast<const T *>(a.X);

  // fixed per-thread columns and coefficients
  const int acc_c = tid % OA::CPR, ar0 = tid / OA::CPR;
  const int bcc = tid % OB::CPR, br0 = tid / OB::CPR;
  const int an = n0 + acc_c * EPC, bk = k0 + bcc * EPC;
  float ca[EPC], cb[EPC], cg[EPC], xs[EPC], xt[EPC];
  int am[EPC];
  if constexpr (DYMODE == PCS_PRO_BWD) {
    load_vec<EPC>(a.alpha, an, ca);
  } else if constexpr (DYMODE == PCS_PRO_BWD_POOL) {
    load_vec<EPC>(a.pool_coef + scene * Cout, an, ca);
#pragma unroll
    for (int e = 0; e < EPC; ++e) am[e] = a.pool_idx[scene * Cout + an + e];
  }
  if constexpr (DYMODE == PCS_PRO_BNRELU) {   // Gram: dy = relu(y*s + t) of the same activations
    load_vec<EPC>(a.s, an, cb);
    load_vec<EPC>(a.t, an, cg);
  } else if constexpr (DYMODE != PCS_PRO_RAW) {
    load_vec<EPC>(a.beta, an, cb);
    load_vec<EPC>(a.gamma, an, cg);
  }
  const bool diag = DYMODE == PCS_PRO_BNRELU && n0 == k0 && TM == TN;
  float csum[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) csum[e] = 0.f;
  if constexpr (XMODE == PCS_PRO_BNRELU) {
    load_vec<EPC>(a.s, bk, xs);
    load_vec<EPC>(a.t, bk, xt);
  }

  // Rows past the slice end are loaded clamped (no branches) and written to LDS as zeros.
  u32x4 rz[OA::NCH], ry[OA::NCH], rx[OB::NCH];
  uint32_t mk[OB::NCH];
  auto load_stage = [&](int64_t m0) {
#pragma unroll
    for (int i = 0; i < OA::NCH; ++i) {
      const int64_t r = pcs_min64(m0 + ar0 + OA::RP * i, hi - 1);
      const int64_t off = (scene * N + r) * Cout + an;
      if constexpr (DYMODE == PCS_PRO_BWD || DYMODE == PCS_PRO_RAW) rz[i] = *reinterpret_cast<const u32x4 *>(dZ + off);
      if constexpr (DYMODE != PCS_PRO_RAW) ry[i] = *reinterpret_cast<const u32x4 *>(Yg + off);
    }
#pragma unroll
    for (int i = 0; i < OB::NCH; ++i) {
      const int64_t r = pcs_min64(m0 + br0 + OB::RP * i, hi - 1);
      const int64_t off = (scene * N + r) * Cin + bk;
      rx[i] = *reinterpret_cast<const u32x4 *>(Xg + off);
      if constexpr (MASK) {
        const uint32_t byte = a.x_mask[off >> 3];
        mk[i] = EPC == 8 ? byte : (byte >> (bk & 7)) & 0xFu;
      }
    }
  };
  auto store_stage = [&](int64_t m0, int buf) {
    char *tA = lds + buf * STAGE;
    char *tB = tA + OA::BYTES;
#pragma unroll
    for (int i = 0; i < OA::NCH; ++i) {
      const int rl = ar0 + OA::RP * i;
      const int64_t r = m0 + rl;
      float y[EPC], v[EPC];
      if constexpr (DYMODE != PCS_PRO_RAW) unpack_chunk(ry[i], y);
      if constexpr (DYMODE == PCS_PRO_RAW) {   // dy = dZ as stored (scaled later, pcs_gram_wgrad)
        unpack_chunk(rz[i], v);
      } else if constexpr (DYMODE == PCS_PRO_BWD) {
        unpack_chunk(rz[i], v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = fmaf(ca[e], v[e], fmaf(cg[e], y[e], cb[e]));
      } else if constexpr (DYMODE == PCS_PRO_BNRELU) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = relu(fmaf(y[e], cb[e], cg[e]));
      } else {
        const int grow = (int)(scene * N + r);
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = fmaf(cg[e], y[e], cb[e]) + (am[e] == grow ? ca[e] : 0.f);
      }
      u32x4 out = pack_chunk(v);
      if (r >= hi) out = mk_u32x4(0, 0, 0, 0);
      *reinterpret_cast<u32x4 *>(tA + TnCfg<T>::prow(rl) * OA::ROWB + acc_c * 16) = out;
    }
#pragma unroll
    for (int i = 0; i < OB::NCH; ++i) {
      const int rl = br0 + OB::RP * i;
      const int64_t r = m0 + rl;
      u32x4 out = rx[i];
      if constexpr (XMODE == PCS_PRO_BNRELU) {
        float v[EPC];
        unpack_chunk(rx[i], v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          float x = relu(fmaf(v[e], xs[e], xt[e]));
          if constexpr (MASK) x *= ((mk[i] >> e) & 1u) ? a.x_keep_scale : 0.f;
          v[e] = x;
        }
        if (diag && r < hi) {
#pragma unroll
          for (int e = 0; e < EPC; ++e) csum[e] += v[e];
        }
        out = pack_chunk(v);
      }
      if (r >= hi) out = mk_u32x4(0, 0, 0, 0);
      *reinterpret_cast<u32x4 *>(tB + TnCfg<T>::prow(rl) * OB::ROWB + bcc * 16) = out;
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Pipeline: compute(st) -> write registers (step st+1) to the other LDS buffer -> issue
  // the loads of step st+2 -> barrier; each load has a full step of MFMAs to land.
  const int nsteps = (int)((hi - lo + MS - 1) / MS);
  if (nsteps > 0) {
    load_stage(lo);
    store_stage(lo, 0);
    __builtin_amdgcn_sched_barrier(0);
    load_stage(lo + MS);   // clamped: harmless when nsteps == 1
    __syncthreads();
  }
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const int64_t m0 = lo + (int64_t)st * MS;
    const char *tA = lds + buf * STAGE;
    const char *tB = tA + OA::BYTES;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < MS / 32; ++kk) {
        // lane group g = lane>>4 holds k = 8g..8g+7 of the MFMA reduction (= m rows)
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int r0 = TnCfg<T>::prow(32 * kk + 8 * g + q), r1 = TnCfg<T>::prow(32 * kk + 8 * g + 4 + q);
        bf16x8 xf[FN], yf[FM];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c = wn * (TN / 2) + j * 16 + 4 * p;
          s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tB + r0 * OB::ROWB + c * 2));
          s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tB + r1 * OB::ROWB + c * 2));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          s16x8 v = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
          xf[j] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int c = wm * (TM / 2) + i * 16 + 4 * p;
          s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tA + r0 * OA::ROWB + c * 2));
          s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tA + r1 * OA::ROWB + c * 2));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          s16x8 v = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
          yf[i] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[j], yf[i], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < MS / 4; ++kk) {
        const int r = kk * 4 + (lane >> 4);
        float xf[FN], yf[FM];
#pragma unroll
        for (int j = 0; j < FN; ++j)
          xf[j] = *reinterpret_cast<const float *>(tB + r * OB::ROWB + (wn * (TN / 2) + j * 16 + (lane & 15)) * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
          yf[i] = *reinterpret_cast<const float *>(tA + r * OA::ROWB + (wm * (TM / 2) + i * 16 + (lane & 15)) * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(xf[j], yf[i], acc[i][j], 0, 0, 0);
      }
    }
    if (st + 1 < nsteps) {
      store_stage(m0 + MS, buf ^ 1);
      __builtin_amdgcn_sched_barrier(0);
      load_stage(m0 + 2 * MS);   // clamped past the end: never consumed
    }
    lds_barrier();
  }

  // partial tile: lane holds dW[n][k..k+3]
  float *out = a.partial + (int64_t)split * Cout * Cin;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int n = n0 + wm * (TM / 2) + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int k = k0 + wn * (TN / 2) + j * 16 + 4 * (lane >> 4);
      *reinterpret_cast<float4 *>(out + (int64_t)n * Cin + k) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
  if (diag) {   // Gram: column sums of the x operand over this slice
    __syncthreads();
    float *red = reinterpret_cast<float *>(lds);   // [RP row groups][TN columns]
#pragma unroll
    for (int e = 0; e < EPC; ++e) red[br0 * TN + bcc * EPC + e] = csum[e];
    __syncthreads();
    for (int c = tid; c < TN; c += THREADS) {
      float v = 0.f;
      for (int j = 0; j < OB::RP; ++j) v += red[j * TN + c];
      const int nsplit = gridDim.x / ntiles;
      a.partial[(int64_t)nsplit * Cout * Cin + (int64_t)split * Cin + k0 + c] = v;
    }
  }
}

template <typename T, int TM, int TN, int DY, int XM>
int launch(const pcs_wgrad_args &a, int64_t rps, hipStream_t s) {
  const int ntn = a.Cin / TN, ntiles = (a.Cout / TM) * ntn;
  const int nb = ntiles * (int)(a.num_scenes * a.splits_per_scene);
  if (XM == PCS_PRO_BNRELU && a.x_mask)
    hipLaunchKernelGGL((wgrad_kernel<T, TM, TN, DY, XM, XM == PCS_PRO_BNRELU>), dim3(nb), dim3(THREADS), 0, s,
                       a, rps, ntn, ntiles);
  else
    hipLaunchKernelGGL((wgrad_kernel<T, TM, TN, DY, XM, false>), dim3(nb), dim3(THREADS), 0, s, a, rps, ntn, ntiles);
  PCS_CHECK_LAUNCH();
  return 0;
}

template <typename T, int TM, int TN>
int dispatch_modes(const pcs_wgrad_args &a, int64_t rps, hipStream_t s) {
  if (a.dy_mode == PCS_PRO_BWD) {
    if (a.x_mode == PCS_PRO_BNRELU) return launch<T, TM, TN, PCS_PRO_BWD, PCS_PRO_BNRELU>(a, rps, s);
    if (a.x_mode == PCS_PRO_RAW) return launch<T, TM, TN, PCS_PRO_BWD, PCS_PRO_RAW>(a, rps, s);
  } else if (a.dy_mode == PCS_PRO_BWD_POOL) {
    if (a.x_mode == PCS_PRO_BNRELU) return launch<T, TM, TN, PCS_PRO_BWD_POOL, PCS_PRO_BNRELU>(a, rps, s);
  } else if (a.dy_mode == PCS_PRO_RAW) {
    if (a.x_mode == PCS_PRO_BNRELU) return launch<T, TM, TN, PCS_PRO_RAW, PCS_PRO_BNRELU>(a, rps, s);
  } else if (a.dy_mode == PCS_PRO_BNRELU && a.x_mode == PCS_PRO_BNRELU && !a.x_mask) {
    return launch<T, TM, TN, PCS_PRO_BNRELU, PCS_PRO_BNRELU>(a, rps, s);
  }
  return pcs_set_einval("pcs_wgrad", "unsupported dy_mode/x_mode");
}

template <typename T>
int dispatch_tiles(const pcs_wgrad_args &a, int64_t rps, hipStream_t s) {
  const bool m128 = a.Cout % 128 == 0, n128 = a.Cin % 128 == 0;
  if (m128 && n128) return dispatch_modes<T, 128, 128>(a, rps, s);
  if (m128) return dispatch_modes<T, 128, 64>(a, rps, s);
  if (n128) return dispatch_modes<T, 64, 128>(a, rps, s);
  return dispatch_modes<T, 64, 64>(a, rps, s);
}

int64_t rows_per_split_of(const pcs_wgrad_args &a, int ms) {
  const int64_t rps = (a.scene_rows + a.splits_per_scene - 1) / a.splits_per_scene;
  return (rps + ms - 1) / ms * ms;
}

}  // namespace

extern "C" int64_t pcs_wgrad_workspace(pcs_wgrad_args *a) {
  if (!a || a->num_scenes <= 0 || a->scene_rows <= 0 || a->Cout <= 0 || a->Cin <= 0)
    return pcs_set_einval("pcs_wgrad_workspace", "bad geometry");
  const int ms = a->dtype == PCS_BF16 ? TnCfg<bf16_t>::MS : TnCfg<float>::MS;
  if (a->splits_per_scene <= 0 && pcs_wgrad_c5_class(*a)) a->splits_per_scene = pcs_wgrad_c5_splits(*a);
  if (a->splits_per_scene <= 0 && pcs_wgrad_big_applicable(*a)) a->splits_per_scene = pcs_wgrad_big_splits(*a);
  if (a->splits_per_scene <= 0) {
    const int tm = a->Cout % 128 == 0 ? 128 : 64, tn = a->Cin % 128 == 0 ? 128 : 64;
    const int64_t ntiles = a->Cin >= 64 ? (int64_t)(a->Cout / tm) * (a->Cin / tn) : 1;
    const int64_t target = 1024;
    int64_t sps = (target + a->num_scenes * ntiles - 1) / (a->num_scenes * ntiles);
    const int64_t max_sps = (a->scene_rows + 4 * ms - 1) / (4 * ms);  // >= 4 steps per split
    if (sps > max_sps) sps = max_sps;
    if (sps < 1) sps = 1;
    a->splits_per_scene = (int32_t)sps;
  }
  const int64_t nslabs = (int64_t)a->num_scenes * a->splits_per_scene;
  return nslabs * a->Cout * a->Cin * 4 + (a->dy_colsum ? nslabs * a->Cout * 4 : 0);
}

extern "C" int pcs_wgrad(const pcs_wgrad_args *ap, pcs_stream_t stream) {
  if (!ap) return pcs_set_einval("pcs_wgrad", "null args");
  pcs_wgrad_args a = *ap;
  if (a.Cout % 64 || a.Cin % 64) return pcs_set_einval("pcs_wgrad", "Cout/Cin must be multiples of 64");
  if (!a.X || !a.partial || !a.dW) return pcs_set_einval("pcs_wgrad", "missing operand");
  if (a.dy_mode == PCS_PRO_RAW ? !a.dZ : (!a.Y || !a.beta || !a.gamma))
    return pcs_set_einval("pcs_wgrad", "dy operands missing (RAW: dZ; BWD/BWD_POOL: Y, beta, gamma)");
  if (a.dy_mode == PCS_PRO_BWD && (!a.dZ || !a.alpha)) return pcs_set_einval("pcs_wgrad", "PRO_BWD needs dZ, alpha");
  if (a.dy_mode == PCS_PRO_BWD_POOL && (!a.pool_idx || !a.pool_coef))
    return pcs_set_einval("pcs_wgrad", "PRO_BWD_POOL needs pool_idx, pool_coef");
  if (a.x_mode == PCS_PRO_BNRELU && (!a.s || !a.t)) return pcs_set_einval("pcs_wgrad", "x BNRELU needs s, t");
  if (a.dy_colsum && !pcs_wgrad_c5_applicable(a))
    return pcs_set_einval("pcs_wgrad", "dy_colsum: conv5's R pass only (bf16, RAW dZ, BNRELU x, Cin 128)");
  if (pcs_wgrad_workspace(&a) < 0) return PCS_EINVAL;
  const int ms = a.dtype == PCS_BF16 ? TnCfg<bf16_t>::MS : TnCfg<float>::MS;
  const int64_t rps = rows_per_split_of(a, ms);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc;
  if (pcs_wgrad_c5_applicable(a)) rc = pcs_wgrad_c5_launch(a, rps, s);
  else if (pcs_wgrad_big_applicable(a)) rc = pcs_wgrad_big_launch(a, s);
  else if (a.dtype == PCS_BF16) rc = dispatch_tiles<bf16_t>(a, rps, s);
  else if (a.dtype == PCS_F32) rc = dispatch_tiles<float>(a, rps, s);
  else return pcs_set_einval("pcs_wgrad", "bad dtype");
  if (rc) return rc;
  const int64_t nslabs = a.num_scenes * a.splits_per_scene;
  if (a.dy_colsum) {
    rc = pcs_reduce_partials(a.partial + nslabs * a.Cout * a.Cin, nslabs, a.Cout, 1.0f, a.dy_colsum, a.Cout, a.Cout,
                             stream);
    if (rc) return rc;
  }
  return pcs_reduce_partials(a.partial, nslabs, (int64_t)a.Cout * a.Cin, 1.0f, a.dW,
                             a.ldw ? a.ldw : a.Cin, a.Cin, stream);
}

// ---------------------------------------------------------------------------------------
// Gram of the BN+ReLU activations (global_feat weight gradient, see gram.hip)
// ---------------------------------------------------------------------------------------
namespace {

pcs_wgrad_args gram_args(const void *Y, const float *s, const float *t, int64_t num_scenes,
                         int64_t scene_rows, int32_t C, int32_t dtype, int32_t sps) {
  pcs_wgrad_args a = {};
  a.num_scenes = num_scenes; a.scene_rows = scene_rows; a.Cout = C; a.Cin = C; a.dtype = dtype;
  a.splits_per_scene = sps; a.dy_mode = PCS_PRO_BNRELU; a.x_mode = PCS_PRO_BNRELU;
  a.Y = Y; a.X = Y; a.s = s; a.t = t; a.x_keep_scale = 1.f;
  return a;
}

// Mirror the upper 64x64 tiles of the summed Gram into the lower ones (the 256x256 kernel
// computes only upper tiles; a transposed copy through LDS keeps both sides coalesced).
__global__ __launch_bounds__(256) void gram_mirror_kernel(float *__restrict__ G, int C) {
  __shared__ float tile[64][65];
  const int nt = C / 64;
  int t = blockIdx.x, tj = 0;
  while (t >= nt - 1 - tj) { t -= nt - 1 - tj; ++tj; }   // strictly upper pairs (tj < tk)
  const int tk = tj + 1 + t;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) tile[r][tx] = G[(int64_t)(tj * 64 + r) * C + tk * 64 + tx];
  __syncthreads();
  for (int r = ty; r < 64; r += 4) G[(int64_t)(tk * 64 + r) * C + tj * 64 + tx] = tile[tx][r];
}

}  // namespace

extern "C" int64_t pcs_gram_workspace(int64_t num_scenes, int64_t scene_rows, int32_t C, int32_t dtype,
                                      int32_t *splits_per_scene) {
  if (num_scenes <= 0 || scene_rows <= 0 || C <= 0 || C % 64 || !splits_per_scene)
    return pcs_set_einval("pcs_gram_workspace", "bad geometry");
  pcs_wgrad_args a = gram_args(nullptr, nullptr, nullptr, num_scenes, scene_rows, C, dtype, 0);
  if (pcs_gram128_class(a)) a.splits_per_scene = pcs_gram128_splits(a);
  const int64_t g = pcs_wgrad_workspace(&a);
  if (g < 0) return g;
  *splits_per_scene = a.splits_per_scene;
  return g + num_scenes * a.splits_per_scene * (int64_t)C * 4;
}

extern "C" int pcs_gram(const void *Y, const float *s, const float *t, int64_t num_scenes, int64_t scene_rows,
                        int32_t C, int32_t dtype, int32_t splits_per_scene, float *workspace, float *G,
                        float *colsum, pcs_stream_t stream) {
  if (!Y || !s != !t || !workspace || !G || !colsum || splits_per_scene <= 0)
    return pcs_set_einval("pcs_gram", "missing operand or splits (s and t both set, or both NULL)");
  if (C % 64) return pcs_set_einval("pcs_gram", "C must be a multiple of 64");
  pcs_wgrad_args a = gram_args(Y, s, t, num_scenes, scene_rows, C, dtype, splits_per_scene);
  a.partial = workspace;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc;
  if (!s && !pcs_wgrad_big_applicable(a))   // s = t = NULL: Y is already the activation
    return pcs_set_einval("pcs_gram", "s = t = NULL needs the 256x256 kernel (bf16, C % 256 == 0)");
  if (pcs_gram128_applicable(a)) {
    rc = pcs_gram128_launch(a, st);
  } else if (pcs_wgrad_big_applicable(a)) {
    rc = pcs_wgrad_big_launch(a, st);
  } else {
    const int ms = dtype == PCS_BF16 ? TnCfg<bf16_t>::MS : TnCfg<float>::MS;
    const int64_t rps = rows_per_split_of(a, ms);
    if (dtype == PCS_BF16) rc = dispatch_tiles<bf16_t>(a, rps, st);
    else if (dtype == PCS_F32) rc = dispatch_tiles<float>(a, rps, st);
    else return pcs_set_einval("pcs_gram", "bad dtype");
  }
  if (rc) return rc;
  const int nsplit = (int)(num_scenes * splits_per_scene);
  const int64_t n = (int64_t)C * C;
  if ((rc = pcs_reduce_partials(workspace, nsplit, n, 1.f, G, C, C, stream))) return rc;
  if ((rc = pcs_reduce_partials(workspace + nsplit * n, nsplit, C, 1.f, colsum, C, C, stream))) return rc;
  const int nt = C / 64;
  if (nt > 1) {
    hipLaunchKernelGGL(gram_mirror_kernel, dim3(nt * (nt - 1) / 2), dim3(256), 0, st, G, C);
    PCS_CHECK_LAUNCH();
  }
  return 0;
}

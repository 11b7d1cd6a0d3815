// Fused input + weight gradient of seg_conv1's local half (autograd of P:117-123 at P:254):
//
//   dy      = alpha * dZ + beta + gamma * Y          (bn_seg1 backward, [M, 512])
//   dA2     = dy . W_l                               ([M, 64], W_l = seg_conv1.weight[:, :64])
//   dW_l   += dy^T . relu(bn2(Y2))                   ([512, 64])
//
// Both gradients read the same dy, which is formed from the two widest tensors of the head
// (dZ and Y of bn_seg1, 2 KB per point in bf16).  Separately (pcs_gemm + pcs_wgrad) they
// read them twice; here each row slab is staged into LDS once and feeds both contractions,
// so the pair moves 2.3 KB per point instead of 4.5 KB.  MFMA work is small (14 % of the
// CU's MFMA time at the HBM rate), so the kernel is HBM-bound by design.
//
// One 512-thread workgroup per CU (W_l^T stays resident in LDS for the workgroup's life),
// scene-aligned row slices as pcs_wgrad, 64-row steps:
//   compute(step s) from LDS -> dA2 tile of step s to LDS -> barrier -> store it, write the
//   registers (step s+1) into LDS, issue the loads of step s+2 -> barrier.
// dgrad: wave w owns rows 16*(w>>1).. and columns 32*(w&1).. (2 accumulators, K = 512);
// wgrad: wave w owns output channels 64*w.. x all 64 inputs (16 accumulators, K = 64 rows).
// The dy tile is a [m][col] image (rows permuted as pcs_wgrad's bf16 tiles, 32-B padding)
// read with ds_read_b128 for the dgrad operand and ds_read_b64_tr_b16 for the wgrad one.
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int COUT = 512, CIN = 64, MS = 64;
constexpr int WT_ROWB = COUT * 2;                  // W_l^T [CIN][COUT], XOR-swizzled 16-B slots
constexpr int DY_ROWB = COUT * 2 + 32;             // dy [MS][COUT] (+32 B pad)
constexpr int X_ROWB = CIN * 2 + 32;               // x  [MS][CIN]
constexpr int OFF_DY = CIN * WT_ROWB;              // 64 KB
constexpr int OFF_X = OFF_DY + MS * DY_ROWB;
constexpr int OFF_OUT = OFF_X + MS * X_ROWB;       // dA2 tile [MS][CIN] bf16, rows OUT_ROWB apart
// (+8 B: the epilogue's 8-B writes of 16 rows at one column hit 16 different banks -- 128-B rows
// put them on two, 16-way (SQ_LDS_BANK_CONFLICT 0.38 of the LDS cycles, r06))
constexpr int OUT_ROWB = CIN * 2 + 8;
constexpr int OFF_COEF = OFF_OUT + MS * OUT_ROWB;  // alpha | beta | gamma [COUT], s | t [CIN]
constexpr int LDS_BYTES = OFF_COEF + (3 * COUT + 2 * CIN) * 4;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
// folded form: s | t | cvec [CIN] f32, then H [CIN][CIN] bf16 (XOR-swizzled 16-B slots)
constexpr int OFF_H = OFF_COEF + 3 * CIN * 4;
constexpr int H_ROWB = CIN * 2;
constexpr int LDS_BYTES_F = OFF_H + CIN * H_ROWB;
static_assert(LDS_BYTES_F <= 160 * 1024, "LDS budget (folded)");
// folded form's per-slice partial slab: R = dz^T x [COUT][CIN] | G = x^T x [CIN][CIN] | S = sum x [CIN]
constexpr int SLAB_F = COUT * CIN + CIN * CIN + CIN;
constexpr int DY_CPR = COUT / 8, DY_RP = THREADS / DY_CPR, DY_NCH = MS / DY_RP;   // 64, 8, 8
constexpr int X_CPR = CIN / 8, X_RP = THREADS / X_CPR;                            // 8, 64
static_assert(X_RP == MS, "one x chunk per thread");

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PCS_DEV int prow(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }
// (slot ^ (c & 15): the dgrad's 16-B fragment reads of 16 rows c at slots 4 kk + g fall in 16
// different slots of a 64-slot row; with c & 7 the two lane groups g met in the same 8, 2-way)
PCS_DEV int wt_off(int c, int slot) { return c * WT_ROWB + ((slot ^ (c & 15)) << 4); }

PCS_DEV void lds_vec8(const float *p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4 *>(p);
  const float4 b = *reinterpret_cast<const float4 *>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

PCS_DEV bf16x8 tr_read(const char *base, int r0, int r1, int rowb, int col) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(base + r0 * rowb + col * 2));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(base + r1 * rowb + col * 2));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// FOLDED (dy_mode RAW): dy is dZ itself and Wt = (diag(alpha) W_l)^T, so the same contractions
// give P = dZ (diag(alpha) W_l) and R = dZ^T x; the input gradient adds x H + cvec[scene] (H =
// W_l^T diag(gamma) W_l, cvec = W_l^T (beta + gamma * scene_bias[b]), pcs_bn_fold algebra:
// gamma * Y' W_l = x H + scene-bias terms, as Y' = x W_l^T + scene_bias[b]), and the slab also
// collects G = x^T x and S = sum x for the Gram-form weight gradient (pcs_dgrad_wgrad_folded)
// -- bn_seg1's stored Y' [M, 512] is not read at all.
template <bool FOLDED>
__global__ __launch_bounds__(THREADS) void dgrad_wgrad_s1_kernel(pcs_wgrad_args a, const bf16_t *__restrict__ Wt,
                                                                 bf16_t *__restrict__ dX, int64_t rows_per_split,
                                                                 const bf16_t *__restrict__ Hg,
                                                                 const float *__restrict__ cvec) {
  __shared__ __attribute__((aligned(16))) char lds[FOLDED ? LDS_BYTES_F : LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int sps = a.splits_per_scene;
  const int scene = L / sps, sis = L % sps;
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int64_t sbase = (int64_t)scene * N;

  const bf16_t *__restrict__ dZ = reinterpret_cast<const bf16_t *>(a.dZ);
  const bf16_t *__restrict__ Yg = reinterpret_cast<const bf16_t *>(a.Y);
  const bf16_t *__restrict__ Xg = reinterpret_cast<const bf16_t *>(a.X);

  // W_l^T [CIN][COUT] -> LDS once (64 KB: 8 chunks per thread)
  for (int i = tid; i < CIN * COUT / 8; i += THREADS) {
    const int c = i / (COUT / 8), slot = i % (COUT / 8);
    *reinterpret_cast<u32x4 *>(lds + wt_off(c, slot)) =
        *reinterpret_cast<const u32x4 *>(Wt + (int64_t)c * COUT + slot * 8);
  }

  // per-channel prologue coefficients -> LDS (read back at each store: fewer live registers)
  float *cf = reinterpret_cast<float *>(lds + OFF_COEF);
  constexpr int CS = FOLDED ? 0 : 3 * COUT;   // x's bn2 scale | shift
  if constexpr (FOLDED) {
    if (tid < CIN) { cf[tid] = a.s[tid]; cf[CIN + tid] = a.t[tid]; cf[2 * CIN + tid] = cvec[scene * CIN + tid]; }
    for (int i = tid; i < CIN * CIN / 8; i += THREADS) {   // H rows [c][j]
      const int c = i / (CIN / 8), slot = i % (CIN / 8);
      *reinterpret_cast<u32x4 *>(lds + OFF_H + c * H_ROWB + ((slot ^ (c & 7)) << 4)) =
          *reinterpret_cast<const u32x4 *>(Hg + (int64_t)c * CIN + slot * 8);
    }
  } else {
    for (int i = tid; i < COUT; i += THREADS) {
      cf[i] = a.alpha[i]; cf[COUT + i] = a.beta[i]; cf[2 * COUT + i] = a.gamma[i];
    }
    if (tid < CIN) { cf[3 * COUT + tid] = a.s[tid]; cf[3 * COUT + CIN + tid] = a.t[tid]; }
  }
  __syncthreads();

  // staging ownership: dy column chunk dc (8 channels), rows dr0 + 8 i; x chunk xc, row xr
  const int dc = tid % DY_CPR, dr0 = tid / DY_CPR;
  const int xc = tid % X_CPR, xr = tid / X_CPR;

  u32x4 rz[DY_NCH], ry[DY_NCH], rx;
  auto load_step = [&](int64_t m0) {   // rows clamped to the slice (zeroed at store time)
#pragma unroll
    for (int i = 0; i < DY_NCH; ++i) {
      const int64_t r = pcs_min64(m0 + dr0 + DY_RP * i, hi - 1);
      const int64_t off = (sbase + r) * COUT + dc * 8;
      rz[i] = *reinterpret_cast<const u32x4 *>(dZ + off);
      if constexpr (!FOLDED) ry[i] = *reinterpret_cast<const u32x4 *>(Yg + off);
    }
    const int64_t r = pcs_min64(m0 + xr, hi - 1);
    rx = *reinterpret_cast<const u32x4 *>(Xg + (sbase + r) * CIN + xc * 8);
  };
  float xsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // FOLDED: this thread's column sums of x
  auto store_step = [&](int64_t m0) {
    if constexpr (FOLDED) {   // dy = dZ: a copy
#pragma unroll
      for (int i = 0; i < DY_NCH; ++i) {
        const int rl = dr0 + DY_RP * i;
        const u32x4 out = m0 + rl >= hi ? mk_u32x4(0, 0, 0, 0) : rz[i];
        *reinterpret_cast<u32x4 *>(lds + OFF_DY + prow(rl) * DY_ROWB + dc * 16) = out;
      }
    } else {
      float ca[8], cb[8], cg[8];
      lds_vec8(cf + dc * 8, ca); lds_vec8(cf + COUT + dc * 8, cb); lds_vec8(cf + 2 * COUT + dc * 8, cg);
#pragma unroll
      for (int i = 0; i < DY_NCH; ++i) {
        const int rl = dr0 + DY_RP * i;
        float v[8], y[8];
        unpack_chunk(rz[i], v);
        unpack_chunk(ry[i], y);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(ca[e], v[e], fmaf(cg[e], y[e], cb[e]));
        u32x4 out = pack_chunk(v);
        if (m0 + rl >= hi) out = mk_u32x4(0, 0, 0, 0);
        *reinterpret_cast<u32x4 *>(lds + OFF_DY + prow(rl) * DY_ROWB + dc * 16) = out;
      }
    }
    float v[8], xs[8], xt[8];
    lds_vec8(cf + CS + xc * 8, xs); lds_vec8(cf + CS + CIN + xc * 8, xt);
    unpack_chunk(rx, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = relu(fmaf(v[e], xs[e], xt[e]));
    u32x4 out = pack_chunk(v);
    if (m0 + xr >= hi) out = mk_u32x4(0, 0, 0, 0);
    if constexpr (FOLDED) {   // the sums of the stored (bf16) x, as the contractions see it
      float d[8];
      unpack_chunk(out, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) xsum[e] += d[e];
    }
    *reinterpret_cast<u32x4 *>(lds + OFF_X + prow(xr) * X_ROWB + xc * 16) = out;
  };

  f32x4 accw[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) accw[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // FOLDED: G = x^T x, tiles (w / 2, 2 (w % 2) + u) of the 4 x 4 16-tiles
  f32x4 accg[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};

  const int nsteps = (int)((hi - lo + MS - 1) / MS);
  if (nsteps > 0) {
    load_step(lo);
    store_step(lo);
    __builtin_amdgcn_sched_barrier(0);
    load_step(lo + MS);   // clamped: harmless when nsteps == 1
  }
  __syncthreads();   // W_l^T, step 0 visible

  const int g = lane >> 4, l16 = lane & 15;
  const int mb = wid >> 1, cb0 = 2 * (wid & 1);   // dgrad rows 16*mb.., column blocks cb0, cb0+1
  const char *tDY = lds + OFF_DY, *tX = lds + OFF_X;
  for (int st = 0; st < nsteps; ++st) {
    const int64_t m0 = lo + (int64_t)st * MS;
    // dgrad: out^T[c][m] = sum_k Wt[c][k] dy[m][k]  (FOLDED: starts at cvec[c], + x H below)
    f32x4 accd[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if constexpr (FOLDED) {
#pragma unroll
      for (int j = 0; j < 2; ++j) accd[j] = *reinterpret_cast<const f32x4 *>(cf + 2 * CIN + (cb0 + j) * 16 + 4 * g);
    }
    const int mrow = prow(mb * 16 + l16);
#pragma unroll 4
    for (int kk = 0; kk < COUT / 32; ++kk) {
      const int slot = 4 * kk + g;
      const bf16x8 yf = *reinterpret_cast<const bf16x8 *>(tDY + mrow * DY_ROWB + slot * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 wf = *reinterpret_cast<const bf16x8 *>(lds + wt_off((cb0 + j) * 16 + l16, slot));
        accd[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, yf, accd[j], 0, 0, 0);
      }
    }
    if constexpr (FOLDED) {   // + x H (K = 64: two k-steps over the staged x tile)
#pragma unroll
      for (int kk = 0; kk < CIN / 32; ++kk) {
        const int slot = 4 * kk + g;
        const bf16x8 xf = *reinterpret_cast<const bf16x8 *>(tX + mrow * X_ROWB + slot * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = (cb0 + j) * 16 + l16;
          const bf16x8 hf = *reinterpret_cast<const bf16x8 *>(lds + OFF_H + c * H_ROWB + ((slot ^ (c & 7)) << 4));
          accd[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf, xf, accd[j], 0, 0, 0);
        }
      }
    }
    // wgrad: dW[o][c] += sum_m dy[m][o] x[m][c]; lane group g holds m = 8g..8g+7 of 32
#pragma unroll
    for (int kk = 0; kk < MS / 32; ++kk) {
      const int q = (lane >> 2) & 3, p = lane & 3;
      const int r0 = prow(32 * kk + 8 * g + q), r1 = prow(32 * kk + 8 * g + 4 + q);
      bf16x8 xf[4], yf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xf[j] = tr_read(tX, r0, r1, X_ROWB, j * 16 + 4 * p);
#pragma unroll
      for (int i = 0; i < 4; ++i) yf[i] = tr_read(tDY, r0, r1, DY_ROWB, wid * 64 + i * 16 + 4 * p);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          accw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[j], yf[i], accw[i][j], 0, 0, 0);
      if constexpr (FOLDED) {   // fragments re-read at this wave's columns (no runtime register index)
        const bf16x8 xi = tr_read(tX, r0, r1, X_ROWB, (wid >> 1) * 16 + 4 * p);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16x8 xj = tr_read(tX, r0, r1, X_ROWB, (2 * (wid & 1) + u) * 16 + 4 * p);
          accg[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xj, xi, accg[u], 0, 0, 0);
        }
      }
    }
    // dA2 tile -> LDS: lane holds out[m = 16 mb + l16][c = 16 cb + 4 g + r]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = (cb0 + j) * 16 + 4 * g;
      *reinterpret_cast<uint2 *>(lds + OFF_OUT + (mb * 16 + l16) * OUT_ROWB + c * 2) =
          make_uint2(pack2bf(accd[j][0], accd[j][1]), pack2bf(accd[j][2], accd[j][3]));
    }
    lds_barrier();   // step st consumed; its dA2 tile complete
    {
      const int r = tid >> 3, ch = tid & 7;   // 64 rows x 8 chunks of 16 B
      if (m0 + r < hi)
        st16(dX + (sbase + m0 + r) * CIN + ch * 8,
             *reinterpret_cast<const u32x4 *>(lds + OFF_OUT + r * OUT_ROWB + ch * 16));
    }
    if (st + 1 < nsteps) {
      store_step(m0 + MS);
      __builtin_amdgcn_sched_barrier(0);
      load_step(m0 + 2 * MS);   // clamped past the end: never consumed
    }
    lds_barrier();
  }

  // this slice's dW partial: lane holds dW[o = 64 w + 16 i + l16][c = 16 j + 4 g ..]
  float *out = a.partial + (int64_t)L * (FOLDED ? SLAB_F : COUT * CIN);
  if constexpr (FOLDED) {
    // G tile (w / 2, 2 (w % 2) + u): lane holds G[16 (w / 2) + l16][16 (2 (w % 2) + u) + 4 g + r]
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<float4 *>(out + COUT * CIN + ((wid >> 1) * 16 + l16) * CIN + (2 * (wid & 1) + u) * 16 + 4 * g) =
          make_float4(accg[u][0], accg[u][1], accg[u][2], accg[u][3]);
    // S: the 64 row-threads of each 8-column chunk, summed in a fixed order through LDS
    __syncthreads();
    float *red = reinterpret_cast<float *>(lds + OFF_DY);   // [64 rows][64 cols]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[xr * CIN + xc * 8 + e] = xsum[e];
    __syncthreads();
    if (tid < CIN) {
      float t = 0.f;
      for (int r = 0; r < X_RP; ++r) t += red[r * CIN + tid];
      out[COUT * CIN + CIN * CIN + tid] = t;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int o = wid * 64 + i * 16 + l16;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<float4 *>(out + o * CIN + j * 16 + 4 * g) =
          make_float4(accw[i][j][0], accw[i][j][1], accw[i][j][2], accw[i][j][3]);
  }
}

int64_t splits_of(const pcs_wgrad_args &a) {
  int64_t sps = (256 + a.num_scenes - 1) / a.num_scenes;   // one workgroup per CU
  const int64_t max_sps = (a.scene_rows + 4 * MS - 1) / (4 * MS);
  if (sps > max_sps) sps = max_sps;
  return sps < 1 ? 1 : sps;
}

bool shapes_ok(const pcs_wgrad_args &a) {
  return a.dtype == PCS_BF16 && a.Cout == COUT && a.Cin == CIN && a.dy_mode == PCS_PRO_BWD &&
         a.x_mode == PCS_PRO_BNRELU && !a.x_mask && !(a.flags & PCS_FLAG_GENERIC);
}

}  // namespace

extern "C" int64_t pcs_dgrad_wgrad_workspace(pcs_wgrad_args *a) {
  if (!a || a->num_scenes <= 0 || a->scene_rows <= 0) return pcs_set_einval("pcs_dgrad_wgrad_workspace", "bad geometry");
  if (!shapes_ok(*a))
    return pcs_set_einval("pcs_dgrad_wgrad_workspace",
                          "bf16, Cout=512, Cin=64, dy_mode PRO_BWD, x_mode PRO_BNRELU, no x_mask only");
  a->splits_per_scene = (int32_t)splits_of(*a);
  return (int64_t)a->num_scenes * a->splits_per_scene * COUT * CIN * 4;
}

extern "C" int pcs_dgrad_wgrad(const pcs_wgrad_args *ap, const void *Wt, void *dX, pcs_stream_t stream) {
  if (!ap || !Wt || !dX) return pcs_set_einval("pcs_dgrad_wgrad", "null argument");
  pcs_wgrad_args a = *ap;
  if (pcs_dgrad_wgrad_workspace(&a) < 0) return PCS_EINVAL;
  if (!a.dZ || !a.Y || !a.alpha || !a.beta || !a.gamma || !a.X || !a.s || !a.t || !a.partial || !a.dW)
    return pcs_set_einval("pcs_dgrad_wgrad", "missing operand");
  if (a.scene_rows * a.num_scenes >= (int64_t)1 << 31) return pcs_set_einval("pcs_dgrad_wgrad", "M must be < 2^31");
  const int64_t rps = ((a.scene_rows + a.splits_per_scene - 1) / a.splits_per_scene + MS - 1) / MS * MS;
  const int nb = (int)(a.num_scenes * a.splits_per_scene);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(dgrad_wgrad_s1_kernel<false>, dim3(nb), dim3(THREADS), 0, s, a, static_cast<const bf16_t *>(Wt),
                     static_cast<bf16_t *>(dX), rps, nullptr, nullptr);
  PCS_CHECK_LAUNCH();
  return pcs_reduce_partials(a.partial, nb, (int64_t)COUT * CIN, 1.0f, a.dW, a.ldw ? a.ldw : CIN, CIN, stream);
}

// ---------------------------------------------------------------------------------------
// Folded form (pcs_dgrad_wgrad_folded): the slab sums, then the Gram-form weight gradient
//   dW_l = diag(alpha) R + beta (x) S + diag(gamma) (W_l G + sum_b scene_bias[b] (x) S_b)
// (dy = alpha dz + beta + gamma Y', Y' = x W_l^T + scene_bias[b]), and the per-scene
// constant row of the input gradient cvec[b] = W_l^T (beta + gamma * scene_bias[b]).
// ---------------------------------------------------------------------------------------
namespace {

constexpr int RG_LEN = COUT * CIN + CIN * CIN;   // R | G, summed over every slab

// red[0 .. RG_LEN) = sum over slabs (fixed order); Sb[b][j] = sum over scene b's slabs
__global__ __launch_bounds__(256) void folded_reduce_kernel(const float *__restrict__ part, int nslab, int sps,
                                                            int B, float *__restrict__ red, float *__restrict__ Sb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < RG_LEN) {
    float t = 0.f;
    for (int sl = 0; sl < nslab; ++sl) t += part[(int64_t)sl * SLAB_F + i];
    red[i] = t;
  } else if (i < RG_LEN + B * CIN) {
    const int b = (i - RG_LEN) / CIN, j = (i - RG_LEN) % CIN;
    float t = 0.f;
    for (int sl = b * sps; sl < (b + 1) * sps; ++sl) t += part[(int64_t)sl * SLAB_F + RG_LEN + j];
    Sb[b * CIN + j] = t;
  }
}

// block = output row k of dW_l (COUT blocks), thread = input channel j (CIN threads)
__global__ __launch_bounds__(CIN) void folded_assemble_kernel(const float *__restrict__ red, const float *__restrict__ Sb,
                                                              int B, const float *__restrict__ W, int64_t ldw,
                                                              const float *__restrict__ alpha,
                                                              const float *__restrict__ beta,
                                                              const float *__restrict__ gamma,
                                                              const float *__restrict__ sbias, float *__restrict__ dW,
                                                              int64_t ldo) {
  __shared__ float wk[CIN];
  const int k = blockIdx.x, j = threadIdx.x;
  wk[j] = W[(int64_t)k * ldw + j];
  __syncthreads();
  const float *G = red + COUT * CIN;
  float wg = 0.f;
  for (int i = 0; i < CIN; ++i) wg = fmaf(wk[i], G[i * CIN + j], wg);
  float S = 0.f, sbs = 0.f;
  for (int b = 0; b < B; ++b) {
    const float sbj = Sb[b * CIN + j];
    S += sbj;
    sbs = fmaf(sbias[(int64_t)b * COUT + k], sbj, sbs);
  }
  dW[(int64_t)k * ldo + j] = fmaf(alpha[k], red[k * CIN + j], fmaf(beta[k], S, gamma[k] * (wg + sbs)));
}

// cvec[b][j] = sum_k (beta[k] + gamma[k] * sbias[b][k]) W[k][j]: block b, thread j
__global__ __launch_bounds__(CIN) void folded_cvec_kernel(const float *__restrict__ W, int64_t ldw,
                                                          const float *__restrict__ beta, const float *__restrict__ gamma,
                                                          const float *__restrict__ sbias, float *__restrict__ cvec) {
  const int b = blockIdx.x, j = threadIdx.x;
  float t = 0.f;
  for (int k = 0; k < COUT; ++k)
    t = fmaf(fmaf(gamma[k], sbias[(int64_t)b * COUT + k], beta[k]), W[(int64_t)k * ldw + j], t);
  cvec[b * CIN + j] = t;
}

bool folded_shapes_ok(const pcs_wgrad_args &a) {
  return a.dtype == PCS_BF16 && a.Cout == COUT && a.Cin == CIN && a.dy_mode == PCS_PRO_RAW &&
         a.x_mode == PCS_PRO_BNRELU && !a.x_mask && !(a.flags & PCS_FLAG_GENERIC);
}

}  // namespace

extern "C" int64_t pcs_dgrad_wgrad_folded_workspace(pcs_wgrad_args *a) {
  if (!a || a->num_scenes <= 0 || a->scene_rows <= 0)
    return pcs_set_einval("pcs_dgrad_wgrad_folded_workspace", "bad geometry");
  if (!folded_shapes_ok(*a))
    return pcs_set_einval("pcs_dgrad_wgrad_folded_workspace",
                          "bf16, Cout=512, Cin=64, dy_mode PRO_RAW, x_mode PRO_BNRELU, no x_mask only");
  a->splits_per_scene = (int32_t)splits_of(*a);
  const int64_t nb = a->num_scenes * a->splits_per_scene;
  return (nb * SLAB_F + RG_LEN + a->num_scenes * CIN + a->num_scenes * CIN) * 4;
}

extern "C" int pcs_dgrad_wgrad_folded(const pcs_wgrad_args *ap, const void *WaT, const void *H, const float *W,
                                      const float *scene_bias, void *dX, pcs_stream_t stream) {
  if (!ap || !WaT || !H || !W || !scene_bias || !dX) return pcs_set_einval("pcs_dgrad_wgrad_folded", "null argument");
  pcs_wgrad_args a = *ap;
  if (pcs_dgrad_wgrad_folded_workspace(&a) < 0) return PCS_EINVAL;
  if (!a.dZ || !a.alpha || !a.beta || !a.gamma || !a.X || !a.s || !a.t || !a.partial || !a.dW || a.ldw < CIN)
    return pcs_set_einval("pcs_dgrad_wgrad_folded", "missing operand (dZ, alpha, beta, gamma, X, s, t, partial, dW, "
                                                    "ldw >= 64)");
  if (a.scene_rows * a.num_scenes >= (int64_t)1 << 31) return pcs_set_einval("pcs_dgrad_wgrad_folded", "M must be < 2^31");
  const int64_t rps = ((a.scene_rows + a.splits_per_scene - 1) / a.splits_per_scene + MS - 1) / MS * MS;
  const int B = (int)a.num_scenes;
  const int nb = B * a.splits_per_scene;
  float *red = a.partial + (int64_t)nb * SLAB_F;
  float *Sb = red + RG_LEN;
  float *cvec = Sb + B * CIN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(folded_cvec_kernel, dim3(B), dim3(CIN), 0, s, W, a.ldw, a.beta, a.gamma, scene_bias, cvec);
  hipLaunchKernelGGL(dgrad_wgrad_s1_kernel<true>, dim3(nb), dim3(THREADS), 0, s, a, static_cast<const bf16_t *>(WaT),
                     static_cast<bf16_t *>(dX), rps, static_cast<const bf16_t *>(H), cvec);
  hipLaunchKernelGGL(folded_reduce_kernel, dim3((RG_LEN + B * CIN + 255) / 256), dim3(256), 0, s, a.partial, nb,
                     a.splits_per_scene, B, red, Sb);
  hipLaunchKernelGGL(folded_assemble_kernel, dim3(COUT), dim3(CIN), 0, s, red, Sb, B, W, a.ldw, a.alpha, a.beta,
                     a.gamma, scene_bias, a.dW, a.ldw);
  PCS_CHECK_LAUNCH();
  return 0;
}

// =======================================================================================
// Fused input + weight gradient of a layer whose input gradient ends in the previous
// layer's ReLU / dropout / BN-statistics epilogue (conv2, conv3, conv4):
//
//   dy   = alpha * dZ + beta + gamma * Y                          ([M, COUT])
//   g    = dy . W  (+ addend)                                     ([M, CIN])
//   dz'  = (es * Yp + et > 0) * keep * ks * g      (stored; S1 = sum dz', S2 = sum dz' Yp)
//   dW  += dy^T . x,   x = relu(es * Yp + et) * keep * ks         ([COUT, CIN])
//
// The dgrad epilogue and the weight gradient read the same Yp (and dropout bits), and both
// contractions read the same dy, so one pass moves dZ, Y, Yp (+ addend) in and dz' out:
// e.g. conv4 0.77 KB per point instead of 1.41 KB for pcs_gemm(DGRAD) + pcs_wgrad.
// A workgroup owns a CB-wide block of the CIN columns (CB = CIN for the 64-wide layers; 128
// for seg_conv2/3, whose W^T and dW do not fit one workgroup): the CIN / CB workgroups of a
// row chunk are consecutive, so they run together on one XCD and the dy slab they all stage
// is served from that XCD's L2 after the first read.
// Structure as dgrad_wgrad_s1_kernel: the W^T block [CB][COUT] resident in LDS, MS-row steps
// with one register prefetch stage; the dgrad accumulators run the epilogue in place (lane:
// one row, 4 consecutive columns per tile), per-lane S1/S2 over the workgroup's rows,
// reduced at the end (16-lane shuffles, then across the waves sharing a column block).
// =======================================================================================
namespace {

template <int COUT, int CIN, int CB, int MS, bool MASK, bool ADD> struct FB {
  static constexpr int NBLK = CIN / CB;
  static constexpr int WT_ROWB = COUT * 2;
  // W^T slot swizzle: c & 15 where a row holds 16 slots or more (as wt_off above), else c & 7
  static constexpr int WSW = COUT >= 128 ? 15 : 7;
  static constexpr int DY_ROWB = COUT * 2 + 32;
  static constexpr int X_ROWB = CB * 2 + 32;
  // Yp / addend rows 16 B and the dz' tile's rows 8 B longer than their data: the epilogue reads
  // (8 B) and writes (8 B) 16 rows at one column, which 128-B rows put on two banks (8-way
  // reads, 16-way writes: SQ_LDS_BANK_CONFLICT 0.5-0.6 of the LDS cycles, r06); padded, the
  // reads are conflict-free and the writes too (the store pass's 16-B reads 2-way)
  static constexpr int YP_ROWB = CB * 2 + 16;
  static constexpr int OUT_ROWB = CB * 2 + 8;
  static constexpr int OFF_DY = CB * WT_ROWB;
  static constexpr int OFF_X = OFF_DY + MS * DY_ROWB;
  static constexpr int OFF_YP = OFF_X + MS * X_ROWB;
  static constexpr int OFF_AD = OFF_YP + MS * YP_ROWB;
  static constexpr int OFF_MK = OFF_AD + (ADD ? MS * YP_ROWB : 0);
  static constexpr int OFF_OUT = OFF_MK + (MASK ? MS * CB / 8 : 0);
  static constexpr int OFF_COEF = OFF_OUT + MS * OUT_ROWB;   // alpha|beta|gamma [COUT], es|et [CB]
  static constexpr int BYTES = OFF_COEF + (3 * COUT + 2 * CB) * 4;
  static constexpr bool FITS = BYTES <= 160 * 1024;   // LDS budget (checked in the kernel)
  static_assert(CIN % CB == 0, "column blocks");
  static constexpr int NCB = CB / 16, NMB = MS / 16, NOB = COUT / 16;
  static constexpr int TPW_D = NMB * NCB / 8, TPW_W = NOB * NCB / 8;   // tiles per wave
  static constexpr int OBW = TPW_W > NCB ? TPW_W / NCB : 1;            // wgrad row blocks per wave
  static_assert(TPW_D >= 1 && TPW_W >= 1 && NCB % TPW_D == 0, "dgrad wave tiling");
  static_assert(TPW_W % NCB == 0 || NCB % TPW_W == 0, "wgrad wave tiling");
  static constexpr int CBW = TPW_W / OBW;                              // wgrad column blocks per wave
  static constexpr int NCH_D = MS * COUT / 8 / THREADS, NCH_P = MS * CB / 8 / THREADS;
  static_assert(NCH_D >= 1 && NCH_P >= 1 && MS % 32 == 0, "staging");
};

PCS_DEV float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
PCS_DEV float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// (the 64-wide layers run two workgroups per CU: at most 128 VGPRs)
template <int COUT, int CIN, int CB, int MS, bool MASK, bool ADD>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(COUT == 64 ? 4 : 1, 8))) void dgrad_wgrad_bn_kernel(pcs_gemm_args a, float *__restrict__ wpart,
                                                                 int64_t rows_per_split) {
  typedef FB<COUT, CIN, CB, MS, MASK, ADD> F;
  static_assert(F::FITS, "LDS budget");
  __shared__ __attribute__((aligned(16))) char lds[F::BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = L / F::NBLK, n0 = (L % F::NBLK) * CB;
  const int sps = a.chunks_per_scene;
  const int scene = chunk / sps, sis = chunk % sps;
  const int64_t N = a.scene_rows;
  const int64_t lo = (int64_t)sis * rows_per_split;
  const int64_t hi = pcs_min64(lo + rows_per_split, N);
  const int64_t sbase = (int64_t)scene * N;
  const bf16_t *__restrict__ dZ = reinterpret_cast<const bf16_t *>(a.A);
  const bf16_t *__restrict__ Yg = reinterpret_cast<const bf16_t *>(a.A2);
  const bf16_t *__restrict__ Ypg = reinterpret_cast<const bf16_t *>(a.Yp);
  const bf16_t *__restrict__ Adg = reinterpret_cast<const bf16_t *>(a.addend);
  const bf16_t *__restrict__ Wt = reinterpret_cast<const bf16_t *>(a.W);
  bf16_t *__restrict__ Cg = reinterpret_cast<bf16_t *>(a.C);
  const float ks = MASK ? a.c_keep_scale : 1.f;

  for (int i = tid; i < CB * COUT / 8; i += THREADS) {   // W^T rows n0.. [CB][COUT] -> LDS
    const int c = i / (COUT / 8), slot = i % (COUT / 8);
    *reinterpret_cast<u32x4 *>(lds + c * F::WT_ROWB + ((slot ^ (c & F::WSW)) << 4)) =
        *reinterpret_cast<const u32x4 *>(Wt + (int64_t)(n0 + c) * COUT + slot * 8);
  }
  float *cf = reinterpret_cast<float *>(lds + F::OFF_COEF);
  for (int i = tid; i < COUT; i += THREADS) { cf[i] = a.pa[i]; cf[COUT + i] = a.pb[i]; cf[2 * COUT + i] = a.pc[i]; }
  for (int i = tid; i < CB; i += THREADS) { cf[3 * COUT + i] = a.es[n0 + i]; cf[3 * COUT + CB + i] = a.et[n0 + i]; }
  __syncthreads();

  u32x4 rz[F::NCH_D], ry[F::NCH_D], rp[F::NCH_P], rd[ADD ? F::NCH_P : 1];
  uint32_t rm[MASK ? F::NCH_P : 1];
  auto load_step = [&](int64_t m0) {
#pragma unroll
    for (int i = 0; i < F::NCH_D; ++i) {
      const int q = tid + THREADS * i, rl = q / (COUT / 8), cc = q % (COUT / 8);
      const int64_t off = (sbase + pcs_min64(m0 + rl, hi - 1)) * COUT + cc * 8;
      rz[i] = *reinterpret_cast<const u32x4 *>(dZ + off);
      ry[i] = *reinterpret_cast<const u32x4 *>(Yg + off);
    }
#pragma unroll
    for (int i = 0; i < F::NCH_P; ++i) {
      const int q = tid + THREADS * i, rl = q / (CB / 8), cc = q % (CB / 8);
      const int64_t off = (sbase + pcs_min64(m0 + rl, hi - 1)) * CIN + n0 + cc * 8;
      rp[i] = *reinterpret_cast<const u32x4 *>(Ypg + off);
      if constexpr (ADD) rd[i] = *reinterpret_cast<const u32x4 *>(Adg + off);
      if constexpr (MASK) rm[i] = a.c_mask[off >> 3];
    }
  };
  auto store_step = [&](int64_t m0) {
#pragma unroll
    for (int i = 0; i < F::NCH_D; ++i) {
      const int q = tid + THREADS * i, rl = q / (COUT / 8), cc = q % (COUT / 8);
      float ca[8], cb[8], cg[8], v[8], y[8];
      lds_vec8(cf + cc * 8, ca); lds_vec8(cf + COUT + cc * 8, cb); lds_vec8(cf + 2 * COUT + cc * 8, cg);
      unpack_chunk(rz[i], v);
      unpack_chunk(ry[i], y);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(ca[e], v[e], fmaf(cg[e], y[e], cb[e]));
      u32x4 out = pack_chunk(v);
      if (m0 + rl >= hi) out = mk_u32x4(0, 0, 0, 0);
      *reinterpret_cast<u32x4 *>(lds + F::OFF_DY + prow(rl) * F::DY_ROWB + cc * 16) = out;
    }
#pragma unroll
    for (int i = 0; i < F::NCH_P; ++i) {
      const int q = tid + THREADS * i, rl = q / (CB / 8), cc = q % (CB / 8);
      float s8[8], t8[8], v[8];
      lds_vec8(cf + 3 * COUT + cc * 8, s8); lds_vec8(cf + 3 * COUT + CB + cc * 8, t8);
      unpack_chunk(rp[i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = relu(fmaf(v[e], s8[e], t8[e]));
        if constexpr (MASK) x = ((rm[i] >> e) & 1u) ? x * ks : 0.f;
        v[e] = x;
      }
      u32x4 out = pack_chunk(v);
      if (m0 + rl >= hi) out = mk_u32x4(0, 0, 0, 0);
      *reinterpret_cast<u32x4 *>(lds + F::OFF_X + prow(rl) * F::X_ROWB + cc * 16) = out;
      *reinterpret_cast<u32x4 *>(lds + F::OFF_YP + rl * F::YP_ROWB + cc * 16) = rp[i];
      if constexpr (ADD) *reinterpret_cast<u32x4 *>(lds + F::OFF_AD + rl * F::YP_ROWB + cc * 16) = rd[i];
      if constexpr (MASK) lds[F::OFF_MK + rl * (CB / 8) + cc] = (char)rm[i];
    }
  };

  f32x4 accw[F::OBW][F::CBW];
#pragma unroll
  for (int o = 0; o < F::OBW; ++o)
#pragma unroll
    for (int u = 0; u < F::CBW; ++u) accw[o][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s1[F::TPW_D][4], s2[F::TPW_D][4];
#pragma unroll
  for (int u = 0; u < F::TPW_D; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[u][r] = 0.f; s2[u][r] = 0.f; }

  const int nsteps = (int)((hi - lo + MS - 1) / MS);
  if (nsteps > 0) {
    load_step(lo);
    store_step(lo);
    __builtin_amdgcn_sched_barrier(0);
    load_step(lo + MS);
  }
  __syncthreads();

  const int g = lane >> 4, l16 = lane & 15;
  const int td0 = wid * F::TPW_D, mb = td0 / F::NCB, cbd = td0 % F::NCB;   // dgrad tiles (same mb)
  const int tw0 = wid * F::TPW_W, ob0 = tw0 / F::NCB, cbw = tw0 % F::NCB;  // wgrad: OBW row blocks x CBW
  const char *tDY = lds + F::OFF_DY, *tX = lds + F::OFF_X;
  const int ml = mb * 16 + l16;   // this lane's row of the dgrad tiles
  for (int st = 0; st < nsteps; ++st) {
    const int64_t m0 = lo + (int64_t)st * MS;
    f32x4 accd[F::TPW_D];
#pragma unroll
    for (int u = 0; u < F::TPW_D; ++u) accd[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int kk = 0; kk < COUT / 32; ++kk) {
      const int slot = 4 * kk + g;
      const bf16x8 yf = *reinterpret_cast<const bf16x8 *>(tDY + prow(ml) * F::DY_ROWB + slot * 16);
#pragma unroll
      for (int u = 0; u < F::TPW_D; ++u) {
        const int c = (cbd + u) * 16 + l16;
        const bf16x8 wf = *reinterpret_cast<const bf16x8 *>(lds + c * F::WT_ROWB + ((slot ^ (c & F::WSW)) << 4));
        accd[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, yf, accd[u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int kk = 0; kk < MS / 32; ++kk) {
      const int q = (lane >> 2) & 3, p = lane & 3;
      const int r0 = prow(32 * kk + 8 * g + q), r1 = prow(32 * kk + 8 * g + 4 + q);
      bf16x8 yf[F::OBW];   // the few dy fragments stay live; x fragments are read one at a time
#pragma unroll
      for (int o = 0; o < F::OBW; ++o) yf[o] = tr_read(tDY, r0, r1, F::DY_ROWB, (ob0 + o) * 16 + 4 * p);
#pragma unroll
      for (int u = 0; u < F::CBW; ++u) {
        const bf16x8 xf = tr_read(tX, r0, r1, F::X_ROWB, (cbw + u) * 16 + 4 * p);
#pragma unroll
        for (int o = 0; o < F::OBW; ++o)
          accw[o][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, yf[o], accw[o][u], 0, 0, 0);
      }
    }
    // epilogue in place: lane holds g[m = ml][c = 16 (cbd + u) + 4 g + r] (block-local c)
    const bool live = m0 + ml < hi;
#pragma unroll
    for (int u = 0; u < F::TPW_D; ++u) {
      const int c = (cbd + u) * 16 + 4 * g;
      const uint2 yp = *reinterpret_cast<const uint2 *>(lds + F::OFF_YP + ml * F::YP_ROWB + c * 2);
      const float y[4] = {bf_lo(yp.x), bf_hi(yp.x), bf_lo(yp.y), bf_hi(yp.y)};
      float v[4] = {accd[u][0], accd[u][1], accd[u][2], accd[u][3]};
      if constexpr (ADD) {
        const uint2 ad = *reinterpret_cast<const uint2 *>(lds + F::OFF_AD + ml * F::YP_ROWB + c * 2);
        v[0] += bf_lo(ad.x); v[1] += bf_hi(ad.x); v[2] += bf_lo(ad.y); v[3] += bf_hi(ad.y);
      }
      uint32_t kb = 0xFu;
      if constexpr (MASK) kb = ((uint32_t)(uint8_t)lds[F::OFF_MK + ml * (CB / 8) + (c >> 3)] >> (c & 7)) & 0xFu;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float gv = v[r];
        if constexpr (MASK) gv = ((kb >> r) & 1u) ? gv * ks : 0.f;
        const float dz = (live && fmaf(y[r], cf[3 * COUT + c + r], cf[3 * COUT + CB + c + r]) > 0.f) ? gv : 0.f;
        v[r] = dz;
        s1[u][r] += dz;
        s2[u][r] = fmaf(dz, y[r], s2[u][r]);
      }
      *reinterpret_cast<uint2 *>(lds + F::OFF_OUT + ml * F::OUT_ROWB + c * 2) =
          make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
    }
    lds_barrier();   // step st consumed; its dz' tile complete
#pragma unroll
    for (int i = 0; i < F::NCH_P; ++i) {
      const int q = tid + THREADS * i, rl = q / (CB / 8), cc = q % (CB / 8);
      if (m0 + rl < hi)
        st16(Cg + (sbase + m0 + rl) * CIN + n0 + cc * 8,
             *reinterpret_cast<const u32x4 *>(lds + F::OFF_OUT + rl * F::OUT_ROWB + cc * 16));
    }
    if (st + 1 < nsteps) {
      store_step(m0 + MS);
      __builtin_amdgcn_sched_barrier(0);
      load_step(m0 + 2 * MS);
    }
    lds_barrier();
  }

  // dW partial (chunk slab, columns n0..): lane holds dW[o = 16 (ob0 + o) + l16][c = 16 (cbw + u) + 4 g ..]
  float *out = wpart + (int64_t)chunk * COUT * CIN + n0;
#pragma unroll
  for (int o = 0; o < F::OBW; ++o)
#pragma unroll
    for (int u = 0; u < F::CBW; ++u)
      *reinterpret_cast<float4 *>(out + ((ob0 + o) * 16 + l16) * CIN + (cbw + u) * 16 + 4 * g) =
          make_float4(accw[o][u][0], accw[o][u][1], accw[o][u][2], accw[o][u][3]);

  // S1 / S2: sum the 16 rows (lanes l16) of each column, then the NMB row blocks via LDS
#pragma unroll
  for (int u = 0; u < F::TPW_D; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[u][r] += __shfl_xor(s1[u][r], o);
        s2[u][r] += __shfl_xor(s2[u][r], o);
      }
  float2 *red = reinterpret_cast<float2 *>(lds);   // [NMB][CB] (W^T area, no longer read)
  if (l16 == 0) {
#pragma unroll
    for (int u = 0; u < F::TPW_D; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[mb * CB + (cbd + u) * 16 + 4 * g + r] = make_float2(s1[u][r], s2[u][r]);
  }
  __syncthreads();
  for (int c = tid; c < CB; c += THREADS) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int b = 0; b < F::NMB; ++b) { t1 += red[b * CB + c].x; t2 += red[b * CB + c].y; }
    *reinterpret_cast<float2 *>(a.stats + ((int64_t)chunk * CIN + n0 + c) * 2) =
        make_float2(t1, a.erstd[n0 + c] * (t2 - a.emean[n0 + c] * t1));
  }
}

template <int COUT, int CIN, int CB, int MS>
int launch_bn(const pcs_gemm_args &a, float *wpart, int64_t rps, hipStream_t s) {
  const int nb = (int)(a.num_scenes * a.chunks_per_scene) * (CIN / CB);
  if (a.c_mask && a.addend) return pcs_set_einval("pcs_dgrad_wgrad_bn", "mask and addend together");
  if (a.c_mask)
    hipLaunchKernelGGL((dgrad_wgrad_bn_kernel<COUT, CIN, CB, MS, true, false>), dim3(nb), dim3(THREADS), 0, s, a, wpart, rps);
  else if (a.addend) {
    if constexpr (FB<COUT, CIN, CB, MS, false, true>::FITS)
      hipLaunchKernelGGL((dgrad_wgrad_bn_kernel<COUT, CIN, CB, MS, false, true>), dim3(nb), dim3(THREADS), 0, s, a, wpart,
                         rps);
    else
      return pcs_set_einval("pcs_dgrad_wgrad_bn", "no addend variant at this shape (LDS)");
  } else
    hipLaunchKernelGGL((dgrad_wgrad_bn_kernel<COUT, CIN, CB, MS, false, false>), dim3(nb), dim3(THREADS), 0, s, a,
                       wpart, rps);
  PCS_CHECK_LAUNCH();
  return 0;
}

// (Cout, Cin) pairs served: (column block, rows per step).  The column-block split also
// instantiates seg_conv3 (128 x 256, CB 128, 64-row steps) and seg_conv2 (256 x 512, CB 128,
// 32-row steps: 64 spill VGPRs); both are correct (tests/test_gpu_fused_bwd.py history) but
// measured no faster at cfg2 than the pcs_gemm + pcs_wgrad pair they replace (seg_conv3
// 4.96 vs 4.73 ms, seg_conv2 12.8 vs 12.6 ms: 2 TB/s, latency-bound at one workgroup per
// CU with the dy slab staged once per column block), so they stay on the pair.
struct BnShape { int cout, cin, cb, ms; };
// (seg_conv2 and seg_conv3 go to the LDS-DMA stream of fused_seg4.hip instead)
constexpr BnShape kBnShapes[] = {{64, 64, 64, 64}, {128, 64, 64, 64}};

const BnShape *bn_shape(int K, int Ncols) {
  for (const BnShape &b : kBnShapes)
    if (b.cout == K && b.cin == Ncols) return &b;
  return nullptr;
}

}  // namespace

extern "C" int64_t pcs_dgrad_wgrad_bn_workspace(pcs_gemm_args *a) {
  if (!a || a->num_scenes <= 0 || a->scene_rows <= 0) return pcs_set_einval("pcs_dgrad_wgrad_bn_workspace", "bad geometry");
  if (pcs_seg4_applicable(*a)) {   // seg_conv2 / seg_conv3: one wave per SIMD (fused_seg4.hip)
    pcs_seg4_geometry(a);
    return (int64_t)a->num_scenes * a->chunks_per_scene * a->K * a->Ncols * 4;
  }
  const BnShape *sh = bn_shape(a->K, a->Ncols);
  if (a->dtype != PCS_BF16 || !sh || (a->flags & PCS_FLAG_GENERIC))
    return pcs_set_einval("pcs_dgrad_wgrad_bn_workspace",
                          "bf16 with (Cout, Cin) = K x Ncols in {64x64, 128x64} only");
  const int nblk = sh->cin / sh->cb;
  // 64 x 64 (conv2, conv3: <= 128 VGPRs) fits two 512-thread workgroups per CU: twice the
  // workgroups, 0.91 -> 0.85 ms at cfg2; 128 x 64 (conv4, 158-164 VGPRs) stays at one
  const int64_t target = sh->cout == 64 ? 512 : 256;
  int64_t sps = (target + a->num_scenes * nblk - 1) / (a->num_scenes * nblk);
  const int64_t max_sps = (a->scene_rows + 4 * sh->ms - 1) / (4 * sh->ms);
  if (sps > max_sps) sps = max_sps;
  if (sps < 1) sps = 1;
  const int64_t rps = ((a->scene_rows + sps - 1) / sps + sh->ms - 1) / sh->ms * sh->ms;
  a->chunks_per_scene = (int32_t)((a->scene_rows + rps - 1) / rps);   // no empty chunks
  return (int64_t)a->num_scenes * a->chunks_per_scene * a->K * a->Ncols * 4;
}

extern "C" int pcs_dgrad_wgrad_bn(const pcs_gemm_args *ap, float *partial, float *dW, int64_t ldw,
                                  pcs_stream_t stream) {
  if (!ap || !partial || !dW) return pcs_set_einval("pcs_dgrad_wgrad_bn", "null argument");
  pcs_gemm_args a = *ap;
  if (pcs_dgrad_wgrad_bn_workspace(&a) < 0) return PCS_EINVAL;
  if (a.chunks_per_scene != ap->chunks_per_scene)
    return pcs_set_einval("pcs_dgrad_wgrad_bn", "chunks_per_scene must come from pcs_dgrad_wgrad_bn_workspace");
  if (!a.A || !a.A2 || !a.pa || !a.pb || !a.pc || !a.W || !a.C || !a.Yp || !a.es || !a.et || !a.emean ||
      !a.erstd || !a.stats)
    return pcs_set_einval("pcs_dgrad_wgrad_bn", "missing operand (A, A2, pa, pb, pc, W, C, Yp, es, et, emean, "
                                                "erstd, stats)");
  if (a.scene_rows * a.num_scenes >= (int64_t)1 << 31) return pcs_set_einval("pcs_dgrad_wgrad_bn", "M must be < 2^31");
  if (pcs_seg4_applicable(a)) {
    const int rc = pcs_seg4_launch(a, partial, reinterpret_cast<hipStream_t>(stream));
    if (rc) return rc;
    const int nslab = (int)(a.num_scenes * a.chunks_per_scene);
    return pcs_reduce_partials(partial, nslab, (int64_t)a.K * a.Ncols, 1.0f, dW, ldw ? ldw : a.Ncols, a.Ncols, stream);
  }
  const BnShape *sh = bn_shape(a.K, a.Ncols);
  const int64_t rps = ((a.scene_rows + a.chunks_per_scene - 1) / a.chunks_per_scene + sh->ms - 1) / sh->ms * sh->ms;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc;
  if (a.K == 64) rc = launch_bn<64, 64, 64, 64>(a, partial, rps, s);
  else rc = launch_bn<128, 64, 64, 64>(a, partial, rps, s);
  if (rc) return rc;
  const int nslab = (int)(a.num_scenes * a.chunks_per_scene);
  return pcs_reduce_partials(partial, nslab, (int64_t)a.K * a.Ncols, 1.0f, dW, ldw ? ldw : a.Ncols, a.Ncols, stream);
}

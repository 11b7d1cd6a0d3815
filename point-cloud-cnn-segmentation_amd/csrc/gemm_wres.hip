// W-resident streaming GEMM for conv5's second pass (P:110 with bn5 + ReLU, the forward of
// the 1024-wide layer's input): a5 = relu(bn5(relu(bn4(y4)) W5^T)), K = 128, stored as bf16
// or fp8 e4m3, with per-chunk column sums of the stored values (S of global_feat's Gram-form
// weight gradient).
//
// At K = 128 the work per output element is small (256 FLOP per 2 or 1 stored bytes); the
// register-staged 256x256 kernel (gemm_big.hip), which drains its pipeline into an LDS tile at
// every epilogue, ran the fp8 form at 2.2 TB/s.  Here (used for the fp8 store; see
// pcs_gemm_wres_applicable for the bf16 measurement):
// * a workgroup owns 256 output columns for its whole row chunk: that 256 x 128 block of W is
//   loaded into LDS once (64 KB, XOR-swizzled 16-B slots) and stays there;
// * y4 streams through a 5-stage LDS ring of 64-row tiles by LDS-DMA
//   (global_load_lds_dwordx4): tile t+4 is requested as soon as tile t-1's stage is free, so
//   four tiles of loads are in flight while tile t computes;
// * a tile's output is stored one tile late -- fp8: staged in the half's own rows of the tile's
//   A stage (dead between its MFMAs and its restaging) and stored as whole 256-B row segments
//   (4.4 -> 4.0 ms against 16 rows x 32 B per store instruction); bf16: packed in registers,
//   16 rows x 64 B per store (its 16 KB per half do not fit those rows) -- and the wait for
//   a tile's DMA is counted: vmcnt(n) with n = the vector-memory operations issued after it
//   (gfx9 retires loads and stores on this counter in issue order, as hipcc itself assumes),
//   so neither the newer loads nor the recent stores are drained;
// * bn4 + ReLU is applied once per element, in place in LDS, one tile ahead of the MFMAs
//   (the narrow-K passes are VALU-bound: transforming each fragment in every column wave
//   cost 4x the VALU, and the epilogue uses packed fp32 math);
// * 8 waves as 2 (rows) x 4 (columns), 32 x 64 outputs per wave; the epilogue applies
//   bn5 + ReLU to the accumulators, rounds to the storage type, widens the stores with
//   v_permlane16_swap (16 B bf16 / 8 B fp8 per lane) and keeps per-lane column sums across
//   the chunk in registers (one 16-lane reduction per chunk, not per tile).
#include "common.h"

#include <type_traits>

namespace {

constexpr int THREADS = 512;
constexpr int K = 128;                  // conv5's input width
constexpr int BMW = 64, BNW = 256;      // row tile, column block
constexpr int NSTAGE = 5;               // A ring depth
constexpr int ROWB = K * 2;             // 256 B per LDS row (W and A)
constexpr int W_BYTES = BNW * ROWB;     // 64 KB
constexpr int A_BYTES = BMW * ROWB;     // 16 KB per stage
constexpr int PIECES = A_BYTES / 1024 / 8;   // 1-KB DMA pieces per wave per tile (2)
constexpr int NI = BMW / 32;            // 16-row MFMA tiles per wave (2)
constexpr int OFF_A = W_BYTES;
constexpr int OFF_RED = OFF_A + NSTAGE * A_BYTES;      // [2 wm][256] f32 column sums (chunk end)
constexpr int OFF_PRO = OFF_RED + 2 * BNW * 4;          // bn4 scale | shift [K] f32
constexpr int LDS_BYTES = OFF_PRO + 2 * K * 4;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

typedef __attribute__((address_space(3))) void lds_void_t;

PCS_DEV int xcd_remap(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
// 16-B slot s of LDS row r holds logical slot s ^ (r & 15): the 16 rows a 16-lane group of
// ds_read_b128 touches at one logical slot land in 16 distinct slots (all 64 banks)
PCS_DEV int swz(int r, int slot) { return slot ^ (r & 15); }

PCS_DEV void glds16(const char *sbase, uint32_t voff, char *lds_dst) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(lds_void_t *)lds_dst;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(m0v)
               : "memory");
}
template <int N> PCS_DEV void wait_vm() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// wait until at most n (rounded down to the ladder) vector-memory operations are outstanding
PCS_DEV void wait_vm_dyn(int n) {
  if (n >= 24) wait_vm<24>();
  else if (n >= 20) wait_vm<20>();
  else if (n >= 16) wait_vm<16>();
  else if (n >= 12) wait_vm<12>();
  else if (n >= 8) wait_vm<8>();
  else if (n >= 6) wait_vm<6>();
  else if (n >= 4) wait_vm<4>();
  else if (n >= 2) wait_vm<2>();
  else wait_vm<0>();
}
PCS_DEV void barrier_raw() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
PCS_DEV void lds_vec8(const float *p, float (&v)[8]) {
  const float4 x = *reinterpret_cast<const float4 *>(p);
  const float4 y = *reinterpret_cast<const float4 *>(p + 4);
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}
PCS_DEV float dpp_sum16(float v) {   // sum over the 16 lanes of a DPP row (every lane gets it)
  auto d = [](float x, auto ctrl) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), decltype(ctrl)::value,
                                                                 0xF, 0xF, false));
  };
  v += d(v, std::integral_constant<int, 0xB1>{});
  v += d(v, std::integral_constant<int, 0x4E>{});
  v += d(v, std::integral_constant<int, 0x141>{});
  return v + d(v, std::integral_constant<int, 0x140>{});
}

template <bool C8>
__global__ __launch_bounds__(THREADS) void wres_bnrelu_kernel(pcs_gemm_args a, int tiles_per_scene, int tiles_per_chunk,
                                                              int ncb) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = L / ncb, cb = L % ncb;
  const int cps = a.chunks_per_scene;
  const int scene = chunk / cps, cis = chunk % cps;
  const int n0 = cb * BNW;
  const int Ncols = a.Ncols;
  const int64_t N = a.scene_rows;
  const int t_begin = cis * tiles_per_chunk;
  const int t_end = min(t_begin + tiles_per_chunk, tiles_per_scene);
  const int64_t scene_row0 = (int64_t)scene * N;
  const int ntl = t_end - t_begin;   // may be <= 0: the chunk's column sums are still written

  // ---- W block (rows n0 .. n0+255 of W [Ncols][K]) -> LDS, once; per-lane coefficients
  const char *Wb = reinterpret_cast<const char *>(a.W) + (int64_t)n0 * ROWB;
  for (int i = tid; i < BNW * (ROWB / 16); i += THREADS) {
    const int r = i / (ROWB / 16), sl = i % (ROWB / 16);
    *reinterpret_cast<u32x4 *>(lds + r * ROWB + swz(r, sl) * 16) =
        *reinterpret_cast<const u32x4 *>(Wb + (int64_t)r * ROWB + sl * 16);
  }
  // bn4 + ReLU coefficients -> LDS (read per fragment k-range)
  float *lpro = reinterpret_cast<float *>(lds + OFF_PRO);
  if (tid < K) { lpro[tid] = a.pa[tid]; lpro[K + tid] = a.pb[tid]; }
  // bn5 (+ bias) of the lane's 16 columns c = n0 + 64 wn + 16 j + 4 lg + (2 h + e), as pairs
  f32x2 es2[4][2], et2[4][2], csum2[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int c = n0 + 64 * wn + 16 * j + 4 * lg + 2 * h + e;
        es2[j][h][e] = a.es[c];
        et2[j][h][e] = a.et[c] + (a.bias ? a.bias[c] * a.es[c] : 0.f);
        csum2[j][h][e] = 0.f;
      }
  __syncthreads();   // W in LDS; every ordinary load above has retired before the first DMA
  // (from here on no ordinary global load: hipcc would wait vmcnt(0) at its first use)

  // ---- A tile DMA: piece g of wave w = rows (PIECES w + g) * 4 + lane / 16, slot lane % 16
  const char *Ab = reinterpret_cast<const char *>(a.A);
  uint32_t poff[PIECES];
  int prow[PIECES];
#pragma unroll
  for (int g = 0; g < PIECES; ++g) {
    prow[g] = (PIECES * wid + g) * 4 + (lane >> 4);
    poff[g] = (uint32_t)swz(prow[g], lane & 15) * 16u;
  }
  // vector-memory operations this wave has issued, and that count right after each stage's
  // DMA (the wait for a stage is vmcnt(issued - mark))
  int issued = 0;
  int mark[NSTAGE];
  auto issue = [&](int t) {   // tile t of the chunk -> stage t % NSTAGE
    if (t >= ntl) return;
    const int64_t rb = scene_row0 + (int64_t)(t_begin + t) * BMW;
    const int valid = (int)pcs_min64(BMW, scene_row0 + N - rb);
    const char *sb = Ab + rb * ROWB;
    char *dst = lds + OFF_A + (t % NSTAGE) * A_BYTES;
#pragma unroll
    for (int g = 0; g < PIECES; ++g) {
      const uint32_t r = (uint32_t)min(prow[g], valid - 1);   // rows past the scene: clamped
      glds16(sb, r * (uint32_t)ROWB + poff[g], dst + (PIECES * wid + g) * 1024);
    }
    issued += PIECES;
    mark[t % NSTAGE] = issued;
  };
#pragma unroll
  for (int t = 0; t < NSTAGE - 1; ++t) issue(t);
  // in-place bn4 + ReLU of a landed stage, each wave half over its own 32 rows (the rows its
  // waves load and read): thread th of the half = chunks th and th + 256 (rows 32 wm + th/16
  // and + 16, physical slot th % 16, whose logical k-range is fixed per thread)
  const int th = tid & 255;
  float ts[8], tt[8];
  {
    const int ls = (th & 15) ^ (th >> 4);
    lds_vec8(lpro + 8 * ls, ts);
    lds_vec8(lpro + K + 8 * ls, tt);
  }
  auto transform = [&](int t) {
    char *st = lds + OFF_A + (t % NSTAGE) * A_BYTES + wm * (BMW / 2) * ROWB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u32x4 *p = reinterpret_cast<u32x4 *>(st + (th + 256 * h) * 16);
      float v[8];
      unpack_chunk(*p, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = relu(fmaf(v[e], ts[e], tt[e]));
      *p = pack_chunk(v);
    }
  };
  if (ntl > 0) {
    wait_vm_dyn(issued - mark[0]);
    barrier_raw();
    transform(0);
  }

  const int scol = n0 + wn * 64 + 16 * (lg & 1) + 8 * (lg >> 1);   // store column of pair q: + 32 q
  constexpr int PW = C8 ? 2 : 4;   // packed dwords per (row i, tile pair q)
  uint32_t pend[NI][2][PW];        // the previous tile's output, stored one tile late
  int64_t pend_rb = 0;
  int pend_valid = 0;
  // fp8: the packed outputs of tile t go to the half's own rows of A stage t (dead once its
  // MFMAs have read it, until it is restaged one iteration later) in the A layout's swizzle,
  // and are stored from there as whole 256-B row segments (16 lanes per row, two 16-B
  // chunks per lane) instead of 16 rows x 32 B per store instruction
  const int hq = tid & 255;   // the thread's index in its half
  auto store_rows = [&](int t) {
    const char *st = lds + OFF_A + (t % NSTAGE) * A_BYTES;
    if (pend_valid == BMW) issued += 2;   // a partial tile may skip stores: count none
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = hq + 256 * h, r = wm * (BMW / 2) + (q >> 4), sl = q & 15;
      const u32x4 v = *reinterpret_cast<const u32x4 *>(st + r * ROWB + swz(r, sl) * 16);
      if (r < pend_valid)
        *reinterpret_cast<u32x4 *>(reinterpret_cast<fp8_t *>(a.C) + (pend_rb + r) * Ncols + n0 + sl * 16) = v;
    }
  };
  auto store_pending = [&]() {
    // a partial tile's stores may skip whole waves: count none of them (over-waits, safely)
    if (pend_valid == BMW) issued += NI * 2;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int m = wm * (BMW / 2) + i * 16 + lr;
      if (m >= pend_valid) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int64_t e0 = (pend_rb + m) * Ncols + scol + 32 * q;
        if constexpr (C8)   // plain store (measured 2 % faster than non-temporal here)
          *reinterpret_cast<uint64_t *>(reinterpret_cast<fp8_t *>(a.C) + e0) = (uint64_t)pend[i][q][1] << 32 | pend[i][q][0];
        else
          st16(reinterpret_cast<bf16_t *>(a.C) + e0, mk_u32x4(pend[i][q][0], pend[i][q][1], pend[i][q][2], pend[i][q][3]));
      }
    }
  };
  // The two wave halves (rows 0-31 / 32-63 of every tile: each half loads, transforms and
  // reads only its own rows) run one barrier apart, and an iteration has two sections: while
  // one half issues its MFMAs (section 1) the other runs its epilogue, stores and transform
  // (section 2), so each SIMD (one wave of each half) overlaps matrix and vector work.
  if (wm == 1) barrier_raw();
  for (int t = 0; t < ntl; ++t) {
    // section 1: tile t's transformed rows are visible to the half (the transform writes of
    // the previous section 2 retired before this barrier)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_raw();
    if constexpr (C8) {
      if (t > 0) store_rows(t - 1);   // tile t-1's rows, staged in its A stage by section 2
    }
    const char *At = lds + OFF_A + (t % NSTAGE) * A_BYTES;
    f32x4 acc[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8 wf[4], af[NI];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + lr;
        wf[j] = *reinterpret_cast<const bf16x8 *>(lds + r * ROWB + swz(r, 4 * kk + lg) * 16);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int r = wm * (BMW / 2) + i * 16 + lr;
        af[i] = *reinterpret_cast<const bf16x8 *>(At + r * ROWB + swz(r, 4 * kk + lg) * 16);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
    }
    // this wave's pieces of tile t+1 have landed (everything issued after them may still be in
    // flight); after the next barrier the half's have
    if (t + 1 < ntl) wait_vm_dyn(issued - mark[(t + 1) % NSTAGE]);
    // section 2: restage tile t-1's rows (read in the previous section 1), store tile t-1,
    // transform tile t+1, epilogue of tile t
    barrier_raw();
    issue(t + NSTAGE - 1);
    if constexpr (!C8) {
      if (t > 0) store_pending();
    }
    if (t + 1 < ntl) transform(t + 1);
    // ---- epilogue: lane holds a5[m = 32 wm + 16 i + lr][c = 64 wn + 16 j + 4 lg + r]
    const int64_t rb = scene_row0 + (int64_t)(t_begin + t) * BMW;
    const int valid = (int)pcs_min64(BMW, scene_row0 + N - rb);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int m = wm * (BMW / 2) + i * 16 + lr;
      const bool ok = m < valid;
      uint32_t pk[4][2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // packed fp32 math (v_pk_fma_f32 / v_pk_add_f32) on column pairs
        f32x2 v2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 x = {acc[i][j][2 * h], acc[i][j][2 * h + 1]};
          v2[h] = __builtin_elementwise_fma(x, es2[j][h], et2[j][h]);
          v2[h][0] = relu(v2[h][0]);
          v2[h][1] = relu(v2[h][1]);
        }
        f32x2 d[2];   // the stored values, decoded
        if constexpr (C8) {
          const uint32_t w = pack4fp8(v2[0][0], v2[0][1], v2[1][0], v2[1][1]);
          pk[j][0] = w;
          d[0] = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false);
          d[1] = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
        } else {
          pk[j][0] = pack2bf(v2[0][0], v2[0][1]);
          pk[j][1] = pack2bf(v2[1][0], v2[1][1]);
#pragma unroll
          for (int h = 0; h < 2; ++h) d[h] = f32x2{bf2f(pk[j][h] & 0xffffu), bf2f(pk[j][h] >> 16)};
        }
        if (ok) {
          csum2[j][0] += d[0];
          csum2[j][1] += d[1];
        }
      }
      if constexpr (C8) {
        // -> this half's rows of stage t: row m, 16-B slot 4 wn + j (swizzled), dword lg
        char *st = lds + OFF_A + (t % NSTAGE) * A_BYTES + m * ROWB;
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<uint32_t *>(st + swz(m, 4 * wn + j) * 16 + 4 * lg) = pk[j][0];
        continue;
      }
      // v_permlane16_swap: lane groups 2h / 2h+1 trade tiles 2q / 2q+1, leaving each lane 8
      // consecutive columns of tile 2q + (lg & 1)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int hmax = C8 ? 1 : 2;
#pragma unroll
        for (int h = 0; h < hmax; ++h) {
          const auto sw = __builtin_amdgcn_permlane16_swap(pk[2 * q][h], pk[2 * q + 1][h], false, false);
          pk[2 * q][h] = sw[0];
          pk[2 * q + 1][h] = sw[1];
        }
        if constexpr (C8) {
          pend[i][q][0] = pk[2 * q][0];
          pend[i][q][1] = pk[2 * q + 1][0];
        } else {
          pend[i][q][0] = pk[2 * q][0]; pend[i][q][1] = pk[2 * q][1];
          pend[i][q][2] = pk[2 * q + 1][0]; pend[i][q][3] = pk[2 * q + 1][1];
        }
      }
    }
    pend_rb = rb;
    pend_valid = valid;
  }
  if constexpr (C8) {
    // the last tile's rows: the half's epilogue writes retire, then one barrier (half 0's
    // matches half 1's last loop barrier), then half 0 re-aligns with half 1's
    if (ntl > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier_raw();
      store_rows(ntl - 1);
    }
    if (wm == 0) barrier_raw();
  } else {
    if (wm == 0) barrier_raw();   // re-align the halves
    if (ntl > 0) store_pending();
  }
  wait_vm<0>();

  // ---- chunk end: column sums over the 16 lanes of each row group, then the two wave rows
  float *red = reinterpret_cast<float *>(lds + OFF_RED);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = dpp_sum16(csum2[j][r >> 1][r & 1]);
      if (lr == 0) red[wm * BNW + wn * 64 + j * 16 + 4 * lg + r] = s;
    }
  __syncthreads();
  if (a.stats && tid < BNW) {
    const int64_t o = (int64_t)chunk * Ncols + n0 + tid;
    *reinterpret_cast<float2 *>(a.stats + o * 2) = make_float2(red[tid] + red[BNW + tid], 0.f);
  }
}

}  // namespace

// Measured at cfg2 (tools/bench_conv5.py): fp8 store 4.0 ms here vs 4.9 ms on the
// register-staged kernel; bf16 store 5.4 vs 5.0 ms, so bf16 stays there (the pass is bound by
// the epilogue's vector work and the store issue, not by the MFMAs or the loads).
bool pcs_gemm_wres_applicable(const pcs_gemm_args &a) {
  if (a.dtype != PCS_BF16 || (a.flags & (PCS_FLAG_GENERIC | PCS_FLAG_NO_GLDS | PCS_FLAG_AW_FP8))) return false;
  if (!(a.flags & PCS_FLAG_C_FP8)) return false;
  return a.prologue == PCS_PRO_BNRELU && a.epilogue == PCS_EPI_BNRELU && a.K == K && a.Ncols % BNW == 0 &&
         !a.a_mask && a.C && a.es && a.et && !a.pool && !a.scene_bias && a.scene_rows * a.num_scenes < ((int64_t)1 << 31);
}

// geometry: the caller's chunks (multiples of 256 rows, pcs_gemm_geometry) in 128-row tiles
int pcs_gemm_wres_launch(const pcs_gemm_args &g, int64_t rows_per_chunk, hipStream_t s) {
  const int ncb = g.Ncols / BNW;
  const int nb = ncb * (int)(g.num_scenes * g.chunks_per_scene);
  const int tps = (int)((g.scene_rows + BMW - 1) / BMW);
  const int tpc = (int)(rows_per_chunk / BMW);
  if (g.flags & PCS_FLAG_C_FP8)
    hipLaunchKernelGGL((wres_bnrelu_kernel<true>), dim3(nb), dim3(THREADS), 0, s, g, tps, tpc, ncb);
  else
    hipLaunchKernelGGL((wres_bnrelu_kernel<false>), dim3(nb), dim3(THREADS), 0, s, g, tps, tpc, ncb);
  PCS_CHECK_LAUNCH();
  return 0;
}

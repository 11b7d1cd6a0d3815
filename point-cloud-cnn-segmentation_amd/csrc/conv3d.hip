// Dense 3-D convolution on channels-last voxel grids: the north star's "3x3x3 Conv3d U-Net with
// LDS-staged stencils, transposed conv" building blocks.  Build-defined: the
// reference (P) has no voxel grid, so parity is against torch.nn.functional.conv3d /
// conv_transpose3d in fp64 (tests/test_gpu_conv3d.py), not against the reference.
//
// Layouts: X [B, D, H, W, C] bf16 (channels innermost), W [Cout, k, k, k, Cin] bf16 (one row of
// taps x input channels per output channel), Y [B, D', H', W', Cout] f32 or bf16.
//   conv       Y[o] = b + sum_t W_t X[o s - p + t]
//   transposed Y[o] = b + sum_t W_t X[(o + p - t) / s]   (only where o + p - t is a multiple of s)
// The input gradient of one is the other with W_t transposed (pcs_conv3d_weight_t), so one
// kernel serves the forward and the input gradient of both; the weight gradient uses the
// forward's index map.
//
// conv3d_kernel: implicit GEMM, rows = output voxels, columns = output channels, k = (tap,
// 32-channel slice).  A k-step gathers the 64 rows' input voxels of one tap into LDS (zero rows
// off the grid or off the stride lattice): the 27-tap stencil is 27 shifted gathers of the same
// channels-last rows, so after the first tap the re-reads come from L2.  The next k-step is
// loaded into registers while the MFMAs of this one run; one barrier per k-step.
// conv3d_wgrad_kernel: dW_t = dY^T X_t over output voxels in 32-voxel k-steps, both operands
// staged row-major and read transposed (ds_read_b64_tr_b16) so the MFMA's k runs over voxels;
// split over voxel slices with fp32 partials summed in a fixed order (deterministic).
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int BN = 64, KS = 32;   // output channels per tile, k-step (bf16 elements)

// 16-B slot swizzle of a 64-B LDS row: conflict-free ds_read_b128 fragment reads (rows 4 apart
// land on different slots of a 256-B bank row)
PCS_DEV int cswz(int row, int slot) { return slot ^ ((-(row >> 2)) & 3); }

// input voxel feeding output voxel (b, z, y, x) through tap (dz, dy, dx); -1 = none (zero)
PCS_DEV int64_t in_voxel(const pcs_conv3d_geom &g, int b, int z, int y, int x, int dz, int dy, int dx) {
  int iz, iy, ix;
  if (!g.transposed) {
    iz = z * g.s - g.p + dz;
    iy = y * g.s - g.p + dy;
    ix = x * g.s - g.p + dx;
  } else {
    const int tz = z + g.p - dz, ty = y + g.p - dy, tx = x + g.p - dx;
    if (tz < 0 || ty < 0 || tx < 0) return -1;
    if (g.s == 2 && ((tz | ty | tx) & 1)) return -1;
    const int sh = g.s == 2 ? 1 : 0;
    iz = tz >> sh;
    iy = ty >> sh;
    ix = tx >> sh;
  }
  if (iz < 0 || iy < 0 || ix < 0 || iz >= g.Di || iy >= g.Hi || ix >= g.Wi) return -1;
  return (((int64_t)b * g.Di + iz) * g.Hi + iy) * g.Wi + ix;
}

// output voxel u -> (b, z, y, x); 32-bit divisions when u fits (a 64-bit division is ~10x dearer)
PCS_DEV void decode(const pcs_conv3d_geom &g, int64_t u, int &b, int &z, int &y, int &x) {
  if (u < ((int64_t)1 << 31)) {
    uint32_t v = (uint32_t)u;
    x = (int)(v % (uint32_t)g.Wo);
    v /= (uint32_t)g.Wo;
    y = (int)(v % (uint32_t)g.Ho);
    v /= (uint32_t)g.Ho;
    z = (int)(v % (uint32_t)g.Do);
    b = (int)(v / (uint32_t)g.Do);
    return;
  }
  x = (int)(u % g.Wo);
  u /= g.Wo;
  y = (int)(u % g.Ho);
  u /= g.Ho;
  z = (int)(u % g.Do);
  b = (int)(u / g.Do);
}

// Transposed form with stride 2: an output voxel o only meets the taps t with o + p - t even, so
// the outputs fall into 8 parity classes c (o = 2 o' + c per dimension), each with its own tap
// subset (t = (c + p) mod 2, + 2, ... < k: one tap per dimension for k = 2).  Tiles are cut per
// class, so no MFMA runs on a tap that is off the lattice for every row.
struct PClass {
  int cz, cy, cx;   // parity of the class
  int nz, ny, nx;   // class sub-grid (output voxels 2 o' + c inside the grid)
  int tz0, ty0, tx0, ntz, nty, ntx;   // first tap and tap count per dimension
};

PCS_DEV PClass pclass(const pcs_conv3d_geom &g, int c) {
  PClass q;
  q.cz = (c >> 2) & 1; q.cy = (c >> 1) & 1; q.cx = c & 1;
  q.nz = (g.Do - q.cz + 1) >> 1; q.ny = (g.Ho - q.cy + 1) >> 1; q.nx = (g.Wo - q.cx + 1) >> 1;
  q.tz0 = (q.cz + g.p) & 1; q.ty0 = (q.cy + g.p) & 1; q.tx0 = (q.cx + g.p) & 1;
  q.ntz = q.tz0 < g.k ? (g.k - q.tz0 + 1) >> 1 : 0;
  q.nty = q.ty0 < g.k ? (g.k - q.ty0 + 1) >> 1 : 0;
  q.ntx = q.tx0 < g.k ? (g.k - q.tx0 + 1) >> 1 : 0;
  return q;
}

// class row u (b, z', y', x' over the class sub-grid) -> output voxel (b, z, y, x)
PCS_DEV void decode_class(const PClass &q, int64_t u, int &b, int &z, int &y, int &x) {
  if (u < ((int64_t)1 << 31)) {
    uint32_t v = (uint32_t)u;
    x = 2 * (int)(v % (uint32_t)q.nx) + q.cx;
    v /= (uint32_t)q.nx;
    y = 2 * (int)(v % (uint32_t)q.ny) + q.cy;
    v /= (uint32_t)q.ny;
    z = 2 * (int)(v % (uint32_t)q.nz) + q.cz;
    b = (int)(v / (uint32_t)q.nz);
    return;
  }
  x = 2 * (int)(u % q.nx) + q.cx;
  u /= q.nx;
  y = 2 * (int)(u % q.ny) + q.cy;
  u /= q.ny;
  z = 2 * (int)(u % q.nz) + q.cz;
  b = (int)(u / q.nz);
}

// BMT = 64 or 128 output voxels per tile (4 waves as 2 x 2: wave tile BMT/2 x BNT/2); KST = 32 or
// 64 input channels per k-step (64: whole 128-B voxel rows per load, 2x the MFMAs per barrier);
// BNT = 64 or 32 output channels per tile (32: a 32-channel U-Net level without zero channels)
template <int BMT, int KST, bool OUT_BF16, int BNT = BN>
__global__ __launch_bounds__(THREADS) void conv3d_kernel(pcs_conv3d_geom g, const bf16_t *__restrict__ X,
                                                         const bf16_t *__restrict__ W, const float *__restrict__ bias,
                                                         void *__restrict__ Y, int64_t M) {
  constexpr int RB = KST * 2;          // LDS row bytes
  constexpr int CPR = KST / 8;         // 16-B chunks per row
  constexpr int RPP = THREADS / CPR;   // rows staged per pass
  constexpr int HA = BMT / RPP, HB = (BNT + RPP - 1) / RPP;   // (BNT < RPP: the first BNT rows' threads)
  constexpr int TI = BMT / 32;         // 16-row MFMA tiles per wave
  constexpr int TJ = BNT / 32;         // 16-channel MFMA tiles per wave
  constexpr int KK = KST / 32;         // MFMA k-steps per k-step
  __shared__ __attribute__((aligned(16))) char lds[2][(BMT + BNT) * RB];   // per buffer: A | B
  auto swzf = [](int row, int slot) { return KST == 32 ? cswz(row, slot) : (slot ^ ((row >> 1) & 7)); };
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  // class mode (transposed, stride 2): blockIdx.x = tile * 8 + class, rows index the class sub-grid
  const bool cm = g.transposed && g.s == 2;
  PClass pc{};
  int64_t Mrows = M;
  int64_t m0 = (int64_t)blockIdx.x * BMT;
  if (cm) {
    pc = pclass(g, blockIdx.x & 7);
    Mrows = g.B * pc.nz * pc.ny * pc.nx;
    m0 = (int64_t)(blockIdx.x >> 3) * BMT;
    if (m0 >= Mrows) return;   // uniform: this class has fewer tiles than the largest
  }
  const int n0 = blockIdx.y * BNT;
  const int srow = tid / CPR, q = tid % CPR;   // staging: chunk q of rows srow + RPP h
  bool rv[HA];
  int vb[HA], vz[HA], vy[HA], vx[HA];
#pragma unroll
  for (int h = 0; h < HA; ++h) {
    const int64_t u = m0 + srow + RPP * h;
    rv[h] = u < Mrows;
    vb[h] = vz[h] = vy[h] = vx[h] = 0;
    if (rv[h]) {
      if (cm) decode_class(pc, u, vb[h], vz[h], vy[h], vx[h]);
      else decode(g, u, vb[h], vz[h], vy[h], vx[h]);
    }
  }
  const int k = g.k, taps = k * k * k, cps = g.Cin / KST;
  const int ctaps = cm ? pc.ntz * pc.nty * pc.ntx : taps;   // taps this tile runs
  const int nks = ctaps * cps;
  const bf16_t *wrow = W + (int64_t)(n0 + srow) * taps * g.Cin + q * 8;
  const int64_t wstep = (int64_t)RPP * taps * g.Cin;

  u32x4 ra[HA], rb[HB];
  auto load = [&](int ks) {
    const int j = ks / cps, c0 = (ks - j * cps) * KST;
    int dz, dy, dx;
    if (cm) {
      dz = pc.tz0 + 2 * (j / (pc.nty * pc.ntx));
      dy = pc.ty0 + 2 * ((j / pc.ntx) % pc.nty);
      dx = pc.tx0 + 2 * (j % pc.ntx);
    } else {
      dz = j / (k * k); dy = (j / k) % k; dx = j % k;
    }
    const int t = (dz * k + dy) * k + dx;
#pragma unroll
    for (int h = 0; h < HA; ++h) {
      const int64_t iv = rv[h] ? in_voxel(g, vb[h], vz[h], vy[h], vx[h], dz, dy, dx) : -1;
      ra[h] = iv >= 0 ? *reinterpret_cast<const u32x4 *>(X + iv * g.Cin + c0 + q * 8) : mk_u32x4(0, 0, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < HB; ++h)
      if (srow + RPP * h < BNT) rb[h] = *reinterpret_cast<const u32x4 *>(wrow + h * wstep + (int64_t)t * g.Cin + c0);
  };
  auto stage = [&](int buf) {
    char *tA = lds[buf], *tB = lds[buf] + BMT * RB;
#pragma unroll
    for (int h = 0; h < HA; ++h) {
      const int r = srow + RPP * h;
      *reinterpret_cast<u32x4 *>(tA + r * RB + swzf(r, q) * 16) = ra[h];
    }
#pragma unroll
    for (int h = 0; h < HB; ++h) {
      const int r = srow + RPP * h;
      if (r < BNT) *reinterpret_cast<u32x4 *>(tB + r * RB + swzf(r, q) * 16) = rb[h];
    }
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nks > 0) {
    load(0);
    stage(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(ks + 1);
    const char *tA = lds[buf], *tB = lds[buf] + BMT * RB;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 af[TI], bw[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wr * (BMT / 2) + i * 16 + lr;
        af[i] = *reinterpret_cast<const bf16x8 *>(tA + r * RB + swzf(r, kk * 4 + lg) * 16);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wc * (BNT / 2) + j * 16 + lr;
        bw[j] = *reinterpret_cast<const bf16x8 *>(tB + r * RB + swzf(r, kk * 4 + lg) * 16);
      }
      // W rows as the MFMA A operand: each lane ends with 4 consecutive output channels of one voxel
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nks) stage(buf ^ 1);   // buf ^ 1 was last read before the previous barrier
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TI; ++i) {
    int64_t uo = m0 + wr * (BMT / 2) + i * 16 + lr;
    if (uo >= Mrows) continue;
    if (cm) {   // class row -> output voxel
      int ob, oz, oy, ox;
      decode_class(pc, uo, ob, oz, oy, ox);
      uo = (((int64_t)ob * g.Do + oz) * g.Ho + oy) * g.Wo + ox;
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int co = n0 + wc * (BNT / 2) + j * 16 + 4 * lg;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
        const float4 bb = *reinterpret_cast<const float4 *>(bias + co);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      }
      if constexpr (OUT_BF16) {
        *reinterpret_cast<uint2 *>(reinterpret_cast<bf16_t *>(Y) + uo * g.Cout + co) =
            make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
      } else {
        *reinterpret_cast<float4 *>(reinterpret_cast<float *>(Y) + uo * g.Cout + co) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// ---- 3x3x3 stride-1 stencil (both forms) with the input block's halo staged in LDS once per
// CS-channel slice (CS = 64, or 32 for a 32-channel level): a 4 x 4 x 8 block of output voxels
// reads its 6 x 6 x 10 input halo (360 voxel rows) from L2 once and every tap's A operand from
// LDS at a shifted row, instead of 27 gathers; the 27 taps' NT x CS weight tiles (NT = 64 or 32
// output channels) stream through a double buffer.  The LDS images keep 128-B rows whatever CS
// (a 32-channel slice fills the first four swizzled slots of a row).
constexpr int SZ = 4, SY = 4, SX = 8;                      // output block: 128 voxels
constexpr int GZ = SZ + 2, GY = SY + 2, GX = SX + 2;
constexpr int HROWS = GZ * GY * GX;                        // 360 halo voxels
constexpr int HIMG = HROWS * 128, WTILE = 64 * 128;        // halo image (64 ch), one tap's W tile

PCS_DEV int swz8(int row, int ch) { return ch ^ ((row >> 1) & 7); }

template <int CS, int NT, bool OUT_BF16>
__global__ __launch_bounds__(THREADS) void stencil3_kernel(pcs_conv3d_geom g, const bf16_t *__restrict__ X,
                                                           const bf16_t *__restrict__ W, const float *__restrict__ bias,
                                                           void *__restrict__ Y) {
  __shared__ __attribute__((aligned(16))) char lds[HIMG + 2 * WTILE];   // 45 KB + 16 KB
  char *halo = lds, *wt = lds + HIMG;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  const int nbx = (g.Wo + SX - 1) / SX, nby = (g.Ho + SY - 1) / SY, nbz = (g.Do + SZ - 1) / SZ;
  uint32_t bid = blockIdx.x;
  const int bx = (int)(bid % nbx); bid /= nbx;
  const int by = (int)(bid % nby); bid /= nby;
  const int bz = (int)(bid % nbz);
  const int b = (int)(bid / nbz);
  const int oz0 = bz * SZ, oy0 = by * SY, ox0 = bx * SX;
  const bool tr = g.transposed;
  // first halo voxel: conv reads o - p + t, the transposed form o + p - t (t = 0..2)
  const int hz0 = tr ? oz0 + g.p - 2 : oz0 - g.p, hy0 = tr ? oy0 + g.p - 2 : oy0 - g.p,
            hx0 = tr ? ox0 + g.p - 2 : ox0 - g.p;
  constexpr int CCH = CS / 8;                 // 16-B chunks per staged row
  constexpr int WCH = NT * CCH;               // W tile chunks
  constexpr int HW = (WCH + THREADS - 1) / THREADS;
  constexpr int TJ = NT / 32, KK = CS / 32;
  const int n0 = blockIdx.y * NT, Cin = g.Cin, cps = Cin / CS;
  // wave tile: output rows wr*64 .. +64 (4 MFMA tiles), channels wc*NT/2 ..; row r = (rz, ry, rx)
  int hrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wr * 64 + i * 16 + lr;
    hrow[i] = ((r >> 5) * GY + ((r >> 3) & 3)) * GX + (r & 7);
  }
  u32x4 rw[HW];   // W staging: NT rows x CCH chunks
  auto loadw = [&](int t, int c0) {
#pragma unroll
    for (int h = 0; h < HW; ++h) {
      const int c = tid + THREADS * h, row = c / CCH, ch = c % CCH;
      if (c < WCH) rw[h] = *reinterpret_cast<const u32x4 *>(W + ((int64_t)(n0 + row) * 27 + t) * Cin + c0 + ch * 8);
    }
  };
  auto stagew = [&](int buf) {
#pragma unroll
    for (int h = 0; h < HW; ++h) {
      const int c = tid + THREADS * h, row = c / CCH, ch = c % CCH;
      if (c < WCH) *reinterpret_cast<u32x4 *>(wt + buf * WTILE + row * 128 + swz8(row, ch) * 16) = rw[h];
    }
  };
  f32x4 acc[4][TJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int cs = 0; cs < cps; ++cs) {
    const int c0 = cs * CS;
    __syncthreads();   // the previous slice's halo and W reads are done
    for (int c = tid; c < HROWS * CCH; c += THREADS) {
      const int hr = c / CCH, ch = c % CCH;
      const int hx = hr % GX, hy = (hr / GX) % GY, hz = hr / (GX * GY);
      const int iz = hz0 + hz, iy = hy0 + hy, ix = hx0 + hx;
      u32x4 v = mk_u32x4(0, 0, 0, 0);
      if (iz >= 0 && iy >= 0 && ix >= 0 && iz < g.Di && iy < g.Hi && ix < g.Wi)
        v = *reinterpret_cast<const u32x4 *>(X + ((((int64_t)b * g.Di + iz) * g.Hi + iy) * g.Wi + ix) * Cin + c0 + ch * 8);
      *reinterpret_cast<u32x4 *>(halo + hr * 128 + swz8(hr, ch) * 16) = v;
    }
    loadw(0, c0);
    stagew(0);
    __syncthreads();
    for (int t = 0; t < 27; ++t) {
      const int buf = t & 1;
      if (t + 1 < 27) loadw(t + 1, c0);
      const int dz = t / 9, dy = (t / 3) % 3, dx = t % 3;
      const int hoff = tr ? ((2 - dz) * GY + (2 - dy)) * GX + (2 - dx) : (dz * GY + dy) * GX + dx;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        bf16x8 af[4], bw[TJ];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int h = hrow[i] + hoff;
          af[i] = *reinterpret_cast<const bf16x8 *>(halo + h * 128 + swz8(h, kk * 4 + lg) * 16);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int r = wc * (NT / 2) + j * 16 + lr;
          bw[j] = *reinterpret_cast<const bf16x8 *>(wt + buf * WTILE + r * 128 + swz8(r, kk * 4 + lg) * 16);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
      }
      if (t + 1 < 27) stagew(buf ^ 1);   // buf ^ 1 was last read before the previous barrier
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wr * 64 + i * 16 + lr;
    const int oz = oz0 + (r >> 5), oy = oy0 + ((r >> 3) & 3), ox = ox0 + (r & 7);
    if (oz >= g.Do || oy >= g.Ho || ox >= g.Wo) continue;
    const int64_t uo = (((int64_t)b * g.Do + oz) * g.Ho + oy) * g.Wo + ox;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int co = n0 + wc * (NT / 2) + j * 16 + 4 * lg;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
        const float4 bb = *reinterpret_cast<const float4 *>(bias + co);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      }
      if constexpr (OUT_BF16) {
        *reinterpret_cast<uint2 *>(reinterpret_cast<bf16_t *>(Y) + uo * g.Cout + co) =
            make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
      } else {
        *reinterpret_cast<float4 *>(reinterpret_cast<float *>(Y) + uo * g.Cout + co) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// ---- weight gradient: dW[co][t][ci] = sum_o dY[o][co] X[in(o, t)][ci], one (co, ci) 64x64 tile
// of one tap per workgroup and voxel slice.  Both operands are staged row-major ([32 voxels][64
// channels], whole 128-B rows, double-buffered) and read as MFMA operands with k over voxels by
// ds_read_b64_tr_b16 (4 voxels x 16 channels per 16-lane group, delivered column-major)
constexpr int WV = 32;   // voxels per k-step
constexpr int WIMG = WV * 128;   // one [32][64] bf16 image

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 16-B chunk swizzle of image row r (even values: a 32-B pair of chunks stays adjacent): the
// eight rows a 32-lane half reads (8g + 4h + q, two groups) land on distinct 32-B bank slots
PCS_DEV int wsw(int r) { return 2 * (((r >> 1) & 1) | ((r >> 2) & 2)); }
PCS_DEV int woff(int r, int byte) { return r * 128 + ((((byte >> 4) ^ wsw(r)) << 4) | (byte & 15)); }

// MFMA operand rows = channels cb .. cb+15 (lane & 15), k = voxels 8 (lane >> 4) .. + 8
PCS_DEV bf16x8 wfrag(const char *img, int cb, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int byte = (cb + 4 * (i & 3)) * 2;   // this lane supplies row 8g (+4) + i/4, columns cb + 4 (i%4)
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + woff(8 * g + (i >> 2), byte)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + woff(8 * g + 4 + (i >> 2), byte)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// One workgroup covers the dx taps of one (dz, dy) (all k of them, sharing the dY image; one tap
// in class mode, where the dx taps meet different voxel sets)
constexpr int TG = 3;

// COT x CIT = the workgroup's (co, ci) tile, 64 or 32 each (a 32-channel level stages half rows)
template <int COT, int CIT>
__global__ __launch_bounds__(THREADS) void conv3d_wgrad_kernel(pcs_conv3d_geom g, const bf16_t *__restrict__ X,
                                                               const bf16_t *__restrict__ dY, float *__restrict__ ws,
                                                               int64_t M, int64_t vps) {
  __shared__ __attribute__((aligned(16))) char lds[2][(1 + TG) * WIMG];   // per buffer: dY | X per dx tap
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  constexpr int NI = COT / 32, NJ = CIT / 32;   // 16-channel MFMA tiles per wave (co, ci)
  const int nco = g.Cout / COT;
  const int co0 = (blockIdx.x % nco) * COT, ci0 = (blockIdx.x / nco) * CIT;
  const int split = blockIdx.z;
  const int k = g.k, taps = k * k * k;
  // transposed, stride 2: tap t only meets the output voxels of parity class (t + p) mod 2, so
  // the slices run over that class's sub-grid, one tap per workgroup
  const bool cm = g.transposed && g.s == 2;
  int dz, dy, dx0, ntg;
  if (cm) {
    const int t = blockIdx.y;
    dz = t / (k * k); dy = (t / k) % k; dx0 = t % k; ntg = 1;
  } else {
    dz = blockIdx.y / k; dy = blockIdx.y % k; dx0 = 0; ntg = k;
  }
  PClass pc{};
  int64_t Mv = M, vs = vps;
  if (cm) {
    pc = pclass(g, (((dz + g.p) & 1) << 2) | (((dy + g.p) & 1) << 1) | ((dx0 + g.p) & 1));
    Mv = g.B * pc.nz * pc.ny * pc.nx;
    vs = ((Mv + gridDim.z - 1) / gridDim.z + WV - 1) / WV * WV;
  }
  const int64_t lo = (int64_t)split * vs, hi = pcs_min64(lo + vs, Mv);
  const int sv = tid >> 3, q8 = tid & 7;   // staging: voxel row sv, 16-B chunk q8 (channels 8 q8 ..)

  f32x4 acc[TG][NI][NJ];
#pragma unroll
  for (int a = 0; a < TG; ++a)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[a][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the next k-step's rows are loaded into registers while this one's MFMAs run
  u32x4 rd, rx[TG];
  auto load = [&](int64_t v0) {
    const int64_t u = v0 + sv;
    rd = mk_u32x4(0, 0, 0, 0);
#pragma unroll
    for (int a = 0; a < TG; ++a) rx[a] = mk_u32x4(0, 0, 0, 0);
    if (u < hi) {
      int b, z, y, x;
      int64_t uo = u;
      if (cm) {
        decode_class(pc, u, b, z, y, x);
        uo = (((int64_t)b * g.Do + z) * g.Ho + y) * g.Wo + x;
      } else {
        decode(g, u, b, z, y, x);
      }
      if (q8 < COT / 8) rd = *reinterpret_cast<const u32x4 *>(dY + uo * g.Cout + co0 + q8 * 8);
#pragma unroll
      for (int a = 0; a < TG; ++a) {
        if (a < ntg) {
          const int64_t iv = in_voxel(g, b, z, y, x, dz, dy, dx0 + a);
          if (iv >= 0 && q8 < CIT / 8) rx[a] = *reinterpret_cast<const u32x4 *>(X + iv * g.Cin + ci0 + q8 * 8);
        }
      }
    }
  };
  auto stage = [&](int buf) {
    *reinterpret_cast<u32x4 *>(lds[buf] + woff(sv, q8 * 16)) = rd;
#pragma unroll
    for (int a = 0; a < TG; ++a)
      if (a < ntg) *reinterpret_cast<u32x4 *>(lds[buf] + (1 + a) * WIMG + woff(sv, q8 * 16)) = rx[a];
  };
  const int nks = (int)((hi - lo + WV - 1) / WV);   // uniform; 0 for an empty slice
  if (nks > 0) {
    load(lo);
    stage(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(lo + (int64_t)(ks + 1) * WV);
    bf16x8 fd[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) fd[i] = wfrag(lds[buf], wr * (COT / 2) + i * 16, lane);
#pragma unroll
    for (int a = 0; a < TG; ++a) {
      if (a < ntg) {   // uniform
        bf16x8 fx[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) fx[j] = wfrag(lds[buf] + (1 + a) * WIMG, wc * (CIT / 2) + j * 16, lane);
        // lane: dW rows co = 4 lg + v of tile i, column ci = lr of tile j
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[a][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx[j], acc[a][i][j], 0, 0, 0);
      }
    }
    if (ks + 1 < nks) stage(buf ^ 1);   // buf ^ 1 was last read before the previous barrier
    __syncthreads();
  }
  float *out = ws + (int64_t)split * g.Cout * taps * g.Cin;
#pragma unroll
  for (int a = 0; a < TG; ++a) {
    if (a >= ntg) continue;
    const int t = (dz * k + dy) * k + dx0 + a;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int ci = ci0 + wc * (CIT / 2) + j * 16 + lr;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int co = co0 + wr * (COT / 2) + i * 16 + 4 * lg + v;
          out[((int64_t)co * taps + t) * g.Cin + ci] = acc[a][i][j][v];
        }
      }
  }
}

// ---- weight gradient of the 3x3x3 stride-1 stencil (both forms) on halo tiles: a workgroup owns
// one (64 co x 64 ci) tile and one dz (9 taps, 144 accumulator VGPRs) and walks a range of 4 x 4 x 8
// output blocks; per block it stages the block's dY rows [128][64] and the 4 input planes of the
// halo it meets at this dz [4][6][10][64] once, and every tap's operand is a shifted set of halo
// rows read transposed (k over the block's voxels)
constexpr int XPL = SZ * GY * GX;   // 240 halo rows of one dz

template <int COT, int CIT>   // the (co, ci) tile: 64 or 32 each
__global__ __launch_bounds__(THREADS) void stencil3_wgrad_kernel(pcs_conv3d_geom g, const bf16_t *__restrict__ X,
                                                                 const bf16_t *__restrict__ dY, float *__restrict__ ws,
                                                                 int64_t nblk, int64_t bps) {
  __shared__ __attribute__((aligned(16))) char lds[(128 + XPL) * 128];   // dY image | halo planes (46 KB)
  char *dimg = lds, *ximg = lds + 128 * 128;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  constexpr int NI = COT / 32, NJ = CIT / 32;   // 16-channel MFMA tiles per wave (co, ci)
  const int nco = g.Cout / COT;
  const int co0 = (blockIdx.x % nco) * COT, ci0 = (blockIdx.x / nco) * CIT;
  const int dz = blockIdx.y, split = blockIdx.z;
  const bool tr = g.transposed;
  const int zoff = tr ? 2 - dz : dz;
  const int nbx = (g.Wo + SX - 1) / SX, nby = (g.Ho + SY - 1) / SY, nbz = (g.Do + SZ - 1) / SZ;
  const int64_t b0 = (int64_t)split * bps, b1 = pcs_min64(b0 + bps, nblk);
  // transposed operand read: rows = 16 channels from cb (lane & 15), k = 8 voxels from 8 (lane >> 4)
  // (4 per ds_read_b64_tr_b16); row_of(k) gives the image row of block voxel k
  auto trfrag = [&](const char *img, int cb, int kb, int dyo, int dxo, bool halo) {
    const int gq = lane >> 4, i = lane & 15;
    const int byte = (cb + 4 * (i & 3)) * 2;
    s16x4 part[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = kb + 8 * gq + 4 * h + (i >> 2);   // block voxel
      const int row = halo ? (((r >> 5) * GY + ((r >> 3) & 3) + dyo) * GX + (r & 7) + dxo) : r;
      part[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4 *)(img + row * 128 + ((((byte >> 4) ^ ((row >> 1) & 7)) << 4) | (byte & 15))));
    }
    const s16x8 v = {part[0][0], part[0][1], part[0][2], part[0][3], part[1][0], part[1][1], part[1][2], part[1][3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  f32x4 acc[9][NI][NJ];
#pragma unroll
  for (int a = 0; a < 9; ++a)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[a][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t blk = b0; blk < b1; ++blk) {
    uint32_t q = (uint32_t)blk;
    const int bx = (int)(q % nbx); q /= nbx;
    const int by = (int)(q % nby); q /= nby;
    const int bz = (int)(q % nbz);
    const int b = (int)(q / nbz);
    const int oz0 = bz * SZ, oy0 = by * SY, ox0 = bx * SX;
    const int hz0 = (tr ? oz0 + g.p - 2 : oz0 - g.p) + zoff, hy0 = tr ? oy0 + g.p - 2 : oy0 - g.p,
              hx0 = tr ? ox0 + g.p - 2 : ox0 - g.p;
    __syncthreads();   // the previous block's reads are done
    for (int c = tid; c < 128 * (COT / 8); c += THREADS) {   // dY rows of the block (zero outside the grid)
      const int r = c / (COT / 8), ch = c % (COT / 8);
      const int oz = oz0 + (r >> 5), oy = oy0 + ((r >> 3) & 3), ox = ox0 + (r & 7);
      u32x4 v = mk_u32x4(0, 0, 0, 0);
      if (oz < g.Do && oy < g.Ho && ox < g.Wo)
        v = *reinterpret_cast<const u32x4 *>(dY + ((((int64_t)b * g.Do + oz) * g.Ho + oy) * g.Wo + ox) * g.Cout + co0 + ch * 8);
      *reinterpret_cast<u32x4 *>(dimg + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4)) = v;
    }
    for (int c = tid; c < XPL * (CIT / 8); c += THREADS) {   // the 4 halo planes of this dz
      const int hr = c / (CIT / 8), ch = c % (CIT / 8);
      const int hx = hr % GX, hy = (hr / GX) % GY, hz = hr / (GX * GY);
      const int iz = hz0 + hz, iy = hy0 + hy, ix = hx0 + hx;
      u32x4 v = mk_u32x4(0, 0, 0, 0);
      if (iz >= 0 && iy >= 0 && ix >= 0 && iz < g.Di && iy < g.Hi && ix < g.Wi)
        v = *reinterpret_cast<const u32x4 *>(X + ((((int64_t)b * g.Di + iz) * g.Hi + iy) * g.Wi + ix) * g.Cin + ci0 + ch * 8);
      *reinterpret_cast<u32x4 *>(ximg + hr * 128 + ((ch ^ ((hr >> 1) & 7)) << 4)) = v;
    }
    __syncthreads();
#pragma unroll 1
    for (int kb = 0; kb < 128; kb += 32) {   // 32 block voxels per MFMA k-step
      bf16x8 fd[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) fd[i] = trfrag(dimg, wr * (COT / 2) + i * 16, kb, 0, 0, false);
#pragma unroll
      for (int a = 0; a < 9; ++a) {
        const int ty = a / 3, tx = a % 3;
        const int dyo = tr ? 2 - ty : ty, dxo = tr ? 2 - tx : tx;
        bf16x8 fx[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) fx[j] = trfrag(ximg, wc * (CIT / 2) + j * 16, kb, dyo, dxo, true);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[a][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx[j], acc[a][i][j], 0, 0, 0);
      }
    }
  }
  float *out = ws + (int64_t)split * g.Cout * 27 * g.Cin;
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    const int t = dz * 9 + a;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int ci = ci0 + wc * (CIT / 2) + j * 16 + lr;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int co = co0 + wr * (COT / 2) + i * 16 + 4 * lg + v;
          out[((int64_t)co * 27 + t) * g.Cin + ci] = acc[a][i][j][v];
        }
      }
  }
}

// db partials: column sums of dY over one voxel slice, [split][Cout]; a thread sums 8 channels
// (one 16-B chunk) of every 32nd row, then the 32 row groups are added in LDS in a fixed order
// (64 channels per workgroup; the last one of a 32-channel multiple runs half)
__global__ __launch_bounds__(THREADS) void conv3d_bgrad_kernel(const bf16_t *__restrict__ dY, int Cout, int64_t M,
                                                               int64_t vps, float *__restrict__ wsb) {
  __shared__ float red[32][64];
  const int ch = threadIdx.x & 7, rg = threadIdx.x >> 3;   // channels c0 + 8 ch .., row group 0..31
  const int c0 = blockIdx.x * 64;
  const int64_t lo = (int64_t)blockIdx.y * vps, hi = pcs_min64(lo + vps, M);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool cv = c0 + ch * 8 < Cout;
  for (int64_t u = cv ? lo + rg : hi; u < hi; u += 32) {
    float v[8];
    unpack_chunk(*reinterpret_cast<const u32x4 *>(dY + u * Cout + c0 + ch * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += v[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rg][ch * 8 + e] = s[e];
  __syncthreads();
  if (threadIdx.x < 64 && c0 + (int)threadIdx.x < Cout) {
    float t = 0.f;
    for (int r = 0; r < 32; ++r) t += red[r][threadIdx.x];
    wsb[(int64_t)blockIdx.y * Cout + c0 + threadIdx.x] = t;
  }
}

// out[i] = sum_s part[s * len + i], fixed order
__global__ __launch_bounds__(256) void conv3d_reduce_kernel(const float *__restrict__ part, int64_t nsl, int64_t len,
                                                            float *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= len) return;
  float s = 0.f;
  for (int64_t sl = 0; sl < nsl; ++sl) s += part[sl * len + i];
  out[i] = s;
}

__global__ __launch_bounds__(256) void conv3d_weight_t_kernel(const bf16_t *__restrict__ W, int Cout, int taps, int Cin,
                                                              bf16_t *__restrict__ Wt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // index into Wt [Cin][taps][Cout]
  const int64_t n = (int64_t)Cout * taps * Cin;
  if (i >= n) return;
  const int co = (int)(i % Cout);
  const int64_t r = i / Cout;
  const int t = (int)(r % taps), ci = (int)(r / taps);
  Wt[i] = W[((int64_t)co * taps + t) * Cin + ci];
}

// ---- submanifold sparse convolution on occupied voxels (the north star's hash-indexed gather,
// BASELINE configs[2]): the rows are the occupied voxels, the input row of (row m, tap t) comes
// from the neighbour map nbr[m][t] (-1: an empty site, zeros) built by pcs_sparse_neighbors.  The
// same gather GEMM as conv3d_kernel; a tile runs only the taps some of its rows have a neighbour
// at (a bit mask collected in LDS first), which is where the sparsity saves MFMA work.
//   Y[m] = b + sum_t W[tw(t)] X[nbr[m][t]],  tw(t) = flip ? taps - 1 - t : t
// With flip and W^T (pcs_conv3d_weight_t) this is the input gradient: offset(taps-1-t) =
// -offset(t) for the centred 3x3x3 taps, so dX[n] = sum_t W_t^T dY[nbr[n][taps-1-t]].
template <int BMT, int KST, bool OUT_BF16>
__global__ __launch_bounds__(THREADS) void sparse_conv_kernel(const int32_t *__restrict__ nbr, int64_t M, int taps,
                                                              const bf16_t *__restrict__ X, int Cin,
                                                              const bf16_t *__restrict__ W, int Cout,
                                                              const float *__restrict__ bias, void *__restrict__ Y,
                                                              int flip) {
  constexpr int RB = KST * 2;
  constexpr int CPR = KST / 8;
  constexpr int RPP = THREADS / CPR;
  constexpr int HA = BMT / RPP, HB = BN / RPP;
  constexpr int TI = BMT / 32;
  constexpr int KK = KST / 32;
  __shared__ __attribute__((aligned(16))) char lds[2][(BMT + BN) * RB];
  __shared__ uint32_t tmask;
  __shared__ int tlist[32];
  __shared__ int ntl;
  auto swzf = [](int row, int slot) { return KST == 32 ? cswz(row, slot) : (slot ^ ((row >> 1) & 7)); };
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * BMT;
  const int n0 = blockIdx.y * BN;
  const int srow = tid / CPR, q = tid % CPR;

  // the taps this tile meets
  if (tid == 0) tmask = 0u;
  __syncthreads();
  uint32_t mym = 0u;
  for (int i = tid; i < BMT * taps; i += THREADS) {
    const int r = i / taps, t = i - r * taps;
    if (m0 + r < M && nbr[(m0 + r) * taps + t] >= 0) mym |= 1u << t;
  }
  if (mym) atomicOr(&tmask, mym);
  __syncthreads();
  if (tid == 0) {
    int c = 0;
    const uint32_t m = tmask;
    for (int t = 0; t < taps; ++t)
      if ((m >> t) & 1u) tlist[c++] = t;
    ntl = c;
  }
  __syncthreads();
  const int cps = Cin / KST;
  const int nks = ntl * cps;
  const bf16_t *wrow = W + (int64_t)(n0 + srow) * taps * Cin + q * 8;
  const int64_t wstep = (int64_t)RPP * taps * Cin;

  u32x4 ra[HA], rb[HB];
  auto load = [&](int ks) {
    const int j = ks / cps, c0 = (ks - j * cps) * KST;
    const int t = tlist[j], tw = flip ? taps - 1 - t : t;
#pragma unroll
    for (int h = 0; h < HA; ++h) {
      const int64_t u = m0 + srow + RPP * h;
      const int iv = u < M ? nbr[u * taps + t] : -1;
      ra[h] = iv >= 0 ? *reinterpret_cast<const u32x4 *>(X + (int64_t)iv * Cin + c0 + q * 8) : mk_u32x4(0, 0, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < HB; ++h) rb[h] = *reinterpret_cast<const u32x4 *>(wrow + h * wstep + (int64_t)tw * Cin + c0);
  };
  auto stage = [&](int buf) {
    char *tA = lds[buf], *tB = lds[buf] + BMT * RB;
#pragma unroll
    for (int h = 0; h < HA; ++h) {
      const int r = srow + RPP * h;
      *reinterpret_cast<u32x4 *>(tA + r * RB + swzf(r, q) * 16) = ra[h];
    }
#pragma unroll
    for (int h = 0; h < HB; ++h) {
      const int r = srow + RPP * h;
      *reinterpret_cast<u32x4 *>(tB + r * RB + swzf(r, q) * 16) = rb[h];
    }
  };

  f32x4 acc[TI][2];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nks > 0) {
    load(0);
    stage(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(ks + 1);
    const char *tA = lds[buf], *tB = lds[buf] + BMT * RB;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 af[TI], bw[2];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wr * (BMT / 2) + i * 16 + lr;
        af[i] = *reinterpret_cast<const bf16x8 *>(tA + r * RB + swzf(r, kk * 4 + lg) * 16);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wc * 32 + j * 16 + lr;
        bw[j] = *reinterpret_cast<const bf16x8 *>(tB + r * RB + swzf(r, kk * 4 + lg) * 16);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nks) stage(buf ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int64_t uo = m0 + wr * (BMT / 2) + i * 16 + lr;
    if (uo >= M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = n0 + wc * 32 + j * 16 + 4 * lg;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
        const float4 bb = *reinterpret_cast<const float4 *>(bias + co);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      }
      if constexpr (OUT_BF16) {
        *reinterpret_cast<uint2 *>(reinterpret_cast<bf16_t *>(Y) + uo * Cout + co) =
            make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
      } else {
        *reinterpret_cast<float4 *>(reinterpret_cast<float *>(Y) + uo * Cout + co) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// weight gradient of the sparse convolution: dW[co][t][ci] = sum_m dY[m][co] X[nbr[m][t]][ci];
// a workgroup owns a (64 co x 64 ci) tile, TG consecutive taps and a slice of rows (the
// structure of conv3d_wgrad_kernel with the neighbour map as the index), partials per slice
__global__ __launch_bounds__(THREADS) void sparse_wgrad_kernel(const int32_t *__restrict__ nbr, int64_t M, int taps,
                                                               const bf16_t *__restrict__ X, int Cin,
                                                               const bf16_t *__restrict__ dY, int Cout,
                                                               float *__restrict__ ws, int64_t vps) {
  __shared__ __attribute__((aligned(16))) char lds[2][(1 + TG) * WIMG];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  const int nco = Cout / 64;
  const int co0 = (blockIdx.x % nco) * 64, ci0 = (blockIdx.x / nco) * 64;
  const int t0 = blockIdx.y * TG, ntg = min(TG, taps - t0);
  const int64_t lo = (int64_t)blockIdx.z * vps, hi = pcs_min64(lo + vps, M);
  const int sv = tid >> 3, q8 = tid & 7;

  f32x4 acc[TG][2][2];
#pragma unroll
  for (int a = 0; a < TG; ++a)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[a][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 rd, rx[TG];
  auto load = [&](int64_t v0) {
    const int64_t u = v0 + sv;
    rd = mk_u32x4(0, 0, 0, 0);
#pragma unroll
    for (int a = 0; a < TG; ++a) rx[a] = mk_u32x4(0, 0, 0, 0);
    if (u < hi) {
      rd = *reinterpret_cast<const u32x4 *>(dY + u * Cout + co0 + q8 * 8);
#pragma unroll
      for (int a = 0; a < TG; ++a) {
        if (a < ntg) {
          const int iv = nbr[u * taps + t0 + a];
          if (iv >= 0) rx[a] = *reinterpret_cast<const u32x4 *>(X + (int64_t)iv * Cin + ci0 + q8 * 8);
        }
      }
    }
  };
  auto stage = [&](int buf) {
    *reinterpret_cast<u32x4 *>(lds[buf] + woff(sv, q8 * 16)) = rd;
#pragma unroll
    for (int a = 0; a < TG; ++a)
      if (a < ntg) *reinterpret_cast<u32x4 *>(lds[buf] + (1 + a) * WIMG + woff(sv, q8 * 16)) = rx[a];
  };
  const int nks = (int)((hi - lo + WV - 1) / WV);
  if (nks > 0) {
    load(lo);
    stage(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(lo + (int64_t)(ks + 1) * WV);
    bf16x8 fd[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fd[i] = wfrag(lds[buf], wr * 32 + i * 16, lane);
#pragma unroll
    for (int a = 0; a < TG; ++a) {
      if (a < ntg) {
        bf16x8 fx[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) fx[j] = wfrag(lds[buf] + (1 + a) * WIMG, wc * 32 + j * 16, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[a][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx[j], acc[a][i][j], 0, 0, 0);
      }
    }
    if (ks + 1 < nks) stage(buf ^ 1);
    __syncthreads();
  }
  float *out = ws + (int64_t)blockIdx.z * Cout * taps * Cin;
#pragma unroll
  for (int a = 0; a < TG; ++a) {
    if (a >= ntg) continue;
    const int t = t0 + a;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ci = ci0 + wc * 32 + j * 16 + lr;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int co = co0 + wr * 32 + i * 16 + 4 * lg + v;
          out[((int64_t)co * taps + t) * Cin + ci] = acc[a][i][j][v];
        }
      }
  }
}

int64_t sparse_wgrad_splits(int64_t M, int taps, int Cin, int Cout) {
  const int64_t tiles = (int64_t)(Cout / 64) * (Cin / 64) * ((taps + TG - 1) / TG);
  int64_t sp = (2048 + tiles - 1) / tiles;
  const int64_t maxsp = (M + 4 * WV - 1) / (4 * WV);
  if (sp > maxsp) sp = maxsp;
  return sp < 1 ? 1 : sp;
}

bool geom_ok(const pcs_conv3d_geom *g, const char **why) {
  if (!g) { *why = "null geometry"; return false; }
  if (g->B <= 0 || g->Di <= 0 || g->Hi <= 0 || g->Wi <= 0 || g->Do <= 0 || g->Ho <= 0 || g->Wo <= 0) {
    *why = "empty grid";
    return false;
  }
  if (g->k < 1 || g->k > 3 || (g->s != 1 && g->s != 2) || g->p < 0 || g->p >= g->k || (g->transposed != 0 && g->transposed != 1)) {
    *why = "k in 1..3, s in {1, 2}, 0 <= p < k, transposed 0 or 1";
    return false;
  }
  const int din[3] = {g->Di, g->Hi, g->Wi}, dout[3] = {g->Do, g->Ho, g->Wo};
  for (int d = 0; d < 3; ++d) {
    // transposed: + output_padding in [0, s) (torch's; the extra planes are plain gather rows)
    const int expect = g->transposed ? (din[d] - 1) * g->s - 2 * g->p + g->k : (din[d] + 2 * g->p - g->k) / g->s + 1;
    const int slack = g->transposed ? g->s - 1 : 0;
    if (dout[d] < expect || dout[d] > expect + slack || (!g->transposed && din[d] + 2 * g->p < g->k)) {
      *why = "output grid must be (in + 2p - k)/s + 1 (conv) or (in - 1)s - 2p + k + op, 0 <= op < s (transposed)";
      return false;
    }
  }
  if (g->B * g->Di * g->Hi * g->Wi >= ((int64_t)1 << 40) || g->B * g->Do * g->Ho * g->Wo >= ((int64_t)1 << 40)) {
    *why = "grid too large";
    return false;
  }
  return true;
}

int64_t out_voxels(const pcs_conv3d_geom &g) { return g.B * g.Do * g.Ho * g.Wo; }

bool stencil3(const pcs_conv3d_geom &g) { return g.k == 3 && g.s == 1; }
// channel tile of a layer: 64, or 32 where the count is an odd multiple of 32 (a 32-channel level)
int ctile(int c) { return c % 64 == 0 ? 64 : 32; }

int64_t stencil_blocks(const pcs_conv3d_geom &g) {
  return g.B * ((g.Do + SZ - 1) / SZ) * ((g.Ho + SY - 1) / SY) * ((g.Wo + SX - 1) / SX);
}

int64_t wgrad_splits(const pcs_conv3d_geom &g) {
  const int64_t M = out_voxels(g);
  if (stencil3(g)) {   // halo-tile kernel: 3 dz workgroups per (co, ci) tile and block range
    const int64_t tiles = (int64_t)(g.Cout / ctile(g.Cout)) * (g.Cin / ctile(g.Cin)) * 3;
    const int64_t sp = (1024 + tiles - 1) / tiles, nb = stencil_blocks(g);
    return sp > nb ? nb : sp;
  }
  const int64_t tiles = (int64_t)(g.Cout / ctile(g.Cout)) * (g.Cin / ctile(g.Cin)) *
                        (g.transposed && g.s == 2 ? g.k * g.k * g.k : g.k * g.k);
  int64_t sp = (2048 + tiles - 1) / tiles;
  const int64_t maxsp = (M + 4 * WV - 1) / (4 * WV);   // at least 4 k-steps per slice
  if (sp > maxsp) sp = maxsp;
  return sp < 1 ? 1 : sp;
}

int64_t wgrad_vps(const pcs_conv3d_geom &g, int64_t sp) {
  const int64_t M = out_voxels(g);
  return ((M + sp - 1) / sp + WV - 1) / WV * WV;
}

// ---- per-tap pair lists of a neighbour map: the sparse convolution as gather-GEMM-reduce.  The
// gather kernel above multiplies a zero row for every row of a tile that lacks a tap the tile
// meets; at low occupancy (1.5 occupied taps per voxel) that is most of its work.  Here each tap's
// (out row, in row) pairs are listed once per neighbour map (rows ascending within a tap, so the
// lists and every sum below are deterministic), the product of tap t is a GEMM over its own pairs
// only, and each output row sums its pairs' products in tap order.
constexpr int PT_MAX = 27;   // taps of the centred 3x3x3 map
struct PairTaps {            // host-built, passed by value: tap t's pairs [tap_off[t], tap_off[t + 1]),
  int64_t tap_off[PT_MAX + 1];   // its GEMM tiles [tile_off[t], tile_off[t + 1]), its weight-gradient
  int32_t tile_off[PT_MAX + 1];  // slices [slice_off[t], slice_off[t + 1]) of slice_len pairs each
  int32_t slice_off[PT_MAX + 1];
  int64_t slice_len;
  int32_t taps;
};

// a block's 256 rows of the neighbour map through LDS: coalesced loads (and, for pair_pos,
// coalesced stores) instead of 27 strided accesses per thread; [row][tap] words, stride 27 (odd:
// the per-tap reads are conflict-free)
PCS_DEV int pairs_rows(const int32_t *__restrict__ nbr, int64_t M, int taps, int32_t *rb) {
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int nr = (int)pcs_min64(256, M - r0), n = nr * taps;
  for (int i = threadIdx.x; i < n; i += 256) rb[i] = nbr[r0 * taps + i];
  __syncthreads();
  return nr;
}

// per-block pair counts of every tap: cnt[block][t] (one thread per row)
__global__ __launch_bounds__(256) void pairs_count_kernel(const int32_t *__restrict__ nbr, int64_t M, int taps,
                                                          int32_t *__restrict__ cnt) {
  __shared__ int32_t wc[4][PT_MAX];
  __shared__ int32_t rb[256 * PT_MAX];
  const int tid = threadIdx.x, w = tid >> 6;
  const int nr = pairs_rows(nbr, M, taps, rb);
  for (int t = 0; t < taps; ++t) {
    const bool has = tid < nr && rb[tid * taps + t] >= 0;
    const uint64_t b = __ballot(has);
    if ((tid & 63) == 0) wc[w][t] = __popcll(b);
  }
  __syncthreads();
  if (tid < taps) cnt[(int64_t)blockIdx.x * taps + tid] = wc[0][tid] + wc[1][tid] + wc[2][tid] + wc[3][tid];
}

// exclusive prefix of the block counts per tap (one workgroup per tap) and the tap totals
__global__ __launch_bounds__(256) void pairs_scan_kernel(int32_t *__restrict__ cnt, int64_t nblk, int taps,
                                                         int64_t *__restrict__ tap_counts) {
  __shared__ int32_t ws[4];
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nblk; b0 += 256) {
    const int64_t b = b0 + tid;
    const int32_t v = b < nblk ? cnt[b * taps + t] : 0;
    int32_t x = v;   // inclusive scan of the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    int32_t before = 0;
    for (int i = 0; i < w; ++i) before += ws[i];
    if (b < nblk) cnt[b * taps + t] = (int32_t)(carry + before + x - v);
    const int32_t tot = ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
    carry += tot;
  }
  if (tid == 0) tap_counts[t] = carry;
}

// pair_in / pair_out at tap_off[t] + (block prefix) + (rank in the block), pair_pos[m][t]:
// two ballot passes (the block's per-wave counts first, then each lane's rank)
__global__ __launch_bounds__(256) void pairs_build_kernel(const int32_t *__restrict__ nbr, int64_t M, int taps,
                                                          const int32_t *__restrict__ pre,
                                                          const int64_t *__restrict__ tap_counts,
                                                          int32_t *__restrict__ pin, int32_t *__restrict__ pout,
                                                          int32_t *__restrict__ ppos) {
  __shared__ int32_t wc[4][PT_MAX];
  __shared__ int64_t toff[PT_MAX];
  __shared__ int32_t rb[256 * PT_MAX];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t m = (int64_t)blockIdx.x * 256 + tid;
  if (tid == 0) {
    int64_t s = 0;
    for (int t = 0; t < taps; ++t) { toff[t] = s; s += tap_counts[t]; }
  }
  const int nr = pairs_rows(nbr, M, taps, rb);
  for (int t = 0; t < taps; ++t) {
    const uint64_t b = __ballot(tid < nr && rb[tid * taps + t] >= 0);
    if (lane == 0) wc[w][t] = __popcll(b);
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int t = 0; t < taps; ++t) {
    const int32_t n = tid < nr ? rb[tid * taps + t] : -1;
    const uint64_t b = __ballot(n >= 0);
    int32_t q = -1;
    if (n >= 0) {
      int64_t pos = toff[t] + pre[(int64_t)blockIdx.x * taps + t] + __popcll(b & lt);
      for (int i = 0; i < w; ++i) pos += wc[i][t];
      q = (int32_t)pos;
      pin[pos] = n;
      pout[pos] = (int32_t)m;
    }
    if (tid < nr) rb[tid * taps + t] = q;   // (only this thread reads or writes its row)
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  for (int i = tid; i < nr * taps; i += 256) ppos[r0 * taps + i] = rb[i];
}

// Z[p][n0 ..] = W[tw(t)] X[pair_in[p]] for the 64 pairs of one tile of tap t (fp32 products).
// (Reducing in the centre tap's GEMM epilogue instead of a separate pass, the centre's products
// never stored, was slower: 26 dependent gathers per lane there against 8 threads per row here.)
template <int KST>
__global__ __launch_bounds__(THREADS) void pair_gemm_kernel(PairTaps pt, const int32_t *__restrict__ pin,
                                                            const bf16_t *__restrict__ X, int Cin,
                                                            const bf16_t *__restrict__ W, int Cout, int flip,
                                                            float *__restrict__ Z) {
  constexpr int BMT = 64, RB = KST * 2, CPR = KST / 8, RPP = THREADS / CPR;
  constexpr int HA = BMT / RPP, HB = BN / RPP, KK = KST / 32;
  __shared__ __attribute__((aligned(16))) char lds[2][(BMT + BN) * RB];
  auto swzf = [](int row, int slot) { return KST == 32 ? cswz(row, slot) : (slot ^ ((row >> 1) & 7)); };
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  const int taps = pt.taps, tile = blockIdx.x;
  int t = 0;
  while (t + 1 < taps && pt.tile_off[t + 1] <= tile) ++t;
  const int tw = flip ? taps - 1 - t : t;
  const int64_t p0 = pt.tap_off[t] + (int64_t)(tile - pt.tile_off[t]) * BMT, pend = pt.tap_off[t + 1];
  const int n0 = blockIdx.y * BN;
  const int srow = tid / CPR, q = tid % CPR;
  int iv[HA];
#pragma unroll
  for (int h = 0; h < HA; ++h) {
    const int64_t p = p0 + srow + RPP * h;
    iv[h] = p < pend ? pin[p] : -1;
  }
  const bf16_t *wrow = W + ((int64_t)(n0 + srow) * taps + tw) * Cin + q * 8;
  const int64_t wstep = (int64_t)RPP * taps * Cin;
  const int nks = Cin / KST;
  u32x4 ra[HA], rb[HB];
  auto load = [&](int ks) {
    const int c0 = ks * KST;
#pragma unroll
    for (int h = 0; h < HA; ++h)
      ra[h] = iv[h] >= 0 ? *reinterpret_cast<const u32x4 *>(X + (int64_t)iv[h] * Cin + c0 + q * 8) : mk_u32x4(0, 0, 0, 0);
#pragma unroll
    for (int h = 0; h < HB; ++h) rb[h] = *reinterpret_cast<const u32x4 *>(wrow + h * wstep + c0);
  };
  auto stage = [&](int buf) {
    char *tA = lds[buf], *tB = lds[buf] + BMT * RB;
#pragma unroll
    for (int h = 0; h < HA; ++h) {
      const int r = srow + RPP * h;
      *reinterpret_cast<u32x4 *>(tA + r * RB + swzf(r, q) * 16) = ra[h];
    }
#pragma unroll
    for (int h = 0; h < HB; ++h) {
      const int r = srow + RPP * h;
      *reinterpret_cast<u32x4 *>(tB + r * RB + swzf(r, q) * 16) = rb[h];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  stage(0);
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(ks + 1);
    const char *tA = lds[buf], *tB = lds[buf] + BMT * RB;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 af[2], bw[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wr * 32 + i * 16 + lr;
        af[i] = *reinterpret_cast<const bf16x8 *>(tA + r * RB + swzf(r, kk * 4 + lg) * 16);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wc * 32 + j * 16 + lr;
        bw[j] = *reinterpret_cast<const bf16x8 *>(tB + r * RB + swzf(r, kk * 4 + lg) * 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nks) stage(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t p = p0 + wr * 32 + i * 16 + lr;
    if (p >= pend) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = n0 + wc * 32 + j * 16 + 4 * lg;
      *reinterpret_cast<f32x4 *>(Z + p * Cout + co) = acc[i][j];
    }
  }
}

// Y[m][c .. c + 7] = b + sum over taps in order of Z[pair_pos[m][t]] (one thread per 8 channels)
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void pair_reduce_kernel(const int32_t *__restrict__ ppos, int64_t M, int taps,
                                                          const float *__restrict__ Z, int Cout,
                                                          const float *__restrict__ bias, void *__restrict__ Y) {
  const int cpr = Cout / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * cpr) return;
  const int64_t m = i / cpr;
  const int c = (int)(i - m * cpr) * 8;
  f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = f32x4{0.f, 0.f, 0.f, 0.f};
  if (bias) {
    a = *reinterpret_cast<const f32x4 *>(bias + c);
    b = *reinterpret_cast<const f32x4 *>(bias + c + 4);
  }
  for (int t = 0; t < taps; ++t) {
    const int32_t q = ppos[m * taps + t];
    if (q < 0) continue;
    a += *reinterpret_cast<const f32x4 *>(Z + (int64_t)q * Cout + c);
    b += *reinterpret_cast<const f32x4 *>(Z + (int64_t)q * Cout + c + 4);
  }
  if constexpr (OUT_BF16) {
    *reinterpret_cast<u32x4 *>(reinterpret_cast<bf16_t *>(Y) + m * Cout + c) =
        mk_u32x4(pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3]));
  } else {
    *reinterpret_cast<f32x4 *>(reinterpret_cast<float *>(Y) + m * Cout + c) = a;
    *reinterpret_cast<f32x4 *>(reinterpret_cast<float *>(Y) + m * Cout + c + 4) = b;
  }
}

// dW_t partial of one pair slice g of tap t: sum over its pairs of dY[pair_out] (x) X[pair_in] into
// ws[g][co][ci] (the k-over-rows MFMA operands of conv3d_wgrad_kernel, gathered through the pair
// list).  Slices are a fixed number of pairs, so a tap's slice count follows its pair count (the
// centre tap has every row) and every workgroup has about the same work.
__global__ __launch_bounds__(THREADS) void pair_wgrad_kernel(PairTaps pt, const int32_t *__restrict__ pin,
                                                             const int32_t *__restrict__ pout,
                                                             const bf16_t *__restrict__ X, int Cin,
                                                             const bf16_t *__restrict__ dY, int Cout,
                                                             float *__restrict__ ws) {
  __shared__ __attribute__((aligned(16))) char lds[2][2 * WIMG];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, lr = lane & 15, lg = lane >> 4;
  const int nco = Cout / 64, taps = pt.taps;
  const int co0 = (blockIdx.x % nco) * 64, ci0 = (blockIdx.x / nco) * 64;
  const int g = blockIdx.y;
  int t = 0;
  while (t + 1 < taps && pt.slice_off[t + 1] <= g) ++t;
  const int64_t cnt = pt.tap_off[t + 1] - pt.tap_off[t], s0 = (int64_t)(g - pt.slice_off[t]) * pt.slice_len;
  const int64_t lo = pt.tap_off[t] + pcs_min64(s0, cnt), hi = pt.tap_off[t] + pcs_min64(s0 + pt.slice_len, cnt);
  const int sv = tid >> 3, q8 = tid & 7;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 rd, rx;
  auto load = [&](int64_t p0) {
    const int64_t p = p0 + sv;
    rd = mk_u32x4(0, 0, 0, 0);
    rx = mk_u32x4(0, 0, 0, 0);
    if (p < hi) {
      rd = *reinterpret_cast<const u32x4 *>(dY + (int64_t)pout[p] * Cout + co0 + q8 * 8);
      rx = *reinterpret_cast<const u32x4 *>(X + (int64_t)pin[p] * Cin + ci0 + q8 * 8);
    }
  };
  auto stage = [&](int buf) {
    *reinterpret_cast<u32x4 *>(lds[buf] + woff(sv, q8 * 16)) = rd;
    *reinterpret_cast<u32x4 *>(lds[buf] + WIMG + woff(sv, q8 * 16)) = rx;
  };
  const int nks = (int)((hi - lo + WV - 1) / WV);   // uniform; 0 for an empty slice
  if (nks > 0) {
    load(lo);
    stage(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(lo + (int64_t)(ks + 1) * WV);
    bf16x8 fd[2], fx[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fd[i] = wfrag(lds[buf], wr * 32 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) fx[j] = wfrag(lds[buf] + WIMG, wc * 32 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx[j], acc[i][j], 0, 0, 0);
    if (ks + 1 < nks) stage(buf ^ 1);
    __syncthreads();
  }
  float *out = ws + (int64_t)g * Cout * Cin;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ci = ci0 + wc * 32 + j * 16 + lr;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int co = co0 + wr * 32 + i * 16 + 4 * lg + v;
        out[(int64_t)co * Cin + ci] = acc[i][j][v];
      }
    }
}

// dW[co][t][ci] = sum over tap t's slices in order of ws[g][co][ci]
__global__ __launch_bounds__(256) void pair_wgrad_reduce_kernel(PairTaps pt, const float *__restrict__ ws, int Cin,
                                                                int Cout, float *__restrict__ dW) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // index into dW [Cout][taps][Cin]
  const int taps = pt.taps;
  if (i >= (int64_t)Cout * taps * Cin) return;
  const int ci = (int)(i % Cin);
  const int64_t r = i / Cin;
  const int t = (int)(r % taps), co = (int)(r / taps);
  float s = 0.f;
  for (int g = pt.slice_off[t]; g < pt.slice_off[t + 1]; ++g) s += ws[((int64_t)g * Cout + co) * Cin + ci];
  dW[i] = s;
}


}  // namespace

extern "C" int pcs_conv3d(const pcs_conv3d_geom *g, const void *X, const void *W, const float *bias, void *Y,
                          int32_t ydtype, pcs_stream_t stream) {
  const char *why = nullptr;
  if (!geom_ok(g, &why)) return pcs_set_einval("pcs_conv3d", why);
  if (!X || !W || !Y) return pcs_set_einval("pcs_conv3d", "X, W and Y are required");
  if (g->Cin % 32 != 0 || g->Cout % 32 != 0 || g->Cin <= 0 || g->Cout <= 0)
    return pcs_set_einval("pcs_conv3d", "Cin and Cout must be multiples of 32");
  if (ydtype != PCS_F32 && ydtype != PCS_BF16) return pcs_set_einval("pcs_conv3d", "Y dtype: PCS_F32 or PCS_BF16");
  const int64_t M = out_voxels(*g);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int cs = ctile(g->Cin), nt = ctile(g->Cout);
  if (stencil3(*g)) {   // halo-staged stencil (both forms)
    const int64_t nblk = stencil_blocks(*g);
    if (nblk > 0x7fffffff) return pcs_set_einval("pcs_conv3d", "grid too large");
    const dim3 sg((unsigned)nblk, (unsigned)(g->Cout / nt));
    const bf16_t *Xs = static_cast<const bf16_t *>(X), *Ws = static_cast<const bf16_t *>(W);
#define PCS_S3(CS, NT)                                                                                          \
  do {                                                                                                          \
    if (ydtype == PCS_BF16) hipLaunchKernelGGL((stencil3_kernel<CS, NT, true>), sg, dim3(THREADS), 0, s, *g, Xs, Ws, bias, Y); \
    else hipLaunchKernelGGL((stencil3_kernel<CS, NT, false>), sg, dim3(THREADS), 0, s, *g, Xs, Ws, bias, Y);   \
  } while (0)
    if (cs == 64) { if (nt == 64) PCS_S3(64, 64); else PCS_S3(64, 32); }
    else { if (nt == 64) PCS_S3(32, 64); else PCS_S3(32, 32); }
#undef PCS_S3
    PCS_CHECK_LAUNCH();
    return 0;
  }
  // transposed stride 2: 8 parity classes, tiles of the largest class's sub-grid each.  128-voxel
  // tiles (8 MFMAs per wave per barrier) once there are enough of them to fill the chip
  const int64_t rows_cls = g->transposed && g->s == 2 ? g->B * ((g->Do + 1) / 2) * ((g->Ho + 1) / 2) * ((g->Wo + 1) / 2) : M;
  const int64_t ncb = g->Cout / nt;
  const int bmt = (rows_cls / 128) * ncb * (g->transposed && g->s == 2 ? 8 : 1) >= 2048 ? 128 : 64;
  const int64_t tiles = (rows_cls + bmt - 1) / bmt * (g->transposed && g->s == 2 ? 8 : 1);
  if (tiles <= 0 || tiles > 0x7fffffff) return pcs_set_einval("pcs_conv3d", "grid too large");
  const dim3 grid((unsigned)tiles, (unsigned)ncb);
  const bf16_t *Xb = static_cast<const bf16_t *>(X), *Wb = static_cast<const bf16_t *>(W);
  const bool k64 = cs == 64;
#define PCS_C3(BMT, KST, OB, NT) \
  hipLaunchKernelGGL((conv3d_kernel<BMT, KST, OB, NT>), grid, dim3(THREADS), 0, s, *g, Xb, Wb, bias, Y, M)
#define PCS_C3K(BMT, OB)                                          \
  do {                                                            \
    if (nt == 64) { if (k64) PCS_C3(BMT, 64, OB, 64); else PCS_C3(BMT, 32, OB, 64); } \
    else { if (k64) PCS_C3(BMT, 64, OB, 32); else PCS_C3(BMT, 32, OB, 32); }          \
  } while (0)
  if (bmt == 128) {
    if (ydtype == PCS_BF16) PCS_C3K(128, true); else PCS_C3K(128, false);
  } else {
    if (ydtype == PCS_BF16) PCS_C3K(64, true); else PCS_C3K(64, false);
  }
#undef PCS_C3K
#undef PCS_C3
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t pcs_conv3d_wgrad_workspace(const pcs_conv3d_geom *g) {
  const char *why = nullptr;
  if (!geom_ok(g, &why)) return pcs_set_einval("pcs_conv3d_wgrad_workspace", why);
  if (g->Cin % 32 != 0 || g->Cout % 32 != 0 || g->Cin <= 0 || g->Cout <= 0)
    return pcs_set_einval("pcs_conv3d_wgrad_workspace", "Cin and Cout must be multiples of 32");
  const int64_t sp = wgrad_splits(*g);
  return sp * ((int64_t)g->Cout * g->k * g->k * g->k * g->Cin + g->Cout) * 4;
}

extern "C" int pcs_conv3d_wgrad(const pcs_conv3d_geom *g, const void *X, const void *dY, void *workspace,
                                int64_t workspace_bytes, float *dW, float *db, pcs_stream_t stream) {
  const int64_t need = pcs_conv3d_wgrad_workspace(g);
  if (need < 0) return (int)need;
  if (!X || !dY || !dW || !workspace || workspace_bytes < need)
    return pcs_set_einval("pcs_conv3d_wgrad", "X, dY, dW and a pcs_conv3d_wgrad_workspace-sized workspace are required");
  const int64_t M = out_voxels(*g), sp = wgrad_splits(*g), vps = wgrad_vps(*g, sp);
  const int taps = g->k * g->k * g->k;
  const int64_t wlen = (int64_t)g->Cout * taps * g->Cin;
  float *ws = static_cast<float *>(workspace), *wsb = ws + sp * wlen;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int cot = ctile(g->Cout), cit = ctile(g->Cin);
  const unsigned ntile = (unsigned)((g->Cout / cot) * (g->Cin / cit));
  const bf16_t *Xb = static_cast<const bf16_t *>(X), *dYb = static_cast<const bf16_t *>(dY);
  if (stencil3(*g)) {
    const int64_t nb = stencil_blocks(*g), bps = (nb + sp - 1) / sp;
    const dim3 grid(ntile, 3u, (unsigned)sp);
#define PCS_SW(CO, CI) hipLaunchKernelGGL((stencil3_wgrad_kernel<CO, CI>), grid, dim3(THREADS), 0, s, *g, Xb, dYb, ws, nb, bps)
    if (cot == 64) { if (cit == 64) PCS_SW(64, 64); else PCS_SW(64, 32); }
    else { if (cit == 64) PCS_SW(32, 64); else PCS_SW(32, 32); }
#undef PCS_SW
  } else {
    const int groups = g->transposed && g->s == 2 ? taps : g->k * g->k;   // workgroups per (co, ci) tile and slice
    const dim3 grid(ntile, (unsigned)groups, (unsigned)sp);
#define PCS_GW(CO, CI) hipLaunchKernelGGL((conv3d_wgrad_kernel<CO, CI>), grid, dim3(THREADS), 0, s, *g, Xb, dYb, ws, M, vps)
    if (cot == 64) { if (cit == 64) PCS_GW(64, 64); else PCS_GW(64, 32); }
    else { if (cit == 64) PCS_GW(32, 64); else PCS_GW(32, 32); }
#undef PCS_GW
  }
  PCS_CHECK_LAUNCH();
  hipLaunchKernelGGL(conv3d_reduce_kernel, dim3((unsigned)((wlen + 255) / 256)), dim3(256), 0, s, ws, sp, wlen, dW);
  PCS_CHECK_LAUNCH();
  if (db) {
    hipLaunchKernelGGL(conv3d_bgrad_kernel, dim3((unsigned)((g->Cout + 63) / 64), (unsigned)sp), dim3(THREADS), 0, s,
                       static_cast<const bf16_t *>(dY), g->Cout, M, vps, wsb);
    PCS_CHECK_LAUNCH();
    hipLaunchKernelGGL(conv3d_reduce_kernel, dim3((unsigned)((g->Cout + 255) / 256)), dim3(256), 0, s, wsb, sp,
                       (int64_t)g->Cout, db);
    PCS_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int pcs_conv3d_weight_t(const void *W, int32_t Cout, int32_t taps, int32_t Cin, void *Wt, pcs_stream_t stream) {
  if (!W || !Wt || Cout <= 0 || taps <= 0 || taps > 27 || Cin <= 0)
    return pcs_set_einval("pcs_conv3d_weight_t", "bad arguments (0 < taps <= 27)");
  const int64_t n = (int64_t)Cout * taps * Cin;
  hipLaunchKernelGGL(conv3d_weight_t_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), static_cast<const bf16_t *>(W), Cout, taps, Cin,
                     static_cast<bf16_t *>(Wt));
  PCS_CHECK_LAUNCH();
  return 0;
}

// ---- submanifold sparse convolution (hash-indexed gather; see sparse_conv_kernel)
extern "C" int pcs_sparse_conv(const int32_t *nbr, int64_t M, int32_t taps, const void *X, int32_t Cin, const void *W,
                               int32_t Cout, const float *bias, void *Y, int32_t ydtype, int32_t flip,
                               pcs_stream_t stream) {
  if (!nbr || !X || !W || !Y || M < 0 || taps < 1 || taps > 27 || Cin <= 0 || Cout <= 0 || Cin % KS != 0 ||
      Cout % BN != 0 || (ydtype != PCS_F32 && ydtype != PCS_BF16))
    return pcs_set_einval("pcs_sparse_conv", "bad arguments (1 <= taps <= 27, Cin % 32 == 0, Cout % 64 == 0, Y f32 | bf16)");
  // flip = 1 reads tap taps - 1 - t for tap t: the input gradient's offset(taps - 1 - t) = -offset(t)
  // holds only for the full centred 27-tap map (or the single centre tap)
  if (flip != 0 && taps != 27 && taps != 1)
    return pcs_set_einval("pcs_sparse_conv", "flip needs the centred 27-tap neighbour map (or taps == 1)");
  if (M == 0) return 0;
  const int64_t tiles = (M + 63) / 64;
  if (tiles > 0x7fffffff) return pcs_set_einval("pcs_sparse_conv", "too many rows");
  const dim3 grid((unsigned)tiles, (unsigned)(Cout / BN));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bf16_t *Xb = static_cast<const bf16_t *>(X), *Wb = static_cast<const bf16_t *>(W);
#define PCS_SC(KST, OB) \
  hipLaunchKernelGGL((sparse_conv_kernel<64, KST, OB>), grid, dim3(THREADS), 0, s, nbr, M, (int)taps, Xb, (int)Cin, Wb, \
                     (int)Cout, bias, Y, (int)flip)
  if (Cin % 64 == 0) {
    if (ydtype == PCS_BF16) PCS_SC(64, true); else PCS_SC(64, false);
  } else {
    if (ydtype == PCS_BF16) PCS_SC(32, true); else PCS_SC(32, false);
  }
#undef PCS_SC
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t pcs_sparse_conv_wgrad_workspace(int64_t M, int32_t taps, int32_t Cin, int32_t Cout) {
  if (M < 0 || taps < 1 || taps > 27 || Cin <= 0 || Cout <= 0 || Cin % 64 != 0 || Cout % 64 != 0)
    return pcs_set_einval("pcs_sparse_conv_wgrad_workspace", "bad arguments (Cin, Cout multiples of 64)");
  const int64_t sp = sparse_wgrad_splits(M, taps, Cin, Cout);
  return sp * ((int64_t)Cout * taps * Cin + Cout) * 4;
}

extern "C" int pcs_sparse_conv_wgrad(const int32_t *nbr, int64_t M, int32_t taps, const void *X, int32_t Cin,
                                     const void *dY, int32_t Cout, void *workspace, int64_t workspace_bytes, float *dW,
                                     float *db, pcs_stream_t stream) {
  const int64_t need = pcs_sparse_conv_wgrad_workspace(M, taps, Cin, Cout);
  if (need < 0) return (int)need;
  if (!nbr || !X || !dY || !dW || !workspace || workspace_bytes < need)
    return pcs_set_einval("pcs_sparse_conv_wgrad", "nbr, X, dY, dW and a workspace of pcs_sparse_conv_wgrad_workspace bytes");
  const int64_t sp = sparse_wgrad_splits(M, taps, Cin, Cout);
  const int64_t vps = ((M + sp - 1) / sp + WV - 1) / WV * WV;
  const int64_t wlen = (int64_t)Cout * taps * Cin;
  float *ws = static_cast<float *>(workspace), *wsb = ws + sp * wlen;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (M > 0) {
    hipLaunchKernelGGL(sparse_wgrad_kernel, dim3((unsigned)((Cout / 64) * (Cin / 64)), (unsigned)((taps + TG - 1) / TG), (unsigned)sp),
                       dim3(THREADS), 0, s, nbr, M, (int)taps, static_cast<const bf16_t *>(X), (int)Cin,
                       static_cast<const bf16_t *>(dY), (int)Cout, ws, vps);
  } else {
    const hipError_t e = hipMemsetAsync(ws, 0, sp * wlen * 4, s);
    if (e != hipSuccess) return pcs_set_error(e, "pcs_sparse_conv_wgrad");
  }
  PCS_CHECK_LAUNCH();
  hipLaunchKernelGGL(conv3d_reduce_kernel, dim3((unsigned)((wlen + 255) / 256)), dim3(256), 0, s, ws, sp, wlen, dW);
  PCS_CHECK_LAUNCH();
  if (db) {
    if (M > 0) {
      hipLaunchKernelGGL(conv3d_bgrad_kernel, dim3((unsigned)(Cout / 64), (unsigned)sp), dim3(THREADS), 0, s,
                         static_cast<const bf16_t *>(dY), (int)Cout, M, vps, wsb);
    } else {
      const hipError_t e = hipMemsetAsync(wsb, 0, sp * Cout * 4, s);
      if (e != hipSuccess) return pcs_set_error(e, "pcs_sparse_conv_wgrad");
    }
    PCS_CHECK_LAUNCH();
    hipLaunchKernelGGL(conv3d_reduce_kernel, dim3((unsigned)((Cout + 255) / 256)), dim3(256), 0, s, wsb, sp,
                       (int64_t)Cout, db);
    PCS_CHECK_LAUNCH();
  }
  return 0;
}

// ---- per-tap pair lists (see pairs_count_kernel)
extern "C" int64_t pcs_sparse_pairs_workspace(int64_t M, int32_t taps) {
  if (M < 0 || taps < 1 || taps > PT_MAX) return pcs_set_einval("pcs_sparse_pairs_workspace", "bad arguments (1 <= taps <= 27)");
  return ((M + 255) / 256 * taps + 1) * 4;
}

extern "C" int pcs_sparse_pairs_count(const int32_t *nbr, int64_t M, int32_t taps, void *workspace, int64_t *tap_counts,
                                      pcs_stream_t stream) {
  const int64_t need = pcs_sparse_pairs_workspace(M, taps);
  if (need < 0) return (int)need;
  if (!nbr || !workspace || !tap_counts) return pcs_set_einval("pcs_sparse_pairs_count", "nbr, workspace and tap_counts are required");
  if (M * taps >= ((int64_t)1 << 31)) return pcs_set_einval("pcs_sparse_pairs_count", "M * taps must be < 2^31");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t nblk = (M + 255) / 256;
  int32_t *cnt = static_cast<int32_t *>(workspace);
  if (nblk > 0)
    hipLaunchKernelGGL(pairs_count_kernel, dim3((unsigned)nblk), dim3(256), 0, s, nbr, M, (int)taps, cnt);
  hipLaunchKernelGGL(pairs_scan_kernel, dim3((unsigned)taps), dim3(256), 0, s, cnt, nblk, (int)taps, tap_counts);
  PCS_CHECK_LAUNCH();
  return 0;
}

extern "C" int pcs_sparse_pairs_build(const int32_t *nbr, int64_t M, int32_t taps, const void *workspace,
                                      const int64_t *tap_counts, int32_t *pair_in, int32_t *pair_out, int32_t *pair_pos,
                                      pcs_stream_t stream) {
  if (pcs_sparse_pairs_workspace(M, taps) < 0) return PCS_EINVAL;
  if (!nbr || !workspace || !tap_counts || !pair_pos || ((!pair_in || !pair_out) && M > 0))
    return pcs_set_einval("pcs_sparse_pairs_build", "nbr, workspace, tap_counts, pair_in, pair_out and pair_pos are required");
  if (M * taps >= ((int64_t)1 << 31)) return pcs_set_einval("pcs_sparse_pairs_build", "M * taps must be < 2^31");
  const int64_t nblk = (M + 255) / 256;
  if (nblk > 0)
    hipLaunchKernelGGL(pairs_build_kernel, dim3((unsigned)nblk), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), nbr, M,
                       (int)taps, static_cast<const int32_t *>(workspace), tap_counts, pair_in, pair_out, pair_pos);
  PCS_CHECK_LAUNCH();
  return 0;
}

namespace {
// the tap and tile offsets of a pair list from the host copy of its tap offsets
const char *pair_taps(const int64_t *tap_off, int32_t taps, PairTaps *pt) {
  if (!tap_off || taps < 1 || taps > PT_MAX) return "tap_off (host, taps + 1 entries) and 1 <= taps <= 27";
  pt->taps = taps;
  int64_t tiles = 0;
  for (int t = 0; t <= taps; ++t) {
    if (tap_off[t] < (t ? tap_off[t - 1] : 0) || (t == 0 && tap_off[0] != 0)) return "tap_off must start at 0 and not decrease";
    pt->tap_off[t] = tap_off[t];
    pt->tile_off[t] = (int32_t)tiles;
    if (t < taps) tiles += (tap_off[t + 1] - tap_off[t] + 63) / 64;
  }
  if (tiles > 0x7fffffff || tap_off[taps] >= ((int64_t)1 << 31)) return "too many pairs";
  return nullptr;
}
}  // namespace

extern "C" int pcs_sparse_conv_pairs(const int32_t *pair_in, const int32_t *pair_pos, const int64_t *tap_off, int32_t taps,
                                     int64_t M, const void *X, int32_t Cin, const void *W, int32_t Cout,
                                     const float *bias, float *Z, void *Y, int32_t ydtype, int32_t flip,
                                     pcs_stream_t stream) {
  PairTaps pt;
  const char *why = pair_taps(tap_off, taps, &pt);
  if (why) return pcs_set_einval("pcs_sparse_conv_pairs", why);
  if (!pair_pos || !X || !W || !Y || M < 0 || Cin <= 0 || Cout <= 0 || Cin % KS != 0 || Cout % BN != 0 ||
      (ydtype != PCS_F32 && ydtype != PCS_BF16) || (tap_off[taps] > 0 && (!pair_in || !Z)))
    return pcs_set_einval("pcs_sparse_conv_pairs", "bad arguments (Cin % 32 == 0, Cout % 64 == 0, Y f32 | bf16, Z [P, Cout] f32)");
  if (flip && taps != 27 && taps != 1)
    return pcs_set_einval("pcs_sparse_conv_pairs", "flip needs the centred 27-tap neighbour map (or taps == 1)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int tiles = pt.tile_off[taps];
  const bf16_t *Xb = static_cast<const bf16_t *>(X), *Wb = static_cast<const bf16_t *>(W);
  if (tiles > 0) {
    const dim3 grid((unsigned)tiles, (unsigned)(Cout / BN));
    if (Cin % 64 == 0) hipLaunchKernelGGL(pair_gemm_kernel<64>, grid, dim3(THREADS), 0, s, pt, pair_in, Xb, (int)Cin, Wb, (int)Cout, (int)flip, Z);
    else hipLaunchKernelGGL(pair_gemm_kernel<32>, grid, dim3(THREADS), 0, s, pt, pair_in, Xb, (int)Cin, Wb, (int)Cout, (int)flip, Z);
    PCS_CHECK_LAUNCH();
  }
  const int64_t n = M * (Cout / 8);
  if (n > 0) {
    const dim3 g((unsigned)((n + 255) / 256));
    if (ydtype == PCS_BF16) hipLaunchKernelGGL(pair_reduce_kernel<true>, g, dim3(256), 0, s, pair_pos, M, (int)taps, Z, (int)Cout, bias, Y);
    else hipLaunchKernelGGL(pair_reduce_kernel<false>, g, dim3(256), 0, s, pair_pos, M, (int)taps, Z, (int)Cout, bias, Y);
    PCS_CHECK_LAUNCH();
  }
  return 0;
}

namespace {
// weight-gradient slices: slice_len pairs each (at least 4 k-steps), ceil(count / slice_len) per
// tap (at least one, so every tap's partial is written), about 2048 workgroups over the slices
// and the 64 x 64 channel tiles together (as sparse_wgrad_splits): each slice holds a full
// Cout x Cin fp32 partial, so the workspace stays near 2048 tiles' worth (34 MB at 64 -> 64, 40 MB
// at 256 -> 256, where a fixed 2048 slices took 544 MB) instead of growing with the channel product
void pair_wgrad_slices(PairTaps *pt, int Cin, int Cout) {
  const int64_t P = pt->tap_off[pt->taps];
  const int64_t tiles = (int64_t)(Cout / 64) * (Cin / 64);
  const int64_t target = (2048 + tiles - 1) / tiles;
  int64_t len = (P + target - 1) / target;
  len = (len < 4 * WV ? 4 * WV : len + WV - 1) / WV * WV;
  pt->slice_len = len;
  int64_t g = 0;
  for (int t = 0; t <= pt->taps; ++t) {
    pt->slice_off[t] = (int32_t)g;
    if (t < pt->taps) {
      const int64_t c = pt->tap_off[t + 1] - pt->tap_off[t];
      g += c > 0 ? (c + len - 1) / len : 1;
    }
  }
}
}  // namespace

extern "C" int64_t pcs_sparse_conv_wgrad_pairs_workspace(const int64_t *tap_off, int32_t taps, int64_t M, int32_t Cin,
                                                         int32_t Cout) {
  PairTaps pt;
  const char *why = pair_taps(tap_off, taps, &pt);
  if (why) return pcs_set_einval("pcs_sparse_conv_wgrad_pairs_workspace", why);
  if (M < 0 || Cin <= 0 || Cout <= 0 || Cin % 64 != 0 || Cout % 64 != 0)
    return pcs_set_einval("pcs_sparse_conv_wgrad_pairs_workspace", "bad arguments (Cin, Cout multiples of 64)");
  pair_wgrad_slices(&pt, Cin, Cout);
  const int64_t spb = sparse_wgrad_splits(M, 1, 64, Cout);
  return ((int64_t)pt.slice_off[taps] * Cout * Cin + spb * Cout) * 4;
}

extern "C" int pcs_sparse_conv_wgrad_pairs(const int32_t *pair_in, const int32_t *pair_out, const int64_t *tap_off,
                                           int32_t taps, int64_t M, const void *X, int32_t Cin, const void *dY,
                                           int32_t Cout, void *workspace, int64_t workspace_bytes, float *dW, float *db,
                                           pcs_stream_t stream) {
  const int64_t need = pcs_sparse_conv_wgrad_pairs_workspace(tap_off, taps, M, Cin, Cout);
  if (need < 0) return (int)need;
  if (!X || !dY || !dW || !workspace || workspace_bytes < need || (tap_off[taps] > 0 && (!pair_in || !pair_out)))
    return pcs_set_einval("pcs_sparse_conv_wgrad_pairs", "pairs, X, dY, dW and a workspace of pcs_sparse_conv_wgrad_pairs_workspace bytes");
  PairTaps pt;
  pair_taps(tap_off, taps, &pt);
  pair_wgrad_slices(&pt, Cin, Cout);
  const int64_t ns = pt.slice_off[taps], wlen = (int64_t)Cout * taps * Cin;
  float *ws = static_cast<float *>(workspace), *wsb = ws + ns * Cout * Cin;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(pair_wgrad_kernel, dim3((unsigned)((Cout / 64) * (Cin / 64)), (unsigned)ns), dim3(THREADS), 0, s,
                     pt, pair_in, pair_out, static_cast<const bf16_t *>(X), (int)Cin, static_cast<const bf16_t *>(dY), (int)Cout, ws);
  PCS_CHECK_LAUNCH();
  hipLaunchKernelGGL(pair_wgrad_reduce_kernel, dim3((unsigned)((wlen + 255) / 256)), dim3(256), 0, s, pt, ws, (int)Cin, (int)Cout, dW);
  PCS_CHECK_LAUNCH();
  if (db) {
    const int64_t spb = sparse_wgrad_splits(M, 1, 64, Cout);
    const int64_t vps = ((M + spb - 1) / spb + WV - 1) / WV * WV;
    if (M > 0) {
      hipLaunchKernelGGL(conv3d_bgrad_kernel, dim3((unsigned)((Cout + 63) / 64), (unsigned)spb), dim3(THREADS), 0, s,
                         static_cast<const bf16_t *>(dY), (int)Cout, M, vps, wsb);
    } else {
      const hipError_t e = hipMemsetAsync(wsb, 0, spb * Cout * 4, s);
      if (e != hipSuccess) return pcs_set_error(e, "pcs_sparse_conv_wgrad_pairs");
    }
    PCS_CHECK_LAUNCH();
    hipLaunchKernelGGL(conv3d_reduce_kernel, dim3((unsigned)((Cout + 255) / 256)), dim3(256), 0, s, wsb, spb, (int64_t)Cout, db);
    PCS_CHECK_LAUNCH();
  }
  return 0;
}

// Probe of the gfx950 MX-scaled fp8 MFMA and the 8-bit transposed LDS read on the device:
//   hipcc --offload-arch=gfx950 -O2 tools/probe_mx.hip -o gpurun_out/probe_mx && gpurun_out/probe_mx
// (1) v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands: which (row, k) each lane's 32
//     bytes hold and which K block each lane's scale byte applies to, checked against a host
//     reference for the assumed map  A[row = l & 15][k = 32 (l >> 4) + j],
//     B[k = 32 (l >> 4) + j][col = l & 15], D[row = 4 (l >> 4) + r][col = l & 15];
// (2) ds_read_b64_tr_b8: what a lane receives from a [row][col] byte image.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

// OCP e4m3fn decode
static float e4m3(unsigned char b) {
  const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  float v = e == 0 ? std::ldexp((float)m, -9) : std::ldexp(1.0f + m / 8.0f, e - 7);
  if (e == 15 && m == 7) v = NAN;
  return s ? -v : v;
}
// small integers and halves are exact in e4m3: encode v in {-8..8} step 0.5
static unsigned char enc(float v) {
  for (int b = 0; b < 256; ++b)
    if (e4m3((unsigned char)b) == v) return (unsigned char)b;
  return 0;
}

__global__ void mfma_probe(const v8i *a, const v8i *b, const int *sa, const int *sb, v4f *d) {
  const int l = threadIdx.x;
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 0, 0, 0, sa[l], 0, sb[l]);
  d[l] = c;
}

typedef __attribute__((address_space(3))) v2i lds_v2i;
__global__ void tr8_probe(const unsigned char *img, int rowb, int *out) {
  __shared__ unsigned char lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = img[i];
  __syncthreads();
  const int l = threadIdx.x;
  // lane l reads at row (l & 7) ... the probe uses the same per-lane address pattern as
  // ds_read_b64_tr_b16 in gram_glds.hip scaled to bytes: row 8g + q, column 8p (bytes)
  // pattern: within each 16-lane group lane i reads row (i >> 1) of an 8-row block, byte
  // column 8 (i & 1); the group's block starts at row 8 (l >> 4)
  const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const int row = 8 * g + ((l & 15) >> 1), col = 8 * (l & 1);
  const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i *)(lds + row * rowb + col));
  (void)g; (void)q; (void)p;
  out[2 * l] = v[0];
  out[2 * l + 1] = v[1];
}

// candidate lane -> k maps for the 32 bytes of a 16x16x128 f8f6f4 operand (lane l, byte j)
static int kmap(int h, int l, int j) {
  const int g = l >> 4;
  if (h == 0) return 32 * g + j;                          // H1: 32 consecutive k per lane group
  if (h == 1) return 8 * g + 32 * (j >> 3) + (j & 7);     // H2: bf16-like 8-k groups, stride 32
  return 16 * g + 64 * (j >> 4) + (j & 15);               // H3: 16-k groups, stride 64
}

static v4f hd[64];
static double run(const unsigned char (&A)[16][128], const unsigned char (&B)[128][16], int h, const int *hsa,
                  const int *hsb, double (*ref)[16], v8i *da, v8i *db, int *dsa, int *dsb, v4f *dd) {
  v8i ha[64], hb[64];
  for (int l = 0; l < 64; ++l) {
    unsigned char ab[32], bb[32];
    for (int j = 0; j < 32; ++j) {
      ab[j] = A[l & 15][kmap(h, l, j)];
      bb[j] = B[kmap(h, l, j)][l & 15];
    }
    memcpy(&ha[l], ab, 32);
    memcpy(&hb[l], bb, 32);
  }
  hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice);
  hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost);
  double maxerr = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) maxerr = fmax(maxerr, fabs(hd[l][r] - ref[4 * (l >> 4) + r][l & 15]));
  return maxerr;
}

int main() {
  // ---- (1) MX fp8 MFMA
  static unsigned char A[16][128], B[128][16];
  srand(7);
  for (int r = 0; r < 16; ++r)
    for (int k = 0; k < 128; ++k) A[r][k] = enc((float)(rand() % 9 - 4) * 0.5f);
  for (int k = 0; k < 128; ++k)
    for (int c = 0; c < 16; ++c) B[k][c] = enc((float)(rand() % 9 - 4) * 0.5f);
  v8i *da, *db;
  int *dsa, *dsb;
  v4f *dd;
  hipMalloc(&da, 64 * sizeof(v8i)); hipMalloc(&db, 64 * sizeof(v8i)); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
  hipMalloc(&dd, 64 * sizeof(v4f));
  static double ref[16][16];
  // unit scales: pin the data layout
  int sa[64], sb[64];
  for (int l = 0; l < 64; ++l) { sa[l] = 127; sb[l] = 127; }
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      double s = 0;
      for (int k = 0; k < 128; ++k) s += (double)e4m3(A[r][k]) * (double)e4m3(B[k][c]);
      ref[r][c] = s;
    }
  int good = -1;
  for (int h = 0; h < 3; ++h) {
    const double e = run(A, B, h, sa, sb, ref, da, db, dsa, dsb, dd);
    printf("unit scales, layout H%d: max |D - ref| = %g\n", h + 1, e);
    if (e < 1e-6 && good < 0) good = h;
  }
  if (good >= 0) {
    // scale semantics: every lane's 32-bit scale register holds 4 distinct E8M0 bytes
    for (int l = 0; l < 64; ++l) {
      sa[l] = sb[l] = 0;
      for (int t = 0; t < 4; ++t) {
        sa[l] |= (127 + ((t + l) % 3) - 1) << (8 * t);
        sb[l] |= (127 + ((t + 2 * l) % 3) - 1) << (8 * t);
      }
    }
    auto byte = [](int v, int t) { return (v >> (8 * t)) & 255; };
    {   // the form the kernels use: one scale per A row and per B column, replicated in all
        // four bytes and in every lane of that row / column
      int ra[64], rb[64];
      for (int l = 0; l < 64; ++l) {
        const int ea = 127 + (l & 15) % 3 - 1, eb = 127 + (l & 15) % 2;
        ra[l] = ea * 0x01010101;
        rb[l] = eb * 0x01010101;
      }
      for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
          double s = 0;
          for (int k = 0; k < 128; ++k)
            s += (double)e4m3(A[r][k]) * (double)e4m3(B[k][c]) * std::ldexp(1.0, (r % 3 - 1) + (c % 2));
          ref[r][c] = s;
        }
      printf("per-row / per-column scales (replicated bytes): max |D - ref| = %g\n",
             run(A, B, good, ra, rb, ref, da, db, dsa, dsb, dd));
    }
    const char *names[5] = {"S3a: A(r,k) <- byte k/32 of lane r, B(k,c) <- byte k/32 of lane c",
                            "S3b: byte 0 of the lane holding the element",
                            "S3c: byte 0 of lane r + 16 (k/32) / lane c + 16 (k/32)",
                            "S3d: byte k/32 of the lane holding the element",
                            "S3e: byte 0 of lane r / lane c (one scale per row / column)"};
    for (int hyp = 0; hyp < 5; ++hyp) {
      for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
          double s = 0;
          for (int k = 0; k < 128; ++k) {
            const int kb = k >> 5;
            int la = -1, lb = -1;
            for (int l = 0; l < 64 && (la < 0 || lb < 0); ++l)
              for (int jj = 0; jj < 32; ++jj)
                if (kmap(good, l, jj) == k) {
                  if ((l & 15) == r) la = l;
                  if ((l & 15) == c) lb = l;
                }
            int ea, eb;
            if (hyp == 0) { ea = byte(sa[r], kb); eb = byte(sb[c], kb); }
            else if (hyp == 1) { ea = byte(sa[la], 0); eb = byte(sb[lb], 0); }
            else if (hyp == 2) { ea = byte(sa[r + 16 * kb], 0); eb = byte(sb[c + 16 * kb], 0); }
            else if (hyp == 3) { ea = byte(sa[la], kb); eb = byte(sb[lb], kb); }
            else { ea = byte(sa[r], 0); eb = byte(sb[c], 0); }
            s += (double)e4m3(A[r][k]) * std::ldexp(1.0, ea - 127) * (double)e4m3(B[k][c]) * std::ldexp(1.0, eb - 127);
          }
          ref[r][c] = s;
        }
      printf("%s: max |D - ref| = %g\n", names[hyp], run(A, B, good, sa, sb, ref, da, db, dsa, dsb, dd));
    }
  }
  double maxerr = good >= 0 ? 0 : 1;

  // ---- (2) ds_read_b64_tr_b8
  unsigned char img[64 * 64];
  for (int r = 0; r < 64; ++r)
    for (int c = 0; c < 64; ++c) img[r * 64 + c] = (unsigned char)((r & 15) * 16 + (c & 15));   // byte = row:col nibbles
  unsigned char *dimg;
  int *dout;
  hipMalloc(&dimg, sizeof(img));
  hipMalloc(&dout, 128 * 4);
  hipMemcpy(dimg, img, sizeof(img), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(tr8_probe, dim3(1), dim3(64), 0, 0, dimg, 64, dout);
  int hout[128];
  hipMemcpy(hout, dout, sizeof(hout), hipMemcpyDeviceToHost);
  printf("ds_read_b64_tr_b8 (lane reads at row 8(l>>4) + ((l&15)>>1), byte col 8(l&1)); bytes as row:col (hex):\n");
  for (int l = 0; l < 64; ++l) {
    unsigned char bytes[8];
    memcpy(bytes, &hout[2 * l], 8);
    printf("  lane %2d:", l);
    for (int j = 0; j < 8; ++j) printf(" %02x", bytes[j]);
    printf("\n");
  }
  return maxerr < 1e-6 ? 0 : 1;
}

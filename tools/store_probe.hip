// HBM store-pattern probe: what the narrow layers' epilogues can write at best.
// Writes a [M x 1024] bf16 matrix (M = 8,388,608: conv5's a5, 17.2 GB) with the store shapes
// the GEMM epilogues use, one persistent grid of (256 CUs x wgs_per_cu) workgroups:
//   lin16   each wave instruction writes 1 KB contiguous (64 lanes x 16 B)           [ideal]
//   r16x64  16 rows x 64 B per instruction (16-B lanes, 4 lanes per row segment)     [glds dgrad]
//   r8x128  8 rows x 128 B per instruction (8 lanes per row segment)
//   r16x32  16 rows x 32 B per instruction (8-B lanes: a 16x16 MFMA tile, no permlane)
// plain and non-temporal; plus a read-only sweep of the same matrix.  Prints TB/s.
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o /tmp/store_probe && /tmp/store_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t M = 8388608, NC = 1024, ROWB = NC * 2;

// A "tile" is 64 rows x 1024 columns (128 KB); workgroups stride over tiles.  Within a tile a
// wave writes its share with the given instruction shape.
template <int SHAPE, bool NT>
__global__ __launch_bounds__(256) void store_kernel(char *out, int64_t ntiles) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const u32x4 v = {(unsigned)lane, 1u, 2u, 3u};
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    char *tile = out + t * 64 * ROWB;
    // 128 KB per tile = 128 instructions of 1 KB; wave w takes instructions w, w + nw, ...
    for (int q = wid; q < 128; q += nw) {
      int64_t off;
      if constexpr (SHAPE == 0) {            // lin16
        off = (int64_t)q * 1024 + lane * 16;
      } else if constexpr (SHAPE == 1) {     // r16x64: 4 row groups of 16 rows x 32 col segments of 64 B
        const int rg = q & 3, cs = q >> 2;   // 32 segments of 64 B per 2-KB row
        off = (int64_t)(rg * 16 + (lane & 15)) * ROWB + cs * 64 + (lane >> 4) * 16;
      } else if constexpr (SHAPE == 2) {     // r8x128: 8 row groups x 16 segments of 128 B
        const int rg = q & 7, cs = q >> 3;
        off = (int64_t)(rg * 8 + (lane & 7)) * ROWB + cs * 128 + (lane >> 3) * 16;
      } else {                               // r16x32, 8-B lanes: 2 KB-rows, 256 instr of 512 B
        const int rg = q & 3, cs = q >> 2;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int64_t o = (int64_t)(rg * 16 + (lane & 15)) * ROWB + (cs * 2 + h) * 32 + (lane >> 4) * 8;
          const unsigned long long w = ((unsigned long long)v.y << 32) | v.x;
          if constexpr (NT) __builtin_nontemporal_store(w, reinterpret_cast<unsigned long long *>(tile + o));
          else *reinterpret_cast<unsigned long long *>(tile + o) = w;
        }
        continue;
      }
      if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(tile + off));
      else *reinterpret_cast<u32x4 *>(tile + off) = v;
    }
  }
}

__global__ __launch_bounds__(256) void read_kernel(const char *in, int64_t ntiles, unsigned *sink) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned acc = 0;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const char *tile = in + t * 64 * ROWB;
    for (int q = wid; q < 128; q += nw) {
      const u32x4 x = *reinterpret_cast<const u32x4 *>(tile + (int64_t)q * 1024 + lane * 16);
      acc ^= x.x + x.y + x.z + x.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename F> float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  char *buf = nullptr;
  unsigned *sink = nullptr;
  const int64_t bytes = M * ROWB, ntiles = M / 64;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  const char *names[4] = {"lin16 ", "r16x64", "r8x128", "r16x32"};
  for (int wpc : {1, 2, 4, 8}) {
    const int grid = 256 * wpc;
    for (int s = 0; s < 4; ++s) {
      for (int nt = 0; nt < 2; ++nt) {
        float ms = timeit([&] {
#define L(S, N) hipLaunchKernelGGL((store_kernel<S, N>), dim3(grid), dim3(256), 0, 0, buf, ntiles)
          if (s == 0) { if (nt) L(0, true); else L(0, false); }
          else if (s == 1) { if (nt) L(1, true); else L(1, false); }
          else if (s == 2) { if (nt) L(2, true); else L(2, false); }
          else { if (nt) L(3, true); else L(3, false); }
#undef L
        });
        printf("store %s %s %d WG/CU (256 thr): %7.3f ms  %5.2f TB/s\n", names[s], nt ? "nt   " : "plain", wpc, ms,
               bytes / ms / 1e9);
      }
    }
    float ms = timeit([&] { hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, buf, ntiles, sink); });
    printf("read  lin16  plain %d WG/CU (256 thr): %7.3f ms  %5.2f TB/s\n", wpc, ms, bytes / ms / 1e9);
    fflush(stdout);
  }
  hipFree(buf);
  return 0;
}

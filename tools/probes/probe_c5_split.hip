// conv5's backward in one read of dz5 by the "two-level split" (DESIGN section 8.3): four
// workgroups per row slice each own 256 of dz5's 1024 columns (their R block fits the register
// file), and each adds its partial input gradient dz5[:, blk] . Ws[blk, :] -- an [M x 128] fp32
// term -- into one accumulator through L2.  This probe prices that hand-off alone at cfg2
// (M = 4 x 128^3): (a) four fp32 atomic adds per element (global_atomic_add_f32, no return);
// (b) four fp32 partials stored, then one pass that sums them; (c) four bf16 partials stored
// and summed.  Against it: the second read of dz5 (17.2 GB at ~6.4 TB/s = 2.7 ms) it would save.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/probe_c5_split.hip -o tools/probes/probe_c5_split
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int64_t M = 4LL * 128 * 128 * 128, C = 128, NBLK = 4;

__global__ void atomic_partials(float *acc, float v) {
  // thread = 4 consecutive floats of one row; the four column blocks' adds in block order
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= M * C) return;
  for (int b = 0; b < NBLK; ++b)
#pragma unroll
    for (int e = 0; e < 4; ++e) unsafeAtomicAdd(acc + i + e, v * (b + 1));   // global_atomic_add_f32
}
__global__ void store_partials_f32(float *part, float v) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= M * C) return;
  for (int b = 0; b < NBLK; ++b)
    *reinterpret_cast<float4 *>(part + b * M * C + i) = make_float4(v, v * 2, v * 3, v * b);
}
__global__ void sum_partials_f32(const float *part, float *out) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= M * C) return;
  float4 s = make_float4(0, 0, 0, 0);
  for (int b = 0; b < NBLK; ++b) {
    const float4 p = *reinterpret_cast<const float4 *>(part + b * M * C + i);
    s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
  }
  *reinterpret_cast<float4 *>(out + i) = s;
}
__global__ void store_partials_bf16(uint16_t *part, float v) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= M * C) return;
  const uint32_t w = __float_as_uint(v) >> 16;
  for (int b = 0; b < NBLK; ++b)
    *reinterpret_cast<uint4 *>(part + b * M * C + i) = make_uint4(w | (w << 16), w, w, w << 16);
}
__global__ void sum_partials_bf16(const uint16_t *part, uint16_t *out) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= M * C) return;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int b = 0; b < NBLK; ++b) {
    const uint4 p = *reinterpret_cast<const uint4 *>(part + b * M * C + i);
    const uint32_t w[4] = {p.x, p.y, p.z, p.w};
    for (int e = 0; e < 4; ++e) {
      s[2 * e] += __uint_as_float(w[e] << 16);
      s[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
    }
  }
  uint32_t o[4];
  for (int e = 0; e < 4; ++e) o[e] = (__float_as_uint(s[2 * e]) >> 16) | (__float_as_uint(s[2 * e + 1]) & 0xffff0000u);
  *reinterpret_cast<uint4 *>(out + i) = make_uint4(o[0], o[1], o[2], o[3]);
}

template <typename F> float timed(F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  float *acc, *part, *out;
  (void)hipMalloc(&acc, M * C * 4);
  (void)hipMalloc(&part, NBLK * M * C * 4);
  (void)hipMalloc(&out, M * C * 4);
  (void)hipMemset(acc, 0, M * C * 4);
  const unsigned g4 = (unsigned)((M * C / 4 + 255) / 256), g8 = (unsigned)((M * C / 8 + 255) / 256);
  const float ta = timed([&] { hipLaunchKernelGGL(atomic_partials, dim3(g4), dim3(256), 0, 0, acc, 1.f); });
  const float tb1 = timed([&] { hipLaunchKernelGGL(store_partials_f32, dim3(g4), dim3(256), 0, 0, part, 1.f); });
  const float tb2 = timed([&] { hipLaunchKernelGGL(sum_partials_f32, dim3(g4), dim3(256), 0, 0, part, out); });
  uint16_t *pb = reinterpret_cast<uint16_t *>(part), *ob = reinterpret_cast<uint16_t *>(out);
  const float tc1 = timed([&] { hipLaunchKernelGGL(store_partials_bf16, dim3(g8), dim3(256), 0, 0, pb, 1.f); });
  const float tc2 = timed([&] { hipLaunchKernelGGL(sum_partials_bf16, dim3(g8), dim3(256), 0, 0, pb, ob); });
  const double gb = M * C * 4 / 1e9;
  printf("M=%lld x %lld, %lld column blocks; one fp32 [M x 128] term = %.2f GB\n", (long long)M, (long long)C,
         (long long)NBLK, gb);
  printf("(a) fp32 atomic adds, 4 per element        %8.3f ms  (%.2f TB/s of added bytes)\n", ta, NBLK * gb / ta);
  printf("(b) 4 fp32 partials stored + summed         %8.3f + %.3f = %.3f ms\n", tb1, tb2, tb1 + tb2);
  printf("(c) 4 bf16 partials stored + summed         %8.3f + %.3f = %.3f ms\n", tc1, tc2, tc1 + tc2);
  return 0;
}

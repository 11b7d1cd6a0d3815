// Issue-rate and latency probe: v_max3_f32 (maxNum, drops NaN) against v_maximum3_f32 (IEEE
// 754-2019 maximum, propagates NaN; gfx950) and v_max_f32: 8 independent chains per lane (issue
// rate) or one dependent chain (latency), 4096 steps, one wave per SIMD in the latency case.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/probe_maximum3.hip -o /tmp/probe_max
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int OP, int CH>
__global__ __launch_bounds__(256) void k(float *out, float seed) {
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = seed + threadIdx.x + i;
  const float b = seed * 0.5f, c = seed * 0.25f;
  for (int it = 0; it < 4096 * 8 / CH; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if constexpr (OP == 0) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(b), "v"(c));
      else if constexpr (OP == 1) asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(b), "v"(c));
      else asm volatile("v_max_f32 %0, %0, %1" : "+v"(v[i]) : "v"(b));
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float *d;
  const int nb = 256 * 8;
  hipMalloc(&d, nb * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char *names[3] = {"v_max3_f32", "v_maximum3_f32", "v_max_f32"};
  for (int rep = 0; rep < 2; ++rep)
    for (int lat = 0; lat < 2; ++lat)
      for (int op = 0; op < 3; ++op) {
        const int g = lat ? 256 : nb;   // latency: one 4-wave block per CU, one wave per SIMD
        hipEventRecord(a);
        if (!lat) {
          if (op == 0) hipLaunchKernelGGL((k<0, 8>), dim3(g), dim3(256), 0, 0, d, 1.f);
          if (op == 1) hipLaunchKernelGGL((k<1, 8>), dim3(g), dim3(256), 0, 0, d, 1.f);
          if (op == 2) hipLaunchKernelGGL((k<2, 8>), dim3(g), dim3(256), 0, 0, d, 1.f);
        } else {
          if (op == 0) hipLaunchKernelGGL((k<0, 1>), dim3(g), dim3(256), 0, 0, d, 1.f);
          if (op == 1) hipLaunchKernelGGL((k<1, 1>), dim3(g), dim3(256), 0, 0, d, 1.f);
          if (op == 2) hipLaunchKernelGGL((k<2, 1>), dim3(g), dim3(256), 0, 0, d, 1.f);
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double inst = (double)g * 4 * 4096 * 8;   // wave-instructions (4 waves per block)
        // cycles per wave-instruction per SIMD at 2.4 GHz: 1024 SIMDs
        printf("%-16s %s %.3f ms  %.2f cyc/wave-instr/SIMD (2.4 GHz)\n", names[op], lat ? "dependent  " : "independent",
               ms, ms * 1e-3 * 2.4e9 * 1024 / inst);
      }
  return 0;
}

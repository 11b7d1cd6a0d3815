// Probe: where does an LDS-DMA load with an instruction offset land?  One wave issues
// global_load_lds_dwordx4 (and buffer_load_dwordx4 ... lds) with M0 = the LDS base, per-lane
// voffset = 16 * lane and offset:1024, from a source whose dword i holds i; the kernel then copies
// the whole 8-KB LDS image out (mode 2: M0 2 KB ahead and offset:-1024).  Build: hipcc --offload-arch=gfx950 -O2 -o probe_lds_dma_offset
// probe_lds_dma_offset.hip; run on the GPU box; it prints the first landed dword and its source.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int su32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

__global__ void probe(const unsigned *src, unsigned *out, int mode) {
  __shared__ __attribute__((aligned(16))) unsigned lds[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = 0xFFFFFFFFu;
  __syncthreads();
  const unsigned m0v = (unsigned)(uintptr_t)(lds_void_t *)lds;
  const unsigned voff = 16u * threadIdx.x;
  if (mode == 0) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 offset:1024\n\ts_waitcnt vmcnt(0)"
                 :: "v"(voff), "s"(src), "s"(m0v) : "memory");
  } else if (mode == 2) {   // M0 one piece ahead, a negative offset back (and the source 2 KB ahead)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 offset:-1024\n\ts_waitcnt vmcnt(0)"
                 :: "v"(voff + 2048u), "s"(src), "s"(m0v + 2048u) : "memory");
  } else {
    su32x4 rs;
    const unsigned long long b = (unsigned long long)src;
    rs.x = (unsigned)b; rs.y = (unsigned)(b >> 32) & 0xffffu; rs.z = 1u << 20; rs.w = 0x00020000u;
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen offset:1024 lds\n\ts_waitcnt vmcnt(0)"
                 :: "v"(voff), "s"(rs), "s"(m0v) : "memory");
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 64) out[i] = lds[i];
}

int main() {
  std::vector<unsigned> h(1 << 18);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned)i;
  unsigned *src, *out;
  hipMalloc(&src, h.size() * 4);
  hipMalloc(&out, 2048 * 4);
  hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out, mode);
    std::vector<unsigned> o(2048);
    hipMemcpy(o.data(), out, 2048 * 4, hipMemcpyDeviceToHost);
    int first = -1, n = 0;
    for (int i = 0; i < 2048; ++i)
      if (o[i] != 0xFFFFFFFFu) { if (first < 0) first = i; ++n; }
    printf("%s: %d dwords landed, first at LDS byte %d holding source byte %u\n",
           mode == 1 ? "buffer_load_dwordx4 lds" : mode == 2 ? "global_load_lds_dwordx4 M0+2K offset:-1024" : "global_load_lds_dwordx4", n, first * 4, first >= 0 ? o[first] * 4 : 0);
  }
  return 0;
}

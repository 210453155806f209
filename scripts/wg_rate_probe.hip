// wg_rate_probe.hip — what limits one channel (workgroup) of the staged kernel at low channel counts?
// A persistent grid of G 512-thread workgroups copies 256 MiB, each thread keeping U 16-byte packs in flight
// (grid-stride over the buffer, like copyRange). Source / destination are plain device memory (hipMalloc,
// nontemporal loads / stores) or the staging slab's kind of memory (hipDeviceMallocUncached, destination
// stored with the library's buffer store sc0|sc1 = system-scope write-through). Prints GB/s of copied bytes
// (read + write) in total and per workgroup. HIP events over back-to-back launches. Diagnostics only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, -1, 0x00020000);
}

// WT: destination stores are system-scope write-through buffer stores (the library's remote-store flavour)
template <int U, bool WT>
__global__ void __launch_bounds__(512) copyK(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  const uint64_t stride = (uint64_t)gridDim.x * 512 * U;
  // 32-bit buffer offsets cover 4 GiB; the probe's buffers are 256 MiB
  __amdgpu_buffer_rsrc_t rd = rsrc(d);
  for (uint64_t i = (uint64_t)blockIdx.x * 512 * U + threadIdx.x; i + (U - 1) * 512 < npk; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(s + i + u * 512);
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (WT) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)((i + u * 512) * 16), 0, 1 | 16);
      else __builtin_nontemporal_store(v[u], d + i + u * 512);
    }
  }
}

template <int U, bool WT>
static double timeIt(u32x4* d, const u32x4* s, uint64_t npk, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL((copyK<U, WT>), dim3(grid), dim3(512), 0, 0, d, s, npk);
  const int iters = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; i++) hipLaunchKernelGGL((copyK<U, WT>), dim3(grid), dim3(512), 0, 0, d, s, npk);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / iters;
}

int main() {
  const size_t bytes = 256ull << 20;
  const uint64_t npk = bytes / 16;
  u32x4 *nS, *nD, *uS, *uD;
  CK(hipMalloc(&nS, bytes));
  CK(hipMalloc(&nD, bytes));
  CK(hipExtMallocWithFlags((void**)&uS, bytes, hipDeviceMallocUncached));
  CK(hipExtMallocWithFlags((void**)&uD, bytes, hipDeviceMallocUncached));
  CK(hipMemset(nS, 1, bytes));
  CK(hipMemset(uS, 2, bytes));
  CK(hipDeviceSynchronize());
  struct Mode { const char* name; u32x4* d; const u32x4* s; bool wt; } modes[] = {
      {"plain->plain(nt)", nD, nS, false}, {"plain->UC(wt)", uD, nS, true},
      {"UC->plain(nt)", nD, uS, false},    {"UC->UC(wt)", uD, uS, true}};
  const int grids[] = {32, 64, 128, 256, 512};
  printf("# 256 MiB copy, 512-thread workgroups, persistent grid-stride; GB/s of read+write bytes\n");
  printf("%-18s %5s %3s %10s %10s %12s\n", "mode", "grid", "U", "us", "GB/s", "GB/s per WG");
  for (const Mode& m : modes)
    for (int g : grids)
      for (int u : {8, 16}) {
        double ms = u == 8 ? (m.wt ? timeIt<8, true>(m.d, m.s, npk, g) : timeIt<8, false>(m.d, m.s, npk, g))
                           : (m.wt ? timeIt<16, true>(m.d, m.s, npk, g) : timeIt<16, false>(m.d, m.s, npk, g));
        double gbs = 2.0 * bytes / (ms * 1e-3) / 1e9;
        printf("%-18s %5d %3d %10.1f %10.1f %12.2f\n", m.name, g, u, ms * 1e3, gbs, gbs / g);
        fflush(stdout);
      }
  CK(hipFree(nS));
  CK(hipFree(nD));
  CK(hipFree(uS));
  CK(hipFree(uD));
  return 0;
}

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
template <int U, bool WT, int BS = 512>
__global__ void __launch_bounds__(BS) copyK(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  const uint64_t stride = (uint64_t)gridDim.x * BS * U;
  // 32-bit buffer offsets cover 4 GiB; the probe's buffers are 256 MiB
  __amdgpu_buffer_rsrc_t rd = rsrc(d);
  for (uint64_t i = (uint64_t)blockIdx.x * BS * U + threadIdx.x; i + (U - 1) * BS < npk; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(s + i + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (WT) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)((i + u * BS) * 16), 0, 1 | 16);
      else __builtin_nontemporal_store(v[u], d + i + u * BS);
    }
  }
}

template <int U, bool WT, int BS = 512>
static double timeIt(u32x4* d, const u32x4* s, uint64_t npk, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL((copyK<U, WT, BS>), dim3(grid), dim3(BS), 0, 0, d, s, npk);
  const int iters = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; i++) hipLaunchKernelGGL((copyK<U, WT, BS>), dim3(grid), dim3(BS), 0, 0, d, s, npk);
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
  // workgroup size at low workgroup counts (plain -> UC write-through, U = 8): is the ~50 GB/s ceiling per
  // workgroup (waves) or per CU?
  printf("# workgroup size: plain->UC(wt), U=8\n");
  for (int g : {32, 64, 128}) {
    double a = timeIt<8, true, 256>(uD, nS, npk, g), b = timeIt<8, true, 512>(uD, nS, npk, g),
           c = timeIt<8, true, 1024>(uD, nS, npk, g);
    double ga = 2.0 * bytes / (a * 1e-3) / 1e9, gb = 2.0 * bytes / (b * 1e-3) / 1e9, gc = 2.0 * bytes / (c * 1e-3) / 1e9;
    printf("grid %4d  256 thr %8.1f GB/s (%6.2f/WG)  512 thr %8.1f (%6.2f/WG)  1024 thr %8.1f (%6.2f/WG)\n", g, ga,
           ga / g, gb, gb / g, gc, gc / g);
    fflush(stdout);
  }
  CK(hipFree(nS));
  CK(hipFree(nD));
  CK(hipFree(uS));
  CK(hipFree(uD));
  return 0;
}

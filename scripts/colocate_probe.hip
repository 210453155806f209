// colocate_probe.hip — do two concurrently running kernels of G workgroups each (two streams = two hardware
// queues, like two ranks sharing the one GPU in the rehearsal) land on the same CUs? Each workgroup records
// its (XCC, SE, CU) from the HW_ID / XCC_ID registers; the host counts distinct CUs per kernel and the CUs
// both kernels used, and times one kernel alone vs both together (persistent 512-thread copy workgroups,
// 8 packs in flight per thread, 256 MiB each). Diagnostics only (scripts/).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <set>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ void __launch_bounds__(512) copyK(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk,
                                             unsigned* where) {
  constexpr int U = 8;
  if (threadIdx.x == 0) {
    // gfx9 HW_ID (hwreg 4): CU_ID bits 11:8, SH_ID bit 12, SE_ID bits 15:13; gfx940+ XCC_ID (hwreg 20) bits 3:0
    unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));
    where[blockIdx.x] = (xcc << 16) | ((hw >> 8) & 0xff);
  }
  const uint64_t stride = (uint64_t)gridDim.x * 512 * U;
  for (uint64_t i = (uint64_t)blockIdx.x * 512 * U + threadIdx.x; i + (U - 1) * 512 < npk; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(s + i + u * 512);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(v[u], d + i + u * 512);
  }
}

int main() {
  const size_t bytes = 256ull << 20;
  const uint64_t npk = bytes / 16;
  u32x4 *s[2], *d[2];
  unsigned* where[2];
  hipStream_t st[2];
  for (int k = 0; k < 2; k++) {
    CK(hipMalloc(&s[k], bytes));
    CK(hipMalloc(&d[k], bytes));
    CK(hipMemset(s[k], k + 1, bytes));
    CK(hipMalloc(&where[k], 4096 * sizeof(unsigned)));
    CK(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int g : {32, 64, 128}) {
    // alone
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(copyK, dim3(g), dim3(512), 0, st[0], d[0], s[0], npk, where[0]);
    CK(hipStreamSynchronize(st[0]));
    auto t0 = std::chrono::steady_clock::now();
    const int iters = 10;
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL(copyK, dim3(g), dim3(512), 0, st[0], d[0], s[0], npk, where[0]);
    CK(hipStreamSynchronize(st[0]));
    double alone = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    // together: both streams, launched back to back each iteration
    for (int i = 0; i < 3; i++)
      for (int k = 0; k < 2; k++) hipLaunchKernelGGL(copyK, dim3(g), dim3(512), 0, st[k], d[k], s[k], npk, where[k]);
    CK(hipDeviceSynchronize());
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++)
      for (int k = 0; k < 2; k++) hipLaunchKernelGGL(copyK, dim3(g), dim3(512), 0, st[k], d[k], s[k], npk, where[k]);
    CK(hipDeviceSynchronize());
    double both = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    unsigned h[2][4096];
    std::set<unsigned> cu[2];
    for (int k = 0; k < 2; k++) {
      CK(hipMemcpy(h[k], where[k], g * sizeof(unsigned), hipMemcpyDeviceToHost));
      for (int i = 0; i < g; i++) cu[k].insert(h[k][i]);
    }
    int shared = 0;
    for (unsigned x : cu[0]) shared += cu[1].count(x);
    printf("grid %4d: alone %8.1f us (%7.1f GB/s)  both %8.1f us (%7.1f GB/s total)  distinct CUs k0 %zu k1 %zu, "
           "CUs used by both %d\n",
           g, alone, 2.0 * bytes / (alone * 1e-6) / 1e9, both, 4.0 * bytes / (both * 1e-6) / 1e9, cu[0].size(),
           cu[1].size(), shared);
    fflush(stdout);
  }
  return 0;
}

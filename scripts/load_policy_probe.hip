// load_policy_probe.hip — the nRanks==1 copy kernel's load side: the library's tile (256 threads x 2 packs,
// one 8 KiB tile per workgroup, sc0|sc1 write-through buffer stores) with the source read under each cache
// policy of gfx950's buffer loads (bits: sc0 = 1, nt = 2, sc1 = 16) against the library's global nontemporal
// load. 256 MiB; "same" re-reads one src/dst pair every launch (bench.py's loop: the Infinity Cache keeps part
// of the source between launches), "rot4" rotates 4 pairs (2 GiB, past the 256 MiB Infinity Cache). HIP events
// over back-to-back launches; GB/s of read + write bytes. Also the same work as ONE launch of 8x the grid over
// 8 pairs laid end to end vs 8 launches, to size the gap between back-to-back launches. Diagnostics only.
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

// LPOL < 0: global nontemporal load (the library's); else buffer load with cache policy LPOL. XCD: workgroup b
// (dispatched to XCD b % 8) copies tile (b % 8) * (grid / 8) + b / 8, so each XCD streams one contiguous eighth
// instead of every eighth tile (grid a multiple of 8).
template <int LPOL, bool XCD = false>
__global__ void __launch_bounds__(256) tileCopy(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  constexpr int U = 2;
  const uint64_t tile = XCD ? (uint64_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : blockIdx.x;
  const uint64_t t0 = tile * 256 * U;
  const uint64_t base = t0 + threadIdx.x;
  u32x4 v[U];
  __amdgpu_buffer_rsrc_t rs;
  if constexpr (LPOL >= 0) rs = rsrc(s + t0);
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + u * 256 < npk) {
      if constexpr (LPOL < 0) v[u] = __builtin_nontemporal_load(s + base + u * 256);
      else v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((threadIdx.x + u * 256) * 16), 0, LPOL);
    }
  __amdgpu_buffer_rsrc_t rd = rsrc(d + t0);
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + u * 256 < npk) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)((threadIdx.x + u * 256) * 16), 0, 17);
}

static u32x4* gS[8];
static u32x4* gD[8];

template <int LPOL, bool XCD = false>
static void run(const char* name, uint64_t npk, size_t bytes, int rot) {
  const int grid = (int)(npk / 512);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 8; i++) hipLaunchKernelGGL((tileCopy<LPOL, XCD>), dim3(grid), dim3(256), 0, 0, gD[i % rot], gS[i % rot], npk);
  const int iters = 40;
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; i++)
    hipLaunchKernelGGL((tileCopy<LPOL, XCD>), dim3(grid), dim3(256), 0, 0, gD[i % rot], gS[i % rot], npk);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= iters;
  printf("%-5s %-40s %9.2f us %9.1f GB/s\n", rot == 1 ? "same" : "rot4", name, ms * 1e3, 2.0 * bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

// 8 launches over the 8 pairs vs one launch over all of them (the pairs are one allocation each side)
static void gap(u32x4* S, u32x4* D, uint64_t npk) {
  const int grid = (int)(npk / 512);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best8 = 1e30f, best1 = 1e30f;
  for (int rep = 0; rep < 6; rep++) {
    float ms = 0;
    CK(hipEventRecord(a));
    for (int i = 0; i < 8; i++) hipLaunchKernelGGL((tileCopy<-1>), dim3(grid), dim3(256), 0, 0, D + i * npk, S + i * npk, npk);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) best8 = ms < best8 ? ms : best8;
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((tileCopy<-1>), dim3(grid * 8), dim3(256), 0, 0, D, S, npk * 8);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) best1 = ms < best1 ? ms : best1;
  }
  printf("gap   8 launches x 256 MiB %9.2f us   1 launch x 2 GiB %9.2f us   per-launch difference %6.2f us\n",
         best8 * 1e3, best1 * 1e3, (best8 - best1) * 1e3 / 8);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

static bool check(uint64_t npk, int i) {
  const size_t bytes = npk * 16;
  unsigned *h1 = (unsigned*)malloc(bytes), *h2 = (unsigned*)malloc(bytes);
  CK(hipMemcpy(h1, gS[i], bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2, gD[i], bytes, hipMemcpyDeviceToHost));
  bool ok = true;
  for (size_t k = 0; k < bytes / 4 && ok; k++) ok = h1[k] == h2[k];
  free(h1);
  free(h2);
  return ok;
}

int main() {
  const size_t bytes = 256ull << 20;
  const uint64_t npk = bytes / 16;
  u32x4 *S, *D;
  CK(hipMalloc(&S, bytes * 8));
  CK(hipMalloc(&D, bytes * 8));
  for (int i = 0; i < 8; i++) {
    gS[i] = S + i * npk;
    gD[i] = D + i * npk;
    CK(hipMemset(gS[i], 0x10 + i, bytes));
  }
  CK(hipDeviceSynchronize());
  printf("# 256 MiB copy, 256 threads x 2 packs (8 KiB tile per workgroup), sc0|sc1 write-through buffer stores\n");
  for (int rot : {1, 4}) {
    run<-1>("global nt load (library)", npk, bytes, rot);
    run<0>("buffer load pol 0", npk, bytes, rot);
    run<2>("buffer load nt", npk, bytes, rot);
    run<1>("buffer load sc0", npk, bytes, rot);
    run<3>("buffer load sc0 nt", npk, bytes, rot);
    run<16>("buffer load sc1", npk, bytes, rot);
    run<18>("buffer load sc1 nt", npk, bytes, rot);
    run<17>("buffer load sc0 sc1", npk, bytes, rot);
    run<19>("buffer load sc0 sc1 nt", npk, bytes, rot);
    run<-1, true>("global nt load, XCD-contiguous tiles", npk, bytes, rot);
    run<-1>("global nt load (library)", npk, bytes, rot);
  }
  gap(S, D, npk);
  bool ok = check(npk, 0) && check(npk, 3);
  printf("check %s\n", ok ? "ok" : "FAILED");
  return ok ? 0 : 1;
}

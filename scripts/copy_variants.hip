// copy_variants.hip — microbenchmark of streaming-copy variants for the nRanks==1 path (256 MiB),
// HIP events over back-to-back launches. Diagnostics only (scripts/), not part of the library.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid-stride, U packs per lane in flight (the library's copyKernel)
template <int BS, int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) gridStride(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  uint64_t stride = (uint64_t)gridDim.x * BS * U;
  for (uint64_t base = (uint64_t)blockIdx.x * BS * U + threadIdx.x; base < npk; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * BS < npk) v[u] = NTL ? __builtin_nontemporal_load(s + base + u * BS) : s[base + u * BS];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * BS < npk) {
        if (NTS) __builtin_nontemporal_store(v[u], d + base + u * BS);
        else d[base + u * BS] = v[u];
      }
  }
}

// contiguous span per block (each block walks its own [lo,hi) range)
template <int BS, int U>
__global__ void __launch_bounds__(BS) spans(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  uint64_t per = (npk + gridDim.x - 1) / gridDim.x;
  uint64_t lo = blockIdx.x * per, hi = lo + per < npk ? lo + per : npk;
  for (uint64_t base = lo + threadIdx.x; base < hi; base += BS * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * BS < hi) v[u] = __builtin_nontemporal_load(s + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * BS < hi) __builtin_nontemporal_store(v[u], d + base + u * BS);
  }
}

// software-pipelined: loads of tile i+1 issued before the stores of tile i
template <int BS, int U>
__global__ void __launch_bounds__(BS) pipelined(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  uint64_t stride = (uint64_t)gridDim.x * BS * U;
  uint64_t base = (uint64_t)blockIdx.x * BS * U + threadIdx.x;
  u32x4 cur[U], nxt[U];
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + u * BS < npk) cur[u] = __builtin_nontemporal_load(s + base + u * BS);
  for (; base < npk; base += stride) {
    uint64_t nb = base + stride;
#pragma unroll
    for (int u = 0; u < U; u++)
      if (nb + u * BS < npk) nxt[u] = __builtin_nontemporal_load(s + nb + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * BS < npk) __builtin_nontemporal_store(cur[u], d + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) cur[u] = nxt[u];
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

static u32x4* gS[4];
static u32x4* gD[4];
static int gRot = 1;  // 1: same buffers every launch; 4: rotate over 4 pairs (2 GiB, defeats the 256 MiB MALL)

template <typename K>
static void run(const char* name, K kern, int grid, int bs, u32x4* d, const u32x4* s, uint64_t npk, size_t bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), 0, 0, gD[i % gRot], gS[i % gRot], npk);
  CK(hipDeviceSynchronize());
  const int it = 50;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < it; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), 0, 0, gD[i % gRot], gS[i % gRot], npk);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= it;
  printf("rot%d %-34s grid %6d  %8.2f us  %7.1f GB/s\n", gRot, name, grid, ms * 1e3, 2.0 * bytes / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t bytes = 256ull << 20;
  const uint64_t npk = bytes / 16;
  u32x4 *s, *d;
  for (int i = 0; i < 4; i++) {
    CK(hipMalloc(&gS[i], bytes));
    CK(hipMalloc(&gD[i], bytes));
    CK(hipMemset(gS[i], 1, bytes));
  }
  s = gS[0];
  d = gD[0];
  for (int rot : {1, 4}) {
    gRot = rot;
    for (int g : {2048, 4096}) run("gridStride<256,4,nt,nt> (library)", gridStride<256, 4, true, true>, g, 256, d, s, npk, bytes);
    for (int g : {1024, 2048, 4096}) run("gridStride<256,4,plain,nt>", gridStride<256, 4, false, true>, g, 256, d, s, npk, bytes);
    for (int g : {2048, 4096}) run("gridStride<256,4,plain,plain>", gridStride<256, 4, false, false>, g, 256, d, s, npk, bytes);
    for (int g : {2048, 4096}) run("gridStride<256,4,nt,plain>", gridStride<256, 4, true, false>, g, 256, d, s, npk, bytes);
    for (int g : {2048}) run("gridStride<256,8,plain,nt>", gridStride<256, 8, false, true>, g, 256, d, s, npk, bytes);
    for (int g : {16384, 32768}) run("gridStride<256,4,plain,nt> 1 tile", gridStride<256, 4, false, true>, g, 256, d, s, npk, bytes);
    for (int g : {16384, 32768}) run("gridStride<256,4,nt,nt> 1 tile", gridStride<256, 4, true, true>, g, 256, d, s, npk, bytes);
  }
  return 0;
}

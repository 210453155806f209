// copy_variants2.hip — round-2 microbenchmark of the nRanks==1 streaming copy (256 MiB): the library's
// one-tile-per-workgroup kernel against wider tiles, more threads, an XCD-contiguous tile order and an
// LDS-DMA (global_load_lds_dwordx4) load path. HIP events over back-to-back launches; buffers rotated over
// 4 pairs (2 GiB, past the 256 MiB Infinity Cache) unless noted. Diagnostics only (scripts/).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

// one tile of BS*U 16-byte packs per workgroup (the library's copyKernel with grid = tiles); XCD: workgroup
// b runs on XCD b % 8, so tile = (b % 8) * (G / 8) + b / 8 gives each XCD one contiguous eighth of the buffer
template <int BS, int U, bool XCD>
__global__ void __launch_bounds__(BS) tileCopy(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  uint64_t t = blockIdx.x;
  if (XCD) {
    const uint64_t g8 = gridDim.x / 8;
    t = (blockIdx.x % 8) * g8 + blockIdx.x / 8;
  }
  const uint64_t base = t * BS * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + u * BS < npk) v[u] = __builtin_nontemporal_load(s + base + u * BS);
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + u * BS < npk) __builtin_nontemporal_store(v[u], d + base + u * BS);
}

// LDS-DMA: every wave loads its U KiB straight into LDS (no VGPR destination), waits, reads LDS back and
// stores nontemporally. Same tile as tileCopy<256,U>.
template <int U>
__global__ void __launch_bounds__(256) ldsCopy(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  __shared__ u32x4 buf[256 * U];
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U;
  const int w = threadIdx.x / 64, lane = threadIdx.x % 64;
#pragma unroll
  for (int u = 0; u < U; u++) {
    // wave w, step u: packs base + (u * 4 + w) * 64 + lane -> LDS slot (u * 4 + w) * 64 + lane
    const uint64_t i = base + (uint64_t)(u * 4 + w) * 64 + lane;
    __builtin_amdgcn_global_load_lds((const void*)(s + i), (__attribute__((address_space(3))) void*)(buf + (u * 4 + w) * 64),
                                     16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int slot = (u * 4 + w) * 64 + lane;
    __builtin_nontemporal_store(buf[slot], d + base + slot);
  }
}

static u32x4* gS[4];
static u32x4* gD[4];
static int gRot = 4;

template <typename K>
static void run(const char* name, K kern, int grid, int bs, uint64_t npk, size_t bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 8; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), 0, 0, gD[i % gRot], gS[i % gRot], npk);
  CK(hipDeviceSynchronize());
  const int it = 60;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < it; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), 0, 0, gD[i % gRot], gS[i % gRot], npk);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= it;
  printf("rot%d %-40s grid %6d  %8.2f us  %7.1f GB/s\n", gRot, name, grid, ms * 1e3, 2.0 * bytes / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t bytes = 256ull << 20;
  const uint64_t npk = bytes / 16;
  for (int i = 0; i < 4; i++) {
    CK(hipMalloc(&gS[i], bytes));
    CK(hipMalloc(&gD[i], bytes));
    CK(hipMemset(gS[i], i + 1, bytes));
  }
  for (int rep = 0; rep < 2; rep++) {
    run("tile<256,4> (library)", tileCopy<256, 4, false>, (int)(npk / 1024), 256, npk, bytes);
    run("tile<256,4> XCD-contiguous", tileCopy<256, 4, true>, (int)(npk / 1024), 256, npk, bytes);
    run("tile<256,8>", tileCopy<256, 8, false>, (int)(npk / 2048), 256, npk, bytes);
    run("tile<512,4>", tileCopy<512, 4, false>, (int)(npk / 2048), 512, npk, bytes);
    run("tile<512,4> XCD-contiguous", tileCopy<512, 4, true>, (int)(npk / 2048), 512, npk, bytes);
    run("tile<1024,2>", tileCopy<1024, 2, false>, (int)(npk / 2048), 1024, npk, bytes);
    run("tile<256,2>", tileCopy<256, 2, false>, (int)(npk / 512), 256, npk, bytes);
    run("lds-dma<4>", ldsCopy<4>, (int)(npk / 1024), 256, npk, bytes);
    run("lds-dma<8>", ldsCopy<8>, (int)(npk / 2048), 256, npk, bytes);
  }
  // check the last lds-dma copy (every rotation slot was written by it with its own source byte)
  unsigned char h[16];
  for (int i = 0; i < 4; i++) {
    CK(hipMemcpy(h, (char*)gD[i] + bytes - 16, 16, hipMemcpyDeviceToHost));
    if (h[0] != (unsigned char)(i + 1)) { printf("lds-dma copy wrong in slot %d\n", i); return 1; }
  }
  printf("check ok\n");
  return 0;
}

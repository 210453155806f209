// copy_shape_probe.hip — (derived from copy_policy_probe.hip) tile shapes of the nRanks==1 copy with the
// write-through store: threads per workgroup x packs per thread, and a grid-stride form. Below: the original
// description of the policy probe.
// copy_policy_probe.hip — the nRanks==1 copy kernel (256-thread workgroups, 4 packs per thread, one 16 KiB
// tile per workgroup: the library's copyKernel) with the destination written under each store cache policy
// of gfx950's buffer stores (bits: sc0 = 1, nt = 2, sc1 = 16) against the library's global nontemporal
// store, and the source read nontemporally or plainly. 256 MiB; "same" re-reads one src/dst pair every
// launch (bench.py's loop), "rot4" rotates 4 pairs (2 GiB, past the 256 MiB Infinity Cache). HIP events over
// back-to-back launches; GB/s of read + write bytes. Diagnostics only (scripts/).
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

// POL < 0: global nontemporal store (the library's); else buffer store with cache policy POL.
// The tile's byte offsets are taken from the workgroup's own base (32-bit offsets: a tile is 16 KiB).
template <int BS, int U, int POL>
__global__ void __launch_bounds__(BS) tileCopy(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t npk) {
  const uint64_t stride = (uint64_t)gridDim.x * BS * U;
  for (uint64_t t0 = (uint64_t)blockIdx.x * BS * U; t0 < npk; t0 += stride) {
    const uint64_t base = t0 + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * BS < npk) v[u] = __builtin_nontemporal_load(s + base + u * BS);
    __amdgpu_buffer_rsrc_t rd = rsrc(d + t0);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * BS < npk) {
        if (POL < 0) __builtin_nontemporal_store(v[u], d + base + u * BS);
        else __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)((threadIdx.x + u * BS) * 16), 0, POL);
      }
  }
}

static u32x4* gS[4];
static u32x4* gD[4];

template <int BS, int U, int POL>
static void run(const char* name, uint64_t npk, size_t bytes, int rot, int gridCap = 0) {
  int grid = (int)(npk / (BS * U));
  if (gridCap > 0 && grid > gridCap) grid = gridCap;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 8; i++) hipLaunchKernelGGL((tileCopy<BS, U, POL>), dim3(grid), dim3(BS), 0, 0, gD[i % rot], gS[i % rot], npk);
  const int iters = 40;
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; i++)
    hipLaunchKernelGGL((tileCopy<BS, U, POL>), dim3(grid), dim3(BS), 0, 0, gD[i % rot], gS[i % rot], npk);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= iters;
  printf("%-5s %-40s grid %6d %9.2f us %9.1f GB/s\n", rot == 1 ? "same" : "rot4", name, grid, ms * 1e3,
         2.0 * bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

static bool check(uint64_t npk) {
  // the last variant run wrote gD[0] from gS[0] for every rotation; compare the words
  const size_t bytes = npk * 16;
  unsigned *h1 = (unsigned*)malloc(bytes), *h2 = (unsigned*)malloc(bytes);
  CK(hipMemcpy(h1, gS[0], bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2, gD[0], bytes, hipMemcpyDeviceToHost));
  bool ok = true;
  for (size_t i = 0; i < bytes / 4 && ok; i++) ok = h1[i] == h2[i];
  free(h1);
  free(h2);
  return ok;
}

int main() {
  const size_t bytes = 256ull << 20;
  const uint64_t npk = bytes / 16;
  for (int i = 0; i < 4; i++) {
    CK(hipMalloc(&gS[i], bytes));
    CK(hipMalloc(&gD[i], bytes));
    CK(hipMemset(gS[i], 0x10 + i, bytes));
  }
  CK(hipDeviceSynchronize());
  printf("# 256 MiB copy with write-through (sc0 sc1) buffer stores: tile shapes\n");
  for (int rot : {1, 4}) {
    run<256, 4, 17>("256 thr x 4 packs (library)", npk, bytes, rot);
    run<256, 2, 17>("256 thr x 2 packs", npk, bytes, rot);
    run<256, 8, 17>("256 thr x 8 packs", npk, bytes, rot);
    run<512, 2, 17>("512 thr x 2 packs", npk, bytes, rot);
    run<512, 4, 17>("512 thr x 4 packs", npk, bytes, rot);
    run<1024, 2, 17>("1024 thr x 2 packs", npk, bytes, rot);
    run<128, 4, 17>("128 thr x 4 packs", npk, bytes, rot);
    run<64, 8, 17>("64 thr x 8 packs", npk, bytes, rot);
    run<256, 4, 17>("256 thr x 4, grid-stride 4096", npk, bytes, rot, 4096);
    run<256, 4, 17>("256 thr x 4, grid-stride 2048", npk, bytes, rot, 2048);
    run<256, 4, -1>("256 thr x 4, global nt store", npk, bytes, rot);
    run<256, 4, 17>("256 thr x 4 packs (library)", npk, bytes, rot);
  }
  bool ok = check(npk);
  printf("check %s\n", ok ? "ok" : "FAILED");
  return ok ? 0 : 1;
}

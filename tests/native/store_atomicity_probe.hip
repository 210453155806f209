// store_atomicity_probe.hip — does a reader ever see a torn line? (the reference gates LL128
// on 128-byte store atomicity, src/graph/tuning.cc:518-536, and asks that the single-copy atomicity of peer
// stores over xGMI be measured before relying on more than 8 bytes.)
//
// A writer GPU stores epochs 1..E into an uncached line area on the reader GPU, exactly as the LL kernels do:
// every lane writes 16 bytes {e,e,e,e} with one system-scope write-through `global_store_dwordx4 ... sc0 sc1`,
// 64 lanes = 1 KiB = eight 128-byte lines per wave-instruction. Reader waves on the reader GPU poll the area
// with system-scope 16-byte loads (one wave-instruction per 1 KiB, like an LL128 reader) and classify every
// 128-byte line they observe:
//   torn8    an 8-byte half of a lane holds two different epochs   (the LL protocol relies on this never happening)
//   torn16   the two halves of one lane's 16 bytes differ           (16-byte single-copy atomicity)
//   torn64   lanes of one 64-byte quarter-wave segment differ       (each lane consistent)
//   torn128  the two 64-byte halves of a 128-byte line differ       (each half consistent; LL128's assumption)
// "changed" counts observations whose line differs from the previous observation of it (the reader really
// raced the writer). Both kernels are bounded (E epochs; the reader stops at epoch E everywhere or after a
// time limit), so the grid always drains.
//   store_atomicity_probe [writer_dev] [reader_dev] [epochs] [KiB] [reader_ms]
// With one GPU, writer and reader are the same device (different XCDs): local HBM, not a link.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
      exit(2);                                                                                  \
    }                                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

enum { C_OBS = 0, C_CHANGED, C_TORN8, C_TORN16, C_TORN64, C_TORN128, C_DONE_WAVES, C_KINDS };

// Each writer wave owns 1 KiB blocks w, w + nWaves, ...; epochs advance block by block.
__global__ void __launch_bounds__(256) writer(u32x4* area, uint64_t nBlocks, uint32_t epochs) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const uint64_t nWaves = (uint64_t)gridDim.x * blockDim.x / 64;
  const int lane = threadIdx.x & 63;
  for (uint32_t e = 1; e <= epochs; e++) {
    for (uint64_t b = wave; b < nBlocks; b += nWaves) {
      u32x4 v = {e, e, e, e};
      u32x4* p = area + b * 64 + lane;
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ u32x4 loadSys(const u32x4* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// Reader wave r polls blocks r, r + nWaves, ... until every one shows `epochs` or the time limit passes.
__global__ void __launch_bounds__(256) reader(const u32x4* area, uint64_t nBlocks, uint32_t epochs,
                                              unsigned long long* cnt, uint64_t limitTicks) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const uint64_t nWaves = (uint64_t)gridDim.x * blockDim.x / 64;
  const int lane = threadIdx.x & 63;
  unsigned long long obs = 0, changed = 0, t8 = 0, t16 = 0, t64 = 0, t128 = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t prev[4] = {0, 0, 0, 0};  // last value this lane saw in its first four blocks
  bool finished = false;
  while (!finished) {
    bool all = true;
    int k = 0;
    for (uint64_t b = wave; b < nBlocks; b += nWaves, k++) {
      const u32x4 v = loadSys(area + b * 64 + lane);
      const bool h0 = v.x == v.y, h1 = v.z == v.w;
      const bool lane16 = h0 && h1 && v.x == v.z;
      const uint32_t mine = v.x;
      // line-level classification on lane 0 of each line (lanes 8j .. 8j+7 hold 128-byte line j; lanes
      // 8j .. 8j+3 and 8j+4 .. 8j+7 its two 64-byte halves)
      const uint32_t segHead = __shfl(mine, lane & ~3);
      const unsigned long long okLane = __ballot(lane16);
      const unsigned long long sameSeg = __ballot(lane16 && mine == segHead);
      const uint32_t lineHead = __shfl(mine, lane & ~7);
      const uint32_t otherHalf = __shfl(mine, (lane & ~7) | 4);
      if ((lane & 7) == 0) {
        obs++;
        const unsigned long long lm = 0xffull << (lane & ~7);
        const bool lanesOk = (okLane & lm) == lm;        // no lane of the line is internally torn
        const bool segsOk = (sameSeg & lm) == lm;        // each 64-byte half holds one epoch
        if (lanesOk && !segsOk) t64++;
        if (lanesOk && segsOk && lineHead != otherHalf) t128++;
      }
      // per-lane internal tearing, counted on the lane itself
      if (!h0 || !h1) t8++;
      else if (v.x != v.z) t16++;
      if (k < 4) {
        if ((lane & 7) == 0 && prev[k] != mine) changed++;
        prev[k] = mine;
      }
      all = all && __all(lane16 && mine == epochs);
    }
    finished = all || (__builtin_amdgcn_s_memrealtime() - t0 > limitTicks);
  }
  atomicAdd(cnt + C_OBS, obs);
  atomicAdd(cnt + C_CHANGED, changed);
  atomicAdd(cnt + C_TORN8, t8);
  atomicAdd(cnt + C_TORN16, t16);
  atomicAdd(cnt + C_TORN64, t64);
  atomicAdd(cnt + C_TORN128, t128);
  if (lane == 0) atomicAdd(cnt + C_DONE_WAVES, 1ull);
}

int main(int argc, char** argv) {
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  const int wdev = argc > 1 ? atoi(argv[1]) : (ndev > 1 ? 1 : 0);
  const int rdev = argc > 2 ? atoi(argv[2]) : 0;
  const uint32_t epochs = argc > 3 ? (uint32_t)atoi(argv[3]) : 20000;
  const uint64_t kib = argc > 4 ? strtoull(argv[4], nullptr, 0) : 64;
  const double readerMs = argc > 5 ? atof(argv[5]) : 3000.0;
  if (wdev >= ndev || rdev >= ndev || kib == 0 || kib > (1 << 20)) {
    printf("{\"error\": \"bad arguments: %d GPUs, writer %d, reader %d, %llu KiB\"}\n", ndev, wdev, rdev,
           (unsigned long long)kib);
    return 1;
  }
  const uint64_t nBlocks = kib;  // 1 KiB per block
  CK(hipSetDevice(rdev));
  u32x4* area = nullptr;
  CK(hipExtMallocWithFlags((void**)&area, nBlocks * 1024, hipDeviceMallocUncached));
  CK(hipMemset(area, 0, nBlocks * 1024));
  unsigned long long* cnt = nullptr;
  CK(hipMalloc(&cnt, C_KINDS * sizeof(unsigned long long)));
  CK(hipMemset(cnt, 0, C_KINDS * sizeof(unsigned long long)));
  CK(hipDeviceSynchronize());
  if (wdev != rdev) {
    CK(hipSetDevice(wdev));
    hipError_t e = hipDeviceEnablePeerAccess(rdev, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) CK(e);
  }
  hipStream_t rs, ws;
  CK(hipSetDevice(rdev));
  CK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
  CK(hipSetDevice(wdev));
  CK(hipStreamCreateWithFlags(&ws, hipStreamNonBlocking));
  // reader: 16 workgroups x 4 waves; writer: 8 workgroups x 4 waves (blocks interleaved across waves)
  const uint64_t limitTicks = (uint64_t)(readerMs * 1e5);  // s_memrealtime runs at 100 MHz
  CK(hipSetDevice(rdev));
  hipEvent_t r0, r1;
  CK(hipEventCreate(&r0));
  CK(hipEventCreate(&r1));
  CK(hipEventRecord(r0, rs));
  hipLaunchKernelGGL(reader, dim3(16), dim3(256), 0, rs, (const u32x4*)area, nBlocks, epochs, cnt, limitTicks);
  CK(hipGetLastError());
  CK(hipEventRecord(r1, rs));
  CK(hipSetDevice(wdev));
  hipLaunchKernelGGL(writer, dim3(8), dim3(256), 0, ws, area, nBlocks, epochs);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ws));
  CK(hipSetDevice(rdev));
  CK(hipStreamSynchronize(rs));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, r0, r1));
  unsigned long long h[C_KINDS];
  CK(hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost));
  printf("{\"writer_dev\": %d, \"reader_dev\": %d, \"link\": %s, \"epochs\": %u, \"area_KiB\": %llu, "
         "\"reader_ms\": %.1f, \"line_observations\": %llu, \"changed\": %llu, \"torn8\": %llu, \"torn16\": %llu, "
         "\"torn64\": %llu, \"torn128\": %llu, \"reader_waves\": %llu, \"completed\": %s}\n",
         wdev, rdev, wdev != rdev ? "true" : "false", epochs, (unsigned long long)kib, ms, h[C_OBS], h[C_CHANGED],
         h[C_TORN8], h[C_TORN16], h[C_TORN64], h[C_TORN128], h[C_DONE_WAVES], ms < readerMs * 0.99 ? "true" : "false");
  CK(hipFree(cnt));
  CK(hipFree(area));
  return 0;
}

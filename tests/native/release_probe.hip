// release_probe.hip — does unmapping an imported dma-buf mapping wait for the device?
//
// A peer's registered buffer is mapped here by hipImportExternalMemory + hipExternalMemoryGetMappedBuffer (ipc.cc
// importFd) and unmapped by hipFree + hipDestroyExternalMemory (ipcRelease). If the unmap waits for this process's
// device work, it may not run inside a collective's enqueue (a queued kernel may wait on a peer that waits for us);
// if it returns at once, it can. This probe maps an allocation of its own (the same runtime calls as a peer's), keeps
// a kernel spinning for SPIN_MS on a non-blocking stream, and times each release call on the host while it spins. It
// also reports whether the exporter's memory comes back (hipMemGetInfo) once the exporter frees it and the mapping is
// gone, the memory-pinning question of test_eager_registration_memory_pinning.
//
//   release_probe [SPIN_MS=300] [MiB=512]   prints one JSON line
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <chrono>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void spin(uint64_t ticks, uint32_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(10);
    t = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)(t - t0);  // vector store
}

static double msSince(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const double spinMs = argc > 1 ? atof(argv[1]) : 300.0;
  const size_t bytes = (size_t)(argc > 2 ? atol(argv[2]) : 512) << 20;
  CHECK(hipSetDevice(0));
  size_t free0 = 0, total = 0;
  CHECK(hipMemGetInfo(&free0, &total));
  void* buf = nullptr;
  CHECK(hipMalloc(&buf, bytes));
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&out, 4096));
  int fd = -1;
  CHECK(hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)buf, bytes, hipMemRangeHandleTypeDmaBufFd, 0));
  hipExternalMemoryHandleDesc hd = {};
  hd.type = hipExternalMemoryHandleTypeOpaqueFd;
  hd.handle.fd = fd;
  hd.size = bytes;
  hipExternalMemory_t em = nullptr;
  CHECK(hipImportExternalMemory(&em, &hd));
  hipExternalMemoryBufferDesc bd = {};
  bd.size = bytes;
  void* mapped = nullptr;
  CHECK(hipExternalMemoryGetMappedBuffer(&mapped, em, &bd));
  CHECK(hipMemset(mapped, 0, 4096));  // the mapping works
  CHECK(hipDeviceSynchronize());

  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const uint64_t ticks = (uint64_t)(spinMs * 1e5);  // s_memrealtime: 100 MHz
  // the owner side frees its allocation while the kernel runs (what a training loop does between steps)
  auto t0 = std::chrono::steady_clock::now();
  hipLaunchKernelGGL(spin, dim3(4), dim3(64), 0, s, ticks, out);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(ev, s));
  const double launchMs = msSince(t0);
  auto tq = std::chrono::steady_clock::now();
  const hipError_t q0 = hipEventQuery(ev);
  const double queryMs = msSince(tq);
  auto tf = std::chrono::steady_clock::now();
  const hipError_t eFree = hipFree(mapped);
  const double freeMs = msSince(tf);
  auto td = std::chrono::steady_clock::now();
  const hipError_t eDestroy = hipDestroyExternalMemory(em);
  const double destroyMs = msSince(td);
  close(fd);
  const hipError_t q1 = hipEventQuery(ev);
  const double afterReleaseMs = msSince(t0);
  auto to = std::chrono::steady_clock::now();
  const hipError_t eOwnerFree = hipFree(buf);
  const double ownerFreeMs = msSince(to);
  const double ownerFreeDoneMs = msSince(t0);
  CHECK(hipStreamSynchronize(s));
  const double kernelDoneMs = msSince(t0);
  size_t free1 = 0;
  CHECK(hipMemGetInfo(&free1, &total));
  printf("{\"spin_ms\": %.1f, \"MiB\": %zu, \"launch_ms\": %.3f, \"event_query_ms\": %.4f, \"event_busy_before\": %s, "
         "\"unmap_hipFree_ms\": %.3f, \"unmap_hipFree_rc\": %d, \"destroyExternalMemory_ms\": %.3f, \"destroy_rc\": %d, "
         "\"event_busy_after_unmap\": %s, \"unmap_done_at_ms\": %.3f, \"owner_hipFree_ms\": %.3f, \"owner_free_rc\": %d, "
         "\"owner_free_done_at_ms\": %.3f, \"kernel_done_at_ms\": %.3f, \"unmap_waited_for_kernel\": %s, "
         "\"free_before_MiB\": %.1f, \"free_after_MiB\": %.1f}\n",
         spinMs, bytes >> 20, launchMs, queryMs, q0 == hipErrorNotReady ? "true" : "false", freeMs, (int)eFree,
         destroyMs, (int)eDestroy, q1 == hipErrorNotReady ? "true" : "false", afterReleaseMs, ownerFreeMs,
         (int)eOwnerFree, ownerFreeDoneMs, kernelDoneMs, afterReleaseMs > 0.8 * spinMs ? "true" : "false",
         free0 / 1048576.0, free1 / 1048576.0);
  return 0;
}

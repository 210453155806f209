// queue_probe.hip — do two HIP streams of one process run kernels concurrently?
// Kernel `waiter` spins (bounded: 0.5 s) on a flag that kernel `setter` (launched later, on another
// stream) sets. If both streams share one hardware queue the waiter times out. Prints one line per
// stream pair. Diagnostics only (scripts/), not part of the library.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void waiter(unsigned* flag, unsigned* result) {
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {  // 0.5 s at 100 MHz
      *result = 2;
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  *result = 1;
}
__global__ void setter(unsigned* flag) { __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      return 1;                                                            \
    }                                                                      \
  } while (0)

static int probe(hipStream_t a, hipStream_t b, unsigned* flag, unsigned* res, const char* what) {
  CK(hipMemset(flag, 0, 4));
  CK(hipMemset(res, 0, 4));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, a, flag, res);
  hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, b, flag);
  CK(hipDeviceSynchronize());
  unsigned r = 0;
  CK(hipMemcpy(&r, res, 4, hipMemcpyDeviceToHost));
  printf("%-40s %s\n", what, r == 1 ? "concurrent" : "SERIALISED");
  return 0;
}

int main() {
  unsigned *flag, *res;
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&res, 4));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<hipStream_t> plain(10);
  for (auto& s : plain) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  char buf[128];
  for (int i = 0; i < 10; i++)
    for (int j = i + 1; j < 10; j++) {
      snprintf(buf, sizeof buf, "plain[%d] -> plain[%d]", i, j);
      if (probe(plain[i], plain[j], flag, res, buf)) return 1;
    }
  std::vector<uint32_t> mask((ncu + 31) / 32, 0);
  for (int c = 0; c < ncu; c++) mask[c / 32] |= 1u << (c % 32);
  std::vector<hipStream_t> cum(4);
  for (auto& s : cum) CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      if (i == j) continue;
      snprintf(buf, sizeof buf, "cumask[%d] -> cumask[%d]", i, j);
      if (probe(cum[i], cum[j], flag, res, buf)) return 1;
    }
  for (int i = 0; i < 4; i++) {
    snprintf(buf, sizeof buf, "cumask[%d] -> plain[%d]", i, i);
    if (probe(cum[i], plain[i], flag, res, buf)) return 1;
    snprintf(buf, sizeof buf, "plain[%d] -> cumask[%d]", i, i);
    if (probe(plain[i], cum[i], flag, res, buf)) return 1;
  }
  printf("done\n");
  return 0;
}

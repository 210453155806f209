// Does a kernel launched behind another on the SAME stream start while the first is still resident? (DESIGN.md §7.2:
// the co-residency cap assumes a rank can have two generations of collectives resident at once.) Kernel A (one
// workgroup) polls a flag for at most 0.5 s of wall clock; kernel B, queued behind it on the same stream, sets the
// flag. If B runs while A is resident, A sees the flag (seen = 1) within microseconds; if the runtime orders the two
// (AQL barrier bit), A times out (seen = 0) and B runs after it. Bounded: A always returns. Prints one JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void pollA(int* flag, int* seen, unsigned long long* waited) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  int s = 0;
  while (wall_clock64() - t0 < 50000000ull) {  // 0.5 s at the 100 MHz wall clock
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) {
      s = 1;
      break;
    }
  }
  *waited = wall_clock64() - t0;
  *seen = s;
}

__global__ void setB(int* flag) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static int run(hipStream_t s, const char* name) {
  int *flag, *seen;
  unsigned long long* waited;
  if (hipMalloc(&flag, sizeof(int)) != hipSuccess || hipMalloc(&seen, sizeof(int)) != hipSuccess ||
      hipMalloc(&waited, sizeof(unsigned long long)) != hipSuccess)
    return 1;
  hipMemset(flag, 0, sizeof(int));
  hipMemset(seen, 0, sizeof(int));
  hipDeviceSynchronize();
  pollA<<<1, 64, 0, s>>>(flag, seen, waited);
  setB<<<1, 64, 0, s>>>(flag);
  if (hipStreamSynchronize(s) != hipSuccess) return 2;
  int hs = -1;
  unsigned long long hw = 0;
  hipMemcpy(&hs, seen, sizeof(int), hipMemcpyDeviceToHost);
  hipMemcpy(&hw, waited, sizeof(hw), hipMemcpyDeviceToHost);
  printf("{\"stream\": \"%s\", \"second_kernel_ran_while_first_resident\": %s, \"first_waited_us\": %.1f}\n", name,
         hs ? "true" : "false", hw / 100.0);
  hipFree(flag);
  hipFree(seen);
  hipFree(waited);
  return 0;
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int rc = run(s, "created (non-blocking)");
  rc |= run(nullptr, "null");
  hipStreamDestroy(s);
  return rc;
}

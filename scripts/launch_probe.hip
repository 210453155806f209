// launch_probe.hip — host cost and back-to-back device time of one kernel launch as a function of the
// kernel-argument size (64 B … 2 KiB), to size the LL kernel's arguments. The device is held busy by a
// spin kernel while the timed launches are queued, so "host" is the pure issue cost and "device" (events
// around the queued launches) the back-to-back execution cost. Build:
//   hipcc --offload-arch=gfx950 -O2 scripts/launch_probe.hip -o scripts/launch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

template <int B>
struct Args {
  unsigned char b[B];
};
template <int B>
__global__ void touch(Args<B> a, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[B - 1] == 7) out[0] = 1;
}

__global__ void spin(long long cycles) {
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
}

template <int B>
void probe(hipStream_t s, int* out, int grid) {
  Args<B> a = {};
  const int iters = 200;
  for (int i = 0; i < 100; i++) hipLaunchKernelGGL(touch<B>, dim3(grid), dim3(512), 0, s, a, out);
  (void)hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 100000LL * 20);  // ~20 ms at the 100 MHz wall clock
  (void)hipEventRecord(e0, s);
  auto h0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; i++) hipLaunchKernelGGL(touch<B>, dim3(grid), dim3(512), 0, s, a, out);
  double host = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count() / iters;
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("kernarg %5d B grid %3d: host %.2f us/launch, device %.2f us/launch\n", B, grid, host, ms * 1e3 / iters);
}

int main() {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  int* out;
  (void)hipMalloc(&out, 4);
  for (int grid : {1, 32}) {
    probe<64>(s, out, grid);
    probe<256>(s, out, grid);
    probe<512>(s, out, grid);
    probe<1024>(s, out, grid);
    probe<2048>(s, out, grid);
  }
  return 0;
}

// xgmi_probe.hip — CU-driven peer-to-peer bandwidth over xGMI (the roofline denominators of DESIGN §5, §7):
// GPU 0 writes to (or reads from) 1 peer and all peers at once with 16-byte vector accesses, the way the
// collective kernels move data, instead of the SDMA engines behind hipMemcpyPeer. Prints one JSON line.
//   xgmi_probe [MiB per peer (default 256)] [iterations (default 10)]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
      exit(2);                                                                                  \
    }                                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Targets {
  u32x4* dst[8];
  const u32x4* src[8];
  int n;
};

// workgroup b moves its share of pair (b % n): a grid-stride copy of `vecs` 16-byte vectors per pair, 4 vectors per
// thread in flight (loads first, then stores), as the collective kernels keep them (kernels.h kFoldUnroll)
template <bool WT>
__global__ void __launch_bounds__(512) copyPairs(Targets t, size_t vecs) {
  constexpr int U = 4;
  const int pair = blockIdx.x % t.n;
  const size_t wgPerPair = gridDim.x / t.n;
  const size_t w = blockIdx.x / t.n;
  u32x4* d = t.dst[pair];
  const u32x4* s = t.src[pair];
  for (size_t b = w * blockDim.x * U + threadIdx.x; b < vecs; b += wgPerPair * blockDim.x * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b + u * blockDim.x < vecs) v[u] = __builtin_nontemporal_load(s + b + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = b + u * blockDim.x;
      if (i >= vecs) continue;
      if (WT)  // the collective kernels' remote store: write-through at system scope (kernels.h storeRemote)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(d + i), "v"(v[u]) : "memory");
      else
        __builtin_nontemporal_store(v[u], d + i);
    }
  }
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 0) : 256;
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  // loopback (argv[3] == "loopback"): the "peers" are 3 more buffers on GPU 0 — a one-GPU self-test of
  // the kernel's indexing and of the data check, not a link measurement
  const bool loop = argc > 3 && argv[3][0] == 'l';
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  if (loop) ndev = 4;
  if (ndev < 2) {
    printf("{\"error\": \"needs 2+ GPUs, found %d\"}\n", ndev);
    return 0;
  }
  if (ndev > 8) ndev = 8;
  const size_t bytes = mib << 20;
  std::vector<void*> buf(ndev);
  std::vector<void*> ubuf(ndev, nullptr);  // uncached peer buffers, like the collective's staging slabs
  for (int d = 0; d < ndev; d++) {
    CK(hipSetDevice(loop ? 0 : d));
    CK(hipMalloc(&buf[d], bytes));
    CK(hipMemset(buf[d], d, bytes));
    CK(hipExtMallocWithFlags(&ubuf[d], bytes, hipDeviceMallocUncached));
  }
  CK(hipSetDevice(0));
  void* local2 = nullptr;
  CK(hipMalloc(&local2, bytes * (ndev - 1)));
  CK(hipMemset(local2, 0xA5, bytes * (ndev - 1)));
  for (int d = 1; d < ndev && !loop; d++) {
    hipError_t e = hipDeviceEnablePeerAccess(d, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) CK(e);
  }
  (void)hipGetLastError();
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // first: the first peer (GPU 1 + first) of the npeers consecutive ones
  auto run = [&](bool write, int npeers, bool wt = false, int first = 0, int wgs = 0) -> double {
    Targets t = {};
    t.n = npeers;
    for (int k = 0; k < npeers; k++) {
      char* mine = (char*)local2 + (size_t)k * bytes;
      const int peer = 1 + first + k;
      if (write) {
        t.src[k] = (const u32x4*)mine;
        t.dst[k] = (u32x4*)(wt ? ubuf[peer] : buf[peer]);
      } else {
        t.src[k] = (const u32x4*)buf[peer];
        t.dst[k] = (u32x4*)mine;
      }
    }
    const int grid = wgs > 0 ? (wgs < npeers ? npeers : wgs / npeers * npeers) : (2 * cus / npeers) * npeers;
    auto launch = [&]() {
      if (wt) hipLaunchKernelGGL(copyPairs<true>, dim3(grid), dim3(512), 0, s, t, bytes / 16);
      else hipLaunchKernelGGL(copyPairs<false>, dim3(grid), dim3(512), 0, s, t, bytes / 16);
    };
    launch();
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; i++) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return (double)bytes * npeers * iters / (ms * 1e-3) / 1e9;
  };
  const int all = ndev - 1;
  double w1 = run(true, 1), wa = run(true, all);
  // every byte of every written peer buffer must now hold local2's pattern (0xA5)
  size_t wrong = 0;
  std::vector<unsigned char> host(bytes);
  for (int k = 0; k < all; k++) {
    CK(hipMemcpy(host.data(), buf[1 + k], bytes, hipMemcpyDefault));
    for (size_t i = 0; i < bytes; i++) wrong += host[i] != 0xA5;
  }
  double r1 = run(false, 1), ra = run(false, all);
  // the collective's own store flavour: write-through system-scope stores into uncached peer memory
  double u1 = run(true, 1, true), ua = run(true, all, true);
  // every link of GPU 0 on its own (GPU 0 -> GPU d): the collective's store flavour and plain reads; a slow or
  // missing link shows here before it shows as a slow collective
  std::string wl = "[", rl = "[";
  char num[32];
  for (int k = 0; k < all; k++) {
    snprintf(num, sizeof(num), "%s%.1f", k ? ", " : "", run(true, 1, true, k));
    wl += num;
    snprintf(num, sizeof(num), "%s%.1f", k ? ", " : "", run(false, 1, false, k));
    rl += num;
  }
  wl += "]";
  rl += "]";
  // the fan-out in the collective's store flavour driven by 8 ... 256 workgroups of 512 threads: the rate one
  // workgroup sustains across the links (enqueue.cc linkChannelBudget assumes the local-copy ~50 GB/s)
  std::string gw = "{";
  int first = 1;
  for (int g : {8, 16, 32, 64, 128, 256}) {
    snprintf(num, sizeof(num), "%s\"%d\": %.1f", first ? "" : ", ", g, run(true, all, true, 0, g));
    gw += num;
    first = 0;
  }
  gw += "}";
  printf("{\"method\": \"CU copy kernel on GPU 0, 16-byte nontemporal vectors, %zu MiB per peer, %d iters%s\", "
         "\"peers\": %d, \"write_1link_GBps\": %.1f, \"read_1link_GBps\": %.1f, \"write_fanout_GBps\": %.1f, "
         "\"read_fanin_GBps\": %.1f, \"wt_uncached_write_1link_GBps\": %.1f, \"wt_uncached_write_fanout_GBps\": %.1f, "
         "\"wt_uncached_write_per_link_GBps\": %s, \"read_per_link_GBps\": %s, "
         "\"wt_uncached_write_fanout_by_workgroups_GBps\": %s, \"wrong_bytes\": %zu}\n",
         mib, iters, loop ? ", LOOPBACK on one GPU" : "", all, w1, r1, wa, ra, u1, ua, wl.c_str(), rl.c_str(), gw.c_str(),
         wrong);
  return wrong ? 1 : 0;
}

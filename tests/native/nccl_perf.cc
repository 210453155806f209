// nccl_perf.cc — a small nccl-tests-style driver written against include/nccl.h only (the C ABI a C/C++
// caller links with -lnccl), used to check the drop-in boundary from native code and to time the
// engine without any Python on the launch path.
//
//   nccl_perf [-d ndev] [-r ranks_per_dev] [-b min_bytes] [-e max_bytes] [-f factor] [-i iters] [-w warmup]
//             [-o op: sum|max] [-t type: float|half|bf16|int] [-g 0|1 (replay a captured hipGraph)]
//             [-c coll: ar|rs|ag|reduce (root 0)] [-H 0|1 (hold: a spin kernel occupies each stream while the timed
//             collectives are issued, so host(us) is the pure issue cost; keep -i small, e.g. 100)]
//             [-G K (K collectives of `bytes` per rank in every group, on K disjoint slices of the buffers: group
//             aggregation; time(us) and host(us) are per group)]
//
// All ranks live in this process (ncclCommInitAll over ndev devices x ranks_per_dev; several ranks per
// device need NCCL_MULTI_RANK_GPU_ENABLE=1). Each rank r fills its input with (r+1), so every element of
// an AllReduce / ReduceScatter sum must be n(n+1)/2 (max: n) and AllGather block q must be q+1; the
// "#wrong" column counts mismatching elements. bytes = the AllReduce buffer, the ReduceScatter input or
// the AllGather output (nccl-tests convention). busBW = algBW * 2(n-1)/n for AllReduce, 1 for Reduce, (n-1)/n for the
// others (reference plugins/profiler/inspector/inspector.cc:1450-1492).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "nccl.h"

#define HIPCK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d HIP error %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                            \
    }                                                                                     \
  } while (0)
#define NCK(x)                                                                               \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) {                                                                 \
      fprintf(stderr, "%s:%d NCCL error %s\n", __FILE__, __LINE__, ncclGetErrorString(r_)); \
      exit(3);                                                                               \
    }                                                                                        \
  } while (0)

__global__ void fillKernel(void* p, size_t n, int type, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (type == ncclFloat32) ((float*)p)[i] = v;
    else if (type == ncclFloat16) ((__half*)p)[i] = __float2half(v);
    else if (type == ncclBfloat16) ((__hip_bfloat16*)p)[i] = __float2bfloat16(v);
    else ((int*)p)[i] = (int)v;
  }
}
__global__ void spinKernel(long long cycles) {
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
}
__global__ void checkKernel(const void* p, size_t n, int type, float want, size_t blk, unsigned long long* bad) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float v;
    if (type == ncclFloat32) v = ((const float*)p)[i];
    else if (type == ncclFloat16) v = __half2float(((const __half*)p)[i]);
    else if (type == ncclBfloat16) v = __bfloat162float(((const __hip_bfloat16*)p)[i]);
    else v = (float)((const int*)p)[i];
    local += v != (blk ? (float)(i / blk + 1) : want);
  }
  if (local) atomicAdd(bad, local);
}

int main(int argc, char** argv) {
  int ndevArg = 0, perDev = 1, iters = 20, warmup = 5, graph = 0, hold = 0, perGroup = 1;
  size_t minB = 8, maxB = 64 << 20;
  double factor = 2;
  ncclRedOp_t op = ncclSum;
  ncclDataType_t type = ncclFloat32;
  char coll = 'a';  // a: AllReduce, r: ReduceScatter, g: AllGather
  int c;
  while ((c = getopt(argc, argv, "d:r:b:e:f:i:w:o:t:g:c:H:G:")) != -1) {
    switch (c) {
      case 'd': ndevArg = atoi(optarg); break;
      case 'r': perDev = atoi(optarg); break;
      case 'b': minB = strtoull(optarg, nullptr, 0); break;
      case 'e': maxB = strtoull(optarg, nullptr, 0); break;
      case 'f': factor = atof(optarg); break;
      case 'i': iters = atoi(optarg); break;
      case 'w': warmup = atoi(optarg); break;
      case 'g': graph = atoi(optarg); break;
      case 'H': hold = atoi(optarg); break;
      case 'G': perGroup = std::max(1, atoi(optarg)); break;
      case 'c': coll = !strcmp(optarg, "rs") ? 'r' : !strcmp(optarg, "ag") ? 'g' : !strcmp(optarg, "reduce") ? 'd' : 'a'; break;
      case 'o': op = !strcmp(optarg, "max") ? ncclMax : ncclSum; break;
      case 't':
        type = !strcmp(optarg, "half") ? ncclFloat16 : !strcmp(optarg, "bf16") ? ncclBfloat16
             : !strcmp(optarg, "int") ? ncclInt32 : ncclFloat32;
        break;
      default: fprintf(stderr, "bad option\n"); return 1;
    }
  }
  int ndevAll = 0;
  HIPCK(hipGetDeviceCount(&ndevAll));
  int ndev = ndevArg > 0 ? std::min(ndevArg, ndevAll) : ndevAll;
  const int n = ndev * perDev;
  std::vector<int> devs(n);
  for (int r = 0; r < n; r++) devs[r] = r / perDev;
  std::vector<ncclComm_t> comms(n);
  NCK(ncclCommInitAll(comms.data(), n, devs.data()));
  int version = 0;
  NCK(ncclGetVersion(&version));
  const size_t es = type == ncclFloat16 || type == ncclBfloat16 ? 2 : 4;
  std::vector<void*> send(n), recv(n);
  std::vector<hipStream_t> streams(n);
  std::vector<hipEvent_t> ev0(n), ev1(n);
  unsigned long long* bad = nullptr;
  for (int r = 0; r < n; r++) {
    HIPCK(hipSetDevice(devs[r]));
    HIPCK(hipMalloc(&send[r], maxB * perGroup));  // -G: K slices of the largest size
    HIPCK(hipMalloc(&recv[r], maxB * perGroup));
    // own hardware queue per rank (ranks sharing a device must run concurrently)
    int ncu = 0;
    HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, devs[r]));
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int cu = 0; cu < ncu; cu++) mask[cu / 32] |= 1u << (cu % 32);
    HIPCK(hipExtStreamCreateWithCUMask(&streams[r], (uint32_t)mask.size(), mask.data()));
    HIPCK(hipEventCreate(&ev0[r]));
    HIPCK(hipEventCreate(&ev1[r]));
    hipLaunchKernelGGL(fillKernel, dim3(1024), dim3(256), 0, streams[r], send[r], maxB * perGroup / es, (int)type,
                       (float)(r + 1));
  }
  HIPCK(hipSetDevice(devs[0]));
  HIPCK(hipMallocManaged(&bad, sizeof(*bad)));
  for (int r = 0; r < n; r++) HIPCK(hipStreamSynchronize(streams[r]));
  const float want = op == ncclSum ? n * (n + 1) / 2.0f : (float)n;
  printf("# nccl_perf: libnccl %d, %s, %d ranks (%d devices x %d), type %d, op %s, %s\n", version,
         coll == 'r' ? "ReduceScatter" : coll == 'g' ? "AllGather" : coll == 'd' ? "Reduce (root 0)" : "AllReduce", n, ndev,
         perDev, (int)type,
         op == ncclSum ? "sum" : "max", graph ? "hipGraph replay" : "eager launches");
  auto issue = [&](int r, size_t count, size_t slice = 0) {
    const size_t off = slice * count * es;  // -G: op k of a group works on bytes [k * bytes, (k + 1) * bytes)
    const char* sb = (const char*)send[r] + off;
    char* rb = (char*)recv[r] + off;
    if (coll == 'r') return ncclReduceScatter(sb, rb, count / n, type, op, comms[r], streams[r]);
    if (coll == 'g') return ncclAllGather(sb, rb, count / n, type, comms[r], streams[r]);
    if (coll == 'd') return ncclReduce(sb, rb, count, type, op, 0, comms[r], streams[r]);
    return ncclAllReduce(sb, rb, count, type, op, comms[r], streams[r]);
  };
  printf("# %12s %12s %10s %10s %10s %8s %9s\n", "bytes", "count", "time(us)", "algbw", "busbw", "#wrong", "host(us)");
  const size_t step = coll == 'a' || coll == 'd' ? es : es * n;
  for (size_t bytes = minB; bytes <= maxB; bytes = std::max(bytes + step, (size_t)(bytes * factor))) {
    if (bytes % step) continue;
    const size_t count = bytes / es;  // elements of the AllReduce buffer / RS input / AG output
    auto enqueue = [&](int iters_) {
      for (int k = 0; k < iters_; k++) {
        NCK(ncclGroupStart());
        for (int r = 0; r < n; r++)
          for (int j = 0; j < perGroup; j++) NCK(issue(r, count, j));
        NCK(ncclGroupEnd());
      }
    };
    enqueue(warmup);
    for (int r = 0; r < n; r++) HIPCK(hipStreamSynchronize(streams[r]));
    std::vector<hipGraphExec_t> execs;
    if (graph) {
      // capture each rank's loop on its own stream (collective launches never block the host)
      for (int r = 0; r < n; r++) {
        HIPCK(hipSetDevice(devs[r]));
        hipGraph_t g;
        HIPCK(hipStreamBeginCapture(streams[r], hipStreamCaptureModeRelaxed));
        for (int k = 0; k < iters; k++) NCK(issue(r, count));
        HIPCK(hipStreamEndCapture(streams[r], &g));
        hipGraphExec_t ex;
        HIPCK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
        HIPCK(hipGraphDestroy(g));
        execs.push_back(ex);
      }
    }
    if (hold)  // ~20 ms on the 100 MHz wall clock: longer than issuing the timed loop
      for (int r = 0; r < n; r++) hipLaunchKernelGGL(spinKernel, dim3(1), dim3(64), 0, streams[r], 2000000LL);
    for (int r = 0; r < n; r++) HIPCK(hipEventRecord(ev0[r], streams[r]));
    double hostUs = 0;  // host time to issue one group of n collectives (eager only)
    if (graph) {
      for (int r = 0; r < n; r++) HIPCK(hipGraphLaunch(execs[r], streams[r]));
    } else {
      auto h0 = std::chrono::steady_clock::now();
      enqueue(iters);
      hostUs = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count() / iters;
    }
    for (int r = 0; r < n; r++) HIPCK(hipEventRecord(ev1[r], streams[r]));
    float ms = 0;
    for (int r = 0; r < n; r++) {
      HIPCK(hipEventSynchronize(ev1[r]));
      float t;
      HIPCK(hipEventElapsedTime(&t, ev0[r], ev1[r]));
      ms = std::max(ms, t);
    }
    for (hipGraphExec_t ex : execs) HIPCK(hipGraphExecDestroy(ex));
    *bad = 0;
    for (int r = 0; r < (coll == 'd' ? 1 : n); r++) {  // Reduce: only the root's output is defined
      HIPCK(hipSetDevice(devs[r]));
      const size_t outCount = (coll == 'r' ? count / n : count) * (perGroup > 1 && coll != 'g' && coll != 'r' ? perGroup : 1);
      hipLaunchKernelGGL(checkKernel, dim3(256), dim3(256), 0, streams[r], recv[r], outCount, (int)type, want,
                         coll == 'g' ? count / n : (size_t)0, bad);
      HIPCK(hipStreamSynchronize(streams[r]));
    }
    for (int r = 0; r < n; r++) {
      ncclResult_t ae;
      NCK(ncclCommGetAsyncError(comms[r], &ae));
      if (ae != ncclSuccess) {
        fprintf(stderr, "rank %d async error %s\n", r, ncclGetErrorString(ae));
        return 4;
      }
    }
    const double us = ms * 1e3 / iters;
    const double algbw = bytes / (us * 1e-6) / 1e9;
    printf("  %12zu %12zu %10.2f %10.2f %10.2f %8llu %9.2f\n", bytes, count, us, algbw,
           coll == 'd' ? algbw : algbw * (coll == 'a' ? 2.0 : 1.0) * (n - 1) / n, (unsigned long long)*bad, hostUs);
    if (*bad) return 5;
  }
  for (int r = 0; r < n; r++) NCK(ncclCommDestroy(comms[r]));
  return 0;
}

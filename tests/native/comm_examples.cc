// comm_examples.cc — the reference's communicator-creation examples, restated against include/nccl.h and
// extended with one AllReduce whose every element has a known answer:
//
//   comm_examples pthread N   one thread per rank, each ncclCommInitRank on a shared ncclUniqueId
//                             (reference docs/examples/01_communicators/02_one_device_per_pthread/c/main.cc:
//                             per-thread init, ncclCommUserRank / ncclCommCount, Finalize then Destroy)
//   comm_examples initall N   ncclCommInitAll over N ranks from one thread (reference
//                             docs/examples/01_communicators/01_multiple_devices_single_process/c/main.cc:
//                             rank i on devices[i], ncclCommUserRank / ncclCommCuDevice / ncclCommCount)
//
// Rank r fills 1M floats with r; the AllReduce sum must be n(n-1)/2 in every element (the value the
// reference's 03_collectives/01_allreduce example checks). Rank i runs on device i % ndev, so N > ndev puts
// several ranks on one GPU (set NCCL_MULTI_RANK_GPU_ENABLE=1). The caller's current device must be the same
// after every call as before it (reference enqueue.cc:3137-3162). Exit 0 and "OK" on success.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <vector>

#include "nccl.h"

static std::atomic<int> gFailures{0};

static void fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
static void fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
  gFailures++;
}
static bool hipOk(hipError_t e, const char* what, int line) {
  if (e != hipSuccess) fail("line %d: %s: %s", line, what, hipGetErrorString(e));
  return e == hipSuccess;
}
static bool ncclOk(ncclResult_t r, const char* what, int line) {
  if (r != ncclSuccess) fail("line %d: %s: %s", line, what, ncclGetErrorString(r));
  return r == ncclSuccess;
}
#define HIPOK(x) hipOk((x), #x, __LINE__)
#define NCCLOK(x) ncclOk((x), #x, __LINE__)
#define FAIL(...) fail(__VA_ARGS__)

static const size_t kCount = 1 << 20;

__global__ void fillRank(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void countWrong(const float* p, size_t n, float want, unsigned long long* bad) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    local += p[i] != want;
  if (local) atomicAdd(bad, local);
}

struct RankBufs {
  float* send = nullptr;
  float* recv = nullptr;
  unsigned long long* bad = nullptr;
  hipStream_t stream = nullptr;
};

static bool setup(RankBufs& b, int dev, int rank) {
  bool ok = HIPOK(hipSetDevice(dev)) && HIPOK(hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking)) &&
            HIPOK(hipMalloc(&b.send, kCount * sizeof(float))) && HIPOK(hipMalloc(&b.recv, kCount * sizeof(float))) &&
            HIPOK(hipMalloc(&b.bad, sizeof(unsigned long long)));
  if (!ok) return false;
  hipLaunchKernelGGL(fillRank, dim3(256), dim3(256), 0, b.stream, b.send, kCount, (float)rank);
  return HIPOK(hipMemsetAsync(b.bad, 0, sizeof(unsigned long long), b.stream)) && HIPOK(hipStreamSynchronize(b.stream));
}

static void verify(RankBufs& b, int dev, int rank, int n) {
  if (!HIPOK(hipSetDevice(dev))) return;
  const float want = (float)(n * (n - 1) / 2);
  hipLaunchKernelGGL(countWrong, dim3(256), dim3(256), 0, b.stream, b.recv, kCount, want, b.bad);
  unsigned long long bad = 0;
  if (HIPOK(hipMemcpyAsync(&bad, b.bad, sizeof(bad), hipMemcpyDeviceToHost, b.stream)) &&
      HIPOK(hipStreamSynchronize(b.stream)) && bad)
    FAIL("rank %d: %llu of %zu elements differ from %g", rank, bad, kCount, want);
}

static void release(RankBufs& b) {
  (void)hipFree(b.send);
  (void)hipFree(b.recv);
  (void)hipFree(b.bad);
  if (b.stream) (void)hipStreamDestroy(b.stream);
}

static void checkQueries(ncclComm_t comm, int rank, int n, int dev) {
  int r = -1, cnt = -1, d = -1;
  if (NCCLOK(ncclCommUserRank(comm, &r)) && r != rank) FAIL("ncclCommUserRank %d, expected %d", r, rank);
  if (NCCLOK(ncclCommCount(comm, &cnt)) && cnt != n) FAIL("ncclCommCount %d, expected %d", cnt, n);
  if (NCCLOK(ncclCommCuDevice(comm, &d)) && d != dev) FAIL("ncclCommCuDevice %d, expected %d", d, dev);
}

// ---- one device per pthread ----
struct ThreadArg {
  int rank, n, ndev;
  ncclUniqueId id;
};

static void* worker(void* p) {
  ThreadArg* a = (ThreadArg*)p;
  const int dev = a->rank % a->ndev;
  RankBufs b;
  if (!setup(b, dev, a->rank)) return nullptr;
  ncclComm_t comm = nullptr;
  if (NCCLOK(ncclCommInitRank(&comm, a->n, a->id, a->rank))) {
    checkQueries(comm, a->rank, a->n, dev);
    if (NCCLOK(ncclAllReduce(b.send, b.recv, kCount, ncclFloat32, ncclSum, comm, b.stream))) {
      int cur = -1;
      if (HIPOK(hipGetDevice(&cur)) && cur != dev) FAIL("rank %d: current device %d after ncclAllReduce", a->rank, cur);
      verify(b, dev, a->rank, a->n);
    }
    NCCLOK(ncclCommFinalize(comm));
    NCCLOK(ncclCommDestroy(comm));
  }
  release(b);
  return nullptr;
}

static void runPthread(int n, int ndev) {
  ncclUniqueId id;
  if (!NCCLOK(ncclGetUniqueId(&id))) return;
  std::vector<pthread_t> th(n);
  std::vector<ThreadArg> args(n);
  for (int i = 0; i < n; i++) {
    args[i] = {i, n, ndev, id};
    pthread_create(&th[i], nullptr, worker, &args[i]);
  }
  for (int i = 0; i < n; i++) pthread_join(th[i], nullptr);
}

// ---- several devices from one thread ----
static void runInitAll(int n, int ndev) {
  std::vector<int> devs(n);
  for (int i = 0; i < n; i++) devs[i] = i % ndev;
  std::vector<RankBufs> b(n);
  for (int i = 0; i < n; i++)
    if (!setup(b[i], devs[i], i)) return;
  // the caller's device before the collectives: the last rank's, set by setup(); every call must leave it
  int before = -1;
  HIPOK(hipGetDevice(&before));
  std::vector<ncclComm_t> comms(n, nullptr);
  if (NCCLOK(ncclCommInitAll(comms.data(), n, devs.data()))) {
    for (int i = 0; i < n; i++) checkQueries(comms[i], i, n, devs[i]);
    NCCLOK(ncclGroupStart());
    for (int i = 0; i < n; i++)
      NCCLOK(ncclAllReduce(b[i].send, b[i].recv, kCount, ncclFloat32, ncclSum, comms[i], b[i].stream));
    NCCLOK(ncclGroupEnd());
    int cur = -1;
    if (HIPOK(hipGetDevice(&cur)) && cur != before) FAIL("current device %d after the group, was %d", cur, before);
    for (int i = 0; i < n; i++) verify(b[i], devs[i], i, n);
    for (int i = 0; i < n; i++) NCCLOK(ncclCommDestroy(comms[i]));
  }
  for (int i = 0; i < n; i++) release(b[i]);
}

int main(int argc, char** argv) {
  if (argc < 3 || (strcmp(argv[1], "pthread") && strcmp(argv[1], "initall"))) {
    fprintf(stderr, "usage: %s pthread|initall NRANKS\n", argv[0]);
    return 2;
  }
  const int n = atoi(argv[2]);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1 || n < 1) {
    fprintf(stderr, "no device (or NRANKS < 1)\n");
    return 2;
  }
  if (!strcmp(argv[1], "pthread")) runPthread(n, ndev);
  else runInitAll(n, ndev);
  if (gFailures.load()) {
    fprintf(stderr, "FAILED: %d check(s)\n", gFailures.load());
    return 1;
  }
  printf("OK %s n=%d on %d device(s): every element %d\n", argv[1], n, ndev, n * (n - 1) / 2);
  return 0;
}

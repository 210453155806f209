// reuse_probe.hip — the importer-side pattern of eager registration churn, without the library:
// process A allocates a buffer, exports it as a dma-buf and hands the fd to process B (SCM_RIGHTS); B imports it
// (hipImportExternalMemory + hipExternalMemoryGetMappedBuffer, as ipc.cc importFd), reads it with a kernel; A frees
// its allocation; B unmaps (hipFree of the mapped buffer + hipDestroyExternalMemory, as ipc.cc releaseLocked), then
// allocates a buffer of its own (hipMalloc: may land on the unmapped range) and writes / reads it with a kernel.
// Repeated ITERS times. Prints one JSON line per process: whether B's new allocation reused the unmapped range, and
// whether every value read back matched. Both processes share GPU 0.
//
//   reuse_probe [ITERS=6] [MiB=256] [OWN=1] [FIXED=0]
//   reuse_probe ... PAIR=1: A also allocates a second, never-written buffer of the same size each iteration and exports
//   it after the first (an AllReduce's recvbuff beside its sendbuff); B maps and unmaps both.
//   OWN=0: B allocates nothing, so its next import follows its unmap directly. FIXED=1: A allocates the same size every
//   iteration (as PyTorch's caching allocator does: the runtime then hands back the same range) and an export that
//   fails is retried (1 ms apart, up to 20 times) and counted instead of ending the run.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "[%s] %s:%d %s: %s\n", who, __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                                    \
    }                                                                                             \
  } while (0)

static const char* who = "?";

__global__ void fill(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v ^ (uint32_t)i;
}
__global__ void check(const uint32_t* p, size_t n, uint32_t v, unsigned long long* bad) {
  unsigned long long b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b += p[i] != (v ^ (uint32_t)i);
  if (b) atomicAdd(bad, b);
}

static int sendFd(int s, int fd, uint64_t v) {
  struct msghdr m = {};
  struct iovec io = {&v, sizeof(v)};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  if (fd >= 0) {
    m.msg_control = ctl;
    m.msg_controllen = sizeof(ctl);
    struct cmsghdr* h = CMSG_FIRSTHDR(&m);
    h->cmsg_level = SOL_SOCKET;
    h->cmsg_type = SCM_RIGHTS;
    h->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(h), &fd, sizeof(int));
  }
  return sendmsg(s, &m, 0) == (ssize_t)sizeof(v) ? 0 : -1;
}
static int recvFd(int s, int* fd, uint64_t* v) {
  struct msghdr m = {};
  struct iovec io = {v, sizeof(*v)};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  m.msg_control = ctl;
  m.msg_controllen = sizeof(ctl);
  *fd = -1;
  if (recvmsg(s, &m, MSG_WAITALL) != (ssize_t)sizeof(*v)) return -1;
  for (struct cmsghdr* h = CMSG_FIRSTHDR(&m); h; h = CMSG_NXTHDR(&m, h))
    if (h->cmsg_level == SOL_SOCKET && h->cmsg_type == SCM_RIGHTS) memcpy(fd, CMSG_DATA(h), sizeof(int));
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 6;
  const size_t bytes = (size_t)(argc > 2 ? atol(argv[2]) : 256) << 20;
  const size_t n = bytes / 4;
  const bool own = argc > 3 ? atoi(argv[3]) != 0 : true;
  const bool fixed = argc > 4 ? atoi(argv[4]) != 0 : false;
  const bool pair = argc > 5 ? atoi(argv[5]) != 0 : false;
  int pairFails = 0, pairRetried = 0;
  int exportFails = 0, exportRetried = 0, exportGaveUp = 0, sameRange = 0;
  uintptr_t lastBuf = 0;
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 1;
  const pid_t pid = fork();  // before any HIP call: each process initialises its own runtime
  if (pid < 0) return 1;
  const bool isA = pid != 0;
  who = isA ? "A" : "B";
  const int s = isA ? sv[0] : sv[1];
  CHECK(hipSetDevice(0));
  unsigned long long* bad = nullptr;
  CHECK(hipMalloc(&bad, sizeof(*bad)));
  int reused = 0, badIters = 0, reusedImport = 0;
  uintptr_t lastMapped = 0;
  void* mine = nullptr;  // B: its own allocation of the previous iteration
  for (int it = 0; it < iters; it++) {
    uint64_t tok = 0;
    if (isA) {
      void* buf = nullptr;
      CHECK(hipMalloc(&buf, bytes + (fixed ? 0 : (size_t)it * 4096)));
      sameRange += (uintptr_t)buf == lastBuf;
      lastBuf = (uintptr_t)buf;
      hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (uint32_t*)buf, n, 0xA0000000u + it);
      CHECK(hipDeviceSynchronize());
      int fd = -1;
      hipError_t e = hipErrorInvalidValue;
      for (int attempt = 0; attempt < (fixed ? 21 : 1); attempt++) {
        e = hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)buf, bytes, hipMemRangeHandleTypeDmaBufFd, 0);
        if (e == hipSuccess) {
          exportRetried += attempt > 0;
          break;
        }
        (void)hipGetLastError();
        exportFails += attempt == 0;
        usleep(1000);
      }
      if (e != hipSuccess && !fixed) CHECK(e);
      if (e != hipSuccess) {  // tell B to skip this iteration
        exportGaveUp++;
        if (sendFd(s, -1, (uint64_t)~0ull) != 0) return 1;
        CHECK(hipFree(buf));
        continue;
      }
      void* buf2 = nullptr;
      int fd2 = -1;
      if (pair) {
        CHECK(hipMalloc(&buf2, bytes));
        hipError_t e2 = hipErrorInvalidValue;
        for (int attempt = 0; attempt < 21; attempt++) {
          e2 = hipMemGetHandleForAddressRange(&fd2, (hipDeviceptr_t)buf2, bytes, hipMemRangeHandleTypeDmaBufFd, 0);
          if (e2 == hipSuccess) {
            pairRetried += attempt > 0;
            break;
          }
          (void)hipGetLastError();
          pairFails += attempt == 0;
          usleep(1000);
        }
        if (e2 != hipSuccess) fd2 = -1;
      }
      if (sendFd(s, fd, (uint64_t)it) != 0) return 1;
      close(fd);
      if (pair && sendFd(s, fd2, fd2 >= 0 ? 1 : 0) != 0) return 1;
      if (fd2 >= 0) close(fd2);
      if (recvFd(s, &fd, &tok) != 0) return 1;  // B has read it through its mapping
      CHECK(hipFree(buf));                       // the owner frees first (B still maps it)
      if (buf2) CHECK(hipFree(buf2));
      if (sendFd(s, -1, 0) != 0) return 1;
    } else {
      int fd = -1;
      if (recvFd(s, &fd, &tok) != 0) return 1;
      if (tok == ~0ull) continue;  // A's export failed this iteration
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
      hipExternalMemory_t em2 = nullptr;
      void* mapped2 = nullptr;
      int fd2 = -1;
      if (pair) {
        uint64_t has = 0;
        if (recvFd(s, &fd2, &has) != 0) return 1;
        if (has) {
          hipExternalMemoryHandleDesc hd2 = {};
          hd2.type = hipExternalMemoryHandleTypeOpaqueFd;
          hd2.handle.fd = fd2;
          hd2.size = bytes;
          CHECK(hipImportExternalMemory(&em2, &hd2));
          CHECK(hipExternalMemoryGetMappedBuffer(&mapped2, em2, &bd));
        }
      }
      CHECK(hipMemset(bad, 0, sizeof(*bad)));
      hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, (const uint32_t*)mapped, n, 0xA0000000u + it, bad);
      CHECK(hipDeviceSynchronize());
      unsigned long long hb = 0;
      CHECK(hipMemcpy(&hb, bad, sizeof(hb), hipMemcpyDeviceToHost));
      badIters += hb != 0;
      if (sendFd(s, -1, 0) != 0) return 1;
      if (recvFd(s, &fd, &tok) != 0) return 1;  // A freed its allocation
      CHECK(hipFree(mapped));                    // unmap, as ipc.cc releaseLocked
      CHECK(hipDestroyExternalMemory(em));
      close(hd.handle.fd);
      if (mapped2) {
        CHECK(hipFree(mapped2));
        CHECK(hipDestroyExternalMemory(em2));
      }
      if (fd2 >= 0) close(fd2);
      reusedImport += (uintptr_t)mapped == lastMapped;
      lastMapped = (uintptr_t)mapped;
      if (!own) continue;
      if (mine) CHECK(hipFree(mine));
      CHECK(hipMalloc(&mine, bytes + (size_t)it * 4096));  // B's own next buffer: may take the unmapped range
      const uintptr_t a = (uintptr_t)mine, m = (uintptr_t)mapped;
      reused += a < m + bytes && m < a + bytes + (size_t)it * 4096;
      hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (uint32_t*)mine, n, 0xB0000000u + it);
      CHECK(hipMemset(bad, 0, sizeof(*bad)));
      hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, (const uint32_t*)mine, n, 0xB0000000u + it, bad);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(&hb, bad, sizeof(hb), hipMemcpyDeviceToHost));
      badIters += hb != 0;
    }
  }
  if (isA) {
    int st = 0;
    waitpid(pid, &st, 0);
    printf("{\"process\": \"A\", \"iters\": %d, \"allocations_at_the_previous_range\": %d, \"exports_failed_first\": %d, "
           "\"exports_ok_after_retry\": %d, \"exports_given_up\": %d, \"second_exports_failed_first\": %d, \"second_exports_ok_after_retry\": %d, "
           "\"child_exit\": %d}\n", iters, sameRange, exportFails, exportRetried, exportGaveUp, pairFails, pairRetried,
           WIFEXITED(st) ? WEXITSTATUS(st) : -1);
  } else {
    printf("{\"process\": \"B\", \"iters\": %d, \"MiB\": %zu, \"new_allocation_on_unmapped_range\": %d, "
           "\"imports_at_the_previous_mapping\": %d, \"iterations_with_wrong_values\": %d}\n", iters, bytes >> 20,
           reused, reusedImport, badIters);
  }
  fflush(stdout);
  return 0;
}

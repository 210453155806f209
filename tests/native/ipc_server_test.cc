// Host-only test of the IPC fd server (nccl_amd/csrc/ipc.cc) that hands dma-buf descriptors to importing
// peers. No GPU: memfds stand in for dma-bufs (the server passes any descriptor). Built plain and under
// ASan/UBSan and TSan (Makefile target `sanitize`, tests/test_sanitizers.py):
//   1. many threads fetch published descriptors concurrently while the main thread publishes and retires
//      other keys; every fetched descriptor reads back its memfd's pattern;
//   2. a forked child fetches across processes (skipped under TSan: fork of a threaded process);
//   3. an unknown key and a server that does not exist fail with ncclRemoteError within the bounded wait;
//   4. stopping the server while clients are fetching ends every fetch (success or error, never a hang).
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../nccl_amd/csrc/core.h"
using namespace ncclamd;

static int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      fprintf(stderr, "ipc_server_test:%d: %s\n", __LINE__, #c);    \
      fails++;                                                      \
    }                                                               \
  } while (0)

static int makeMemfd(char pattern, size_t size) {
  int fd = memfd_create("ncclamd-test", MFD_CLOEXEC);
  if (fd < 0) return -1;
  std::vector<char> buf(size, pattern);
  if (write(fd, buf.data(), size) != (ssize_t)size) return -1;
  return fd;
}

static bool readsBack(int fd, char pattern, size_t size) {
  std::vector<char> buf(size, 0);
  if (pread(fd, buf.data(), size, 0) != (ssize_t)size) return false;
  for (char c : buf)
    if (c != pattern) return false;
  return true;
}

int main(int argc, char** argv) {
  const bool allowFork = !(argc > 1 && !strcmp(argv[1], "nofork"));
  setenv("NCCL_AMD_IPC_TIMEOUT_MS", "400", 1);  // before any thread starts (getenv vs setenv)
  const size_t kSize = 8192;
  ncclComm* comm = new ncclComm();
  CHECK(ipcServerStart(comm) == ncclSuccess);
  CHECK(comm->fdServer != nullptr);

  IpcDesc da, db;
  CHECK(ipcPublish(comm, makeMemfd('a', kSize), kSize, &da) == ncclSuccess);
  CHECK(ipcPublish(comm, makeMemfd('b', kSize), kSize, &db) == ncclSuccess);
  CHECK(da.key != db.key && !strcmp(da.server, db.server));

  // 1. concurrent fetches vs publish / retire churn
  std::atomic<int> bad{0}, done{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; t++)
    ts.emplace_back([&, t]() {
      for (int i = 0; i < 40; i++) {
        const IpcDesc& d = (i + t) % 2 ? da : db;
        int fd = -1;
        if (ipcFetchFd(d, &fd) != ncclSuccess || !readsBack(fd, (i + t) % 2 ? 'a' : 'b', kSize)) bad++;
        if (fd >= 0) close(fd);
      }
      done++;
    });
  for (int i = 0; i < 200; i++) {
    IpcDesc dc;
    CHECK(ipcPublish(comm, makeMemfd('c', 64), 64, &dc) == ncclSuccess);
    ipcUnexport(comm, dc);
  }
  for (auto& t : ts) t.join();
  CHECK(bad.load() == 0);
  CHECK(done.load() == 8);

  // 2. another process
  if (allowFork) {
    pid_t p = fork();
    if (p == 0) {
      int fd = -1;
      bool ok = ipcFetchFd(da, &fd) == ncclSuccess && readsBack(fd, 'a', kSize);
      _exit(ok ? 0 : 1);
    }
    int st = 0;
    waitpid(p, &st, 0);
    CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }

  // 3. bounded failures
  IpcDesc unknown = da;
  unknown.key = 0xdeadbeefull;
  int fd = -1;
  auto t0 = std::chrono::steady_clock::now();
  CHECK(ipcFetchFd(unknown, &fd) == ncclRemoteError && fd == -1);
  IpcDesc nowhere = da;
  snprintf(nowhere.server, sizeof(nowhere.server), "ncclamd.nobody.%d", (int)getpid());
  CHECK(ipcFetchFd(nowhere, &fd) == ncclRemoteError && fd == -1);
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  CHECK(secs < 5.0);
  ipcUnexport(comm, db);
  CHECK(ipcFetchFd(db, &fd) == ncclRemoteError);  // retired: refused, not served stale

  // 3b. the registration requests (register.cc): a RELEASE of a mapping the server does not hold is a no-op
  // success, an IMPORT without a descriptor attached is refused (status != 0 -> ncclRemoteError), neither
  // touches the GPU; fetches keep working around them
  ipcRemoteRelease(da.server, 3, 0x1234);
  uint64_t addr = 0;
  CHECK(ipcRemoteImport(da.server, 3, 0x1234, -1, 4096, &addr) == ncclRemoteError && addr == 0);
  CHECK(ipcRemoteImport(nowhere.server, 3, 0x1234, -1, 4096, &addr) == ncclRemoteError);
  fd = -1;
  CHECK(ipcFetchFd(da, &fd) == ncclSuccess && readsBack(fd, 'a', kSize));
  if (fd >= 0) close(fd);
  // server names carry a random nonce besides pid and serial (pid reuse across PID namespaces)
  CHECK(strlen(da.server) > strlen("ncclamd.") + 8);

  // 3c. legacy hipIpc handles (NCCL_AMD_IPC=legacy) are refused on runtimes older than 7.2 at any size; a
  // fallback handle rides along a dma-buf export below 2 GiB there, at any size on 7.2+
  CHECK(!ipcLegacyAllowed(70051831, 4096, true));
  CHECK(!ipcLegacyAllowed(70051831, (size_t)3 << 30, true));
  CHECK(ipcLegacyAllowed(70200000, (size_t)3 << 30, true));
  CHECK(ipcLegacyAllowed(70051831, 4096, false));
  CHECK(!ipcLegacyAllowed(70051831, (size_t)2 << 30, false));
  CHECK(ipcLegacyAllowed(70253211, (size_t)2 << 30, false));

  // 4. stop while clients fetch
  std::atomic<int> finished{0};
  std::vector<std::thread> late;
  for (int t = 0; t < 4; t++)
    late.emplace_back([&]() {
      for (int i = 0; i < 5; i++) {
        int f = -1;
        if (ipcFetchFd(da, &f) == ncclSuccess) close(f);
      }
      finished++;
    });
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  ipcServerStop(comm);
  CHECK(comm->fdServer == nullptr);
  for (auto& t : late) t.join();
  CHECK(finished.load() == 4);
  delete comm;
  printf("ipc_server_test fork=%d failures=%d\n", allowFork ? 1 : 0, fails);
  return fails ? 1 : 0;
}

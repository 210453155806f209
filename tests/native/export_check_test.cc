// CPU test of the stale-export checks (ipc.cc ipcAdmitExport) with memfd files standing in for the
// dma-bufs an export hands back: the allocation's own file is admitted (again too), a file of another size or one
// exported before for another allocation — by this process or by another — is refused. The registry lives in
// $NCCL_AMD_DMABUF_NODE_DIR (the caller's fresh directory). Prints one line per case; exit status = failures.
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include "../../nccl_amd/csrc/core.h"

using namespace ncclamd;

static int file(size_t size) {
  const int fd = memfd_create("dmabuf", 0);
  if (fd < 0 || ftruncate(fd, (off_t)size) != 0) return -1;
  return fd;
}

int main() {
  if (!getenv("NCCL_AMD_DMABUF_NODE_DIR")) {
    fprintf(stderr, "set NCCL_AMD_DMABUF_NODE_DIR to a fresh directory\n");
    return 100;
  }
  int fails = 0;
  auto expect = [&](bool got, bool want, const char* what) {
    printf("%s %s\n", got == want ? "ok" : "FAIL", what);
    if (got != want) fails++;
  };
  const size_t MiB = (size_t)1 << 20;
  void* const A = (void*)0x100000000ull;
  void* const B = (void*)0x200000000ull;
  const int a = file(4 * MiB), big = file(8 * MiB), rounded = file(4 * MiB + 4096), shared = file(2 * MiB);
  if (a < 0 || big < 0 || rounded < 0 || shared < 0) return 101;
  expect(ipcAdmitExport(dup(a), A, 4 * MiB), true, "a fresh dma-buf of the allocation's size is admitted");
  expect(ipcAdmitExport(dup(a), A, 4 * MiB), true, "the same allocation's dma-buf handed back again is admitted");
  expect(ipcAdmitExport(dup(a), B, 4 * MiB), false, "a dma-buf exported before for another allocation is refused");
  expect(ipcAdmitExport(dup(big), B, 4 * MiB), false, "a dma-buf larger than the allocation is refused");
  expect(ipcAdmitExport(dup(big), B, 16 * MiB), false, "a dma-buf smaller than the allocation is refused");
  expect(ipcAdmitExport(dup(rounded), B, 4 * MiB), true, "a dma-buf rounded up by less than 2 MiB is admitted");
  const pid_t child = fork();
  if (child == 0) {  // another process of the node exports `shared` for its allocation at A
    _exit(ipcAdmitExport(dup(shared), A, 2 * MiB) ? 0 : 1);
  }
  int st = 0;
  waitpid(child, &st, 0);
  expect(WIFEXITED(st) && WEXITSTATUS(st) == 0, true, "another process's fresh export is admitted there");
  expect(ipcAdmitExport(dup(shared), A, 2 * MiB), false,
         "its dma-buf handed back here, even for the same address, is refused (the node registry)");
  return fails;
}

// Host-only test of the TCP bootstrap (nccl_amd/csrc/bootstrap.cc): the parent creates a unique id,
// forks nranks children that rendezvous, all-gather a payload, barrier, and verify. No GPU needed.
#include <sys/wait.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../nccl_amd/csrc/core.h"
using namespace ncclamd;

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 4;
  int rounds = argc > 2 ? atoi(argv[2]) : 3;
  ncclUniqueId id;
  if (bootstrapGetUniqueId(&id) != ncclSuccess) return 2;
  std::vector<pid_t> kids;
  for (int r = 0; r < n; r++) {
    pid_t p = fork();
    if (p == 0) {
      Bootstrap* b = nullptr;
      if (bootstrapInit(&id, r, n, &b) != ncclSuccess) _exit(3);
      for (int k = 0; k < rounds; k++) {
        std::vector<uint64_t> v(n * 4, 0);
        for (int j = 0; j < 4; j++) v[r * 4 + j] = 1000ull * r + k * 10 + j;
        if (bootstrapAllGather(b, v.data(), 4 * sizeof(uint64_t)) != ncclSuccess) _exit(4);
        for (int q = 0; q < n; q++)
          for (int j = 0; j < 4; j++)
            if (v[q * 4 + j] != 1000ull * q + k * 10 + j) _exit(5);
        if (bootstrapBarrier(b) != ncclSuccess) _exit(6);
      }
      bootstrapClose(b);
      _exit(0);
    }
    kids.push_back(p);
  }
  int bad = 0;
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad++;
  }
  printf("bootstrap_test n=%d rounds=%d failures=%d\n", n, rounds, bad);
  return bad ? 1 : 0;
}

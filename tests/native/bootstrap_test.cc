// Host-only test of the TCP bootstrap (nccl_amd/csrc/bootstrap.cc): the parent creates a unique id,
// forks nranks children that rendezvous, all-gather a payload, barrier, and verify. No GPU needed.
// Mode "threads" runs the ranks as threads of one process instead (as ncclCommInitAll and a group of inits
// do): the form the TSan build checks (tests/test_sanitizers.py). Mode "scalable <nId>" gives the ranks nId
// ids as ncclCommInitRankScalable does: they rendezvous at id 0 and release the others' roots, which must
// then refuse connections.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>
#include "../../nccl_amd/csrc/core.h"
using namespace ncclamd;

static int runRank(ncclUniqueId* id, int r, int n, int rounds) {
  Bootstrap* b = nullptr;
  if (bootstrapInit(id, r, n, &b) != ncclSuccess) return 3;
  for (int k = 0; k < rounds; k++) {
    std::vector<uint64_t> v(n * 4, 0);
    for (int j = 0; j < 4; j++) v[r * 4 + j] = 1000ull * r + k * 10 + j;
    if (bootstrapAllGather(b, v.data(), 4 * sizeof(uint64_t)) != ncclSuccess) return 4;
    for (int q = 0; q < n; q++)
      for (int j = 0; j < 4; j++)
        if (v[q * 4 + j] != 1000ull * q + k * 10 + j) return 5;
    if (bootstrapBarrier(b) != ncclSuccess) return 6;
  }
  bootstrapClose(b);
  return 0;
}

// true once the root behind `id` no longer accepts connections (the id's payload holds its sockaddr_in at
// byte 16, bootstrap.cc IdPayload); gives up after 5 s.
static bool rootGone(const ncclUniqueId& id) {
  struct sockaddr_in a;
  memcpy(&a, id.internal + 16, sizeof(a));
  auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5)) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    int rc = connect(fd, (struct sockaddr*)&a, sizeof(a));
    close(fd);
    if (rc != 0) return true;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  return false;
}

static int scalable(int n, int rounds, int nId) {
  std::vector<ncclUniqueId> ids(nId);
  for (auto& id : ids)
    if (bootstrapGetUniqueId(&id) != ncclSuccess) return 2;
  std::vector<pid_t> kids;
  for (int r = 0; r < n; r++) {
    pid_t p = fork();
    if (p == 0) {
      if (bootstrapReleaseUnused(ids.data(), nId, r, n) != ncclSuccess) _exit(7);
      _exit(runRank(&ids[0], r, n, rounds));
    }
    kids.push_back(p);
  }
  int bad = 0;
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad++;
  }
  int alive = 0;
  for (int k = 1; k < nId; k++) alive += !rootGone(ids[k]);
  printf("bootstrap_test scalable n=%d nId=%d rounds=%d failures=%d roots_left=%d\n", n, nId, rounds, bad, alive);
  return bad || alive ? 1 : 0;
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 4;
  int rounds = argc > 2 ? atoi(argv[2]) : 3;
  const bool threads = argc > 3 && !strcmp(argv[3], "threads");
  if (argc > 4 && !strcmp(argv[3], "scalable")) return scalable(n, rounds, atoi(argv[4]));
  ncclUniqueId id;
  if (bootstrapGetUniqueId(&id) != ncclSuccess) return 2;
  int bad = 0;
  if (threads) {
    std::vector<int> rc(n, -1);
    std::vector<std::thread> ts;
    for (int r = 0; r < n; r++) ts.emplace_back([&, r]() { rc[r] = runRank(&id, r, n, rounds); });
    for (auto& t : ts) t.join();
    for (int x : rc) bad += x != 0;
    printf("bootstrap_test threads n=%d rounds=%d failures=%d\n", n, rounds, bad);
    return bad ? 1 : 0;
  }
  std::vector<pid_t> kids;
  for (int r = 0; r < n; r++) {
    pid_t p = fork();
    if (p == 0) _exit(runRank(&id, r, n, rounds));
    kids.push_back(p);
  }
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad++;
  }
  printf("bootstrap_test n=%d rounds=%d failures=%d\n", n, rounds, bad);
  return bad ? 1 : 0;
}

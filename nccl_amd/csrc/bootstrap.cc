// bootstrap.cc — out-of-band rendezvous for ncclCommInitRank (one node).
//
// Reference: src/bootstrap.cc:405-462 (root listener created by ncclGetUniqueId, address carried in
// the 128-byte ncclUniqueId), :674-884 (bootstrapInit), :1194 (bootstrapAllGather), bootstrapBarrier.
// The reference builds a socket ring between ranks so it scales to thousands of nodes. This engine
// is intra-node only (≤ 8 GPUs of one MI355X node), so the root thread stays alive as a
// star: every rank keeps one TCP connection to it and each collective round is "all ranks send
// their block, the root returns the concatenation". Only init-time metadata travels here (peer
// info + HIP IPC handles) and the destroy barrier; nothing on the data path.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <random>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "core.h"

namespace ncclamd {

static constexpr uint64_t kIdMagic = 0x424f4f5453545250ull;  // "BOOTSTRP"

struct IdPayload {  // lives inside ncclUniqueId::internal (128 bytes)
  uint64_t magic;
  uint64_t commId;
  struct sockaddr_in addr;
};
static_assert(sizeof(IdPayload) <= NCCL_UNIQUE_ID_BYTES, "unique id payload too large");

struct Hello {
  uint64_t magic;
  uint64_t commId;
  int32_t rank;
  int32_t nranks;
};

struct Bootstrap {
  int fd = -1;
  int rank = 0;
  int nranks = 0;
};

static bool sendAll(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
// returns 1 ok, 0 clean EOF before any byte, -1 error
static int recvAll(int fd, void* p, size_t n) {
  char* c = (char*)p;
  size_t got = 0;
  while (got < n) {
    ssize_t k = ::recv(fd, c + got, n - got, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k == 0) return got == 0 ? 0 : -1;
    if (k < 0) return -1;
    got += (size_t)k;
  }
  return 1;
}

static int64_t bootstrapTimeoutMs() { return paramInt("NCCL_AMD_BOOTSTRAP_TIMEOUT_MS", 600000); }

// Hello.rank of a release message (ncclCommInitRankScalable): the root is not needed, exit.
static constexpr int32_t kReleaseRank = -1;

// Root service: accept nranks connections, then serve all-gather rounds until every rank hangs up.
static void rootThread(int listenFd, uint64_t commId) {
  std::vector<int> fds;
  int nranks = -1;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(bootstrapTimeoutMs());
  while (true) {  // until every rank has said hello
    struct pollfd pfd = {listenFd, POLLIN, 0};
    int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
    if (left <= 0) { WARN("bootstrap root: timed out waiting for ranks"); goto done; }
    int pr = poll(&pfd, 1, left);
    if (pr <= 0) continue;
    int fd = accept(listenFd, nullptr, nullptr);
    if (fd < 0) continue;
    Hello h;
    const bool got = recvAll(fd, &h, sizeof(h)) == 1;
    if (got && h.magic == kIdMagic && h.commId == commId && h.rank == kReleaseRank && nranks < 0) {
      close(fd);  // an unused id of ncclCommInitRankScalable: no rank will connect here
      goto done;
    }
    if (!got || h.magic != kIdMagic || h.commId != commId || h.nranks <= 0 ||
        h.rank < 0 || h.rank >= h.nranks || (nranks >= 0 && h.nranks != nranks)) {
      WARN("bootstrap root: rejected connection (bad hello)");
      close(fd);
      continue;
    }
    if (nranks < 0) { nranks = h.nranks; fds.assign(nranks, -1); }
    if (fds[h.rank] != -1) { WARN("bootstrap root: duplicate rank %d", h.rank); close(fd); continue; }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    fds[h.rank] = fd;
    int connected = 0;
    for (int f : fds) connected += (f != -1);
    if (connected == nranks) break;
  }
  // serve rounds
  while (true) {
    std::vector<std::vector<char>> blocks(nranks);
    int closed = 0;
    for (int r = 0; r < nranks; r++) {
      uint64_t sz;
      int rc = recvAll(fds[r], &sz, sizeof(sz));
      if (rc == 0) { closed++; continue; }
      if (rc < 0) goto done;
      blocks[r].resize(sz);
      if (sz && recvAll(fds[r], blocks[r].data(), sz) != 1) goto done;
    }
    if (closed == nranks) break;
    if (closed) { WARN("bootstrap root: %d rank(s) left mid-round", closed); break; }
    std::vector<char> all;
    for (int r = 0; r < nranks; r++) {
      if (blocks[r].size() != blocks[0].size()) { WARN("bootstrap root: block size mismatch"); goto done; }
      all.insert(all.end(), blocks[r].begin(), blocks[r].end());
    }
    for (int r = 0; r < nranks; r++)
      if (!sendAll(fds[r], all.data(), all.size())) goto done;
  }
done:
  for (int f : fds)
    if (f >= 0) close(f);
  close(listenFd);
}

ncclResult_t bootstrapGetUniqueId(ncclUniqueId* id) {
  memset(id, 0, sizeof(*id));
  IdPayload p;
  memset(&p, 0, sizeof(p));
  p.magic = kIdMagic;
  std::random_device rd;
  p.commId = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)getpid();
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  SYSCHECK(fd >= 0, "socket");
  struct sockaddr_in a;
  memset(&a, 0, sizeof(a));
  a.sin_family = AF_INET;
  const char* ip = paramStr("NCCL_AMD_BOOTSTRAP_ADDR");  // intra-node: loopback by default
  if (inet_pton(AF_INET, ip ? ip : "127.0.0.1", &a.sin_addr) != 1) {
    close(fd);
    WARN("bad NCCL_AMD_BOOTSTRAP_ADDR %s", ip);
    return ncclInvalidArgument;
  }
  a.sin_port = 0;
  if (bind(fd, (struct sockaddr*)&a, sizeof(a)) != 0 || listen(fd, 128) != 0) {
    close(fd);
    WARN("bootstrap: bind/listen failed: %s", strerror(errno));
    return ncclSystemError;
  }
  socklen_t len = sizeof(a);
  getsockname(fd, (struct sockaddr*)&a, &len);
  p.addr = a;
  memcpy(id->internal, &p, sizeof(p));
  std::thread(rootThread, fd, p.commId).detach();
  INFO("bootstrap root listening on %s:%d", inet_ntoa(a.sin_addr), ntohs(a.sin_port));
  return ncclSuccess;
}

ncclResult_t bootstrapInit(const ncclUniqueId* id, int rank, int nranks, Bootstrap** out) {
  IdPayload p;
  memcpy(&p, id->internal, sizeof(p));
  if (p.magic != kIdMagic) {
    WARN("ncclCommInitRank: invalid ncclUniqueId (was it produced by ncclGetUniqueId?)");
    return ncclInvalidArgument;
  }
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(bootstrapTimeoutMs());
  int fd = -1;
  while (true) {
    fd = socket(AF_INET, SOCK_STREAM, 0);
    SYSCHECK(fd >= 0, "socket");
    if (connect(fd, (struct sockaddr*)&p.addr, sizeof(p.addr)) == 0) break;
    int err = errno;
    close(fd);
    fd = -1;
    if (std::chrono::steady_clock::now() > deadline) {
      WARN("bootstrap: connect to root failed: %s", strerror(err));
      return ncclRemoteError;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  Hello h = {kIdMagic, p.commId, rank, nranks};
  if (!sendAll(fd, &h, sizeof(h))) {
    close(fd);
    WARN("bootstrap: hello failed");
    return ncclRemoteError;
  }
  Bootstrap* b = new Bootstrap;
  b->fd = fd;
  b->rank = rank;
  b->nranks = nranks;
  *out = b;
  return ncclSuccess;
}

// ncclCommInitRankScalable hands every rank nId ids (reference bootstrap.cc:59-89 spreads the ranks over
// nId roots). This engine's star needs one root, so every rank rendezvouses at id 0 and the first rank of
// each other id's rank group (the reference's block partition, rootIdFromRank) tells that id's root to
// exit instead of waiting for ranks that never come. Bounded like every bootstrap connect.
ncclResult_t bootstrapRelease(const ncclUniqueId* id) {
  IdPayload p;
  memcpy(&p, id->internal, sizeof(p));
  if (p.magic != kIdMagic) {
    WARN("ncclCommInitRankScalable: invalid ncclUniqueId (was it produced by ncclGetUniqueId?)");
    return ncclInvalidArgument;
  }
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(bootstrapTimeoutMs());
  while (true) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    SYSCHECK(fd >= 0, "socket");
    if (connect(fd, (struct sockaddr*)&p.addr, sizeof(p.addr)) == 0) {
      Hello h = {kIdMagic, p.commId, kReleaseRank, 0};
      bool ok = sendAll(fd, &h, sizeof(h));
      close(fd);
      if (ok) return ncclSuccess;
    } else {
      close(fd);
    }
    if (std::chrono::steady_clock::now() > deadline) {
      WARN("bootstrap: could not release an unused root");
      return ncclRemoteError;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

// Root of rank r when nranks ranks are spread over nRoots ids (reference bootstrap.cc:59-69, offset 0).
static int rootIdFromRank(int r, int nranks, int nRoots) {
  const int rmr = nranks % nRoots, rpr = nranks / nRoots, D = rmr * (rpr + 1);
  return r < D ? r / (rpr + 1) : (r - D) / rpr + rmr;
}

// Each id k >= 1 is released by exactly one rank: the first rank of root k's group, or rank k % nranks
// for an id no rank maps to (nId > nranks). An id listed twice is one root (still in use if it equals id 0).
ncclResult_t bootstrapReleaseUnused(const ncclUniqueId* ids, int nId, int rank, int nranks) {
  for (int k = 1; k < nId; k++) {
    bool dup = false;
    for (int j = 0; j < k && !dup; j++) dup = memcmp(&ids[j], &ids[k], sizeof(ncclUniqueId)) == 0;
    if (dup) continue;
    int releaser = k % nranks;
    for (int r = 0; r < nranks; r++)
      if (rootIdFromRank(r, nranks, nId) == k) {
        releaser = r;
        break;
      }
    if (releaser == rank) NCCLCHECK(bootstrapRelease(&ids[k]));
  }
  return ncclSuccess;
}

// data holds nranks blocks of bytesPerRank; this rank's block (index rank) is sent, all are received.
ncclResult_t bootstrapAllGather(Bootstrap* b, void* data, size_t bytesPerRank) {
  uint64_t sz = bytesPerRank;
  char* d = (char*)data;
  if (!sendAll(b->fd, &sz, sizeof(sz)) || !sendAll(b->fd, d + (size_t)b->rank * bytesPerRank, bytesPerRank)) {
    WARN("bootstrap allgather: send failed");
    return ncclRemoteError;
  }
  if (recvAll(b->fd, d, bytesPerRank * (size_t)b->nranks) != 1) {
    WARN("bootstrap allgather: recv failed (a peer exited?)");
    return ncclRemoteError;
  }
  return ncclSuccess;
}

ncclResult_t bootstrapBarrier(Bootstrap* b) {
  std::vector<char> tmp(b->nranks);
  return bootstrapAllGather(b, tmp.data(), 1);
}

// In-process all-gather for the comms of one ncclCommInitAll (no sockets: they share this object).
// Two generation-counted barriers per round: all blocks are in, then all copies are out, so a fast rank
// cannot start the next round while a slow one still reads this one.
struct LocalClique {
  std::mutex m;
  std::condition_variable cv;
  int n = 0;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<char> buf;
};

std::shared_ptr<LocalClique> cliqueCreate(int nranks) {
  auto c = std::make_shared<LocalClique>();
  c->n = nranks;
  return c;
}

static void cliqueBarrier(LocalClique* c, std::unique_lock<std::mutex>& lk) {
  uint64_t g = c->gen;
  if (++c->arrived == c->n) {
    c->arrived = 0;
    c->gen++;
    c->cv.notify_all();
  } else {
    c->cv.wait(lk, [&] { return c->gen != g; });
  }
}

ncclResult_t cliqueAllGather(LocalClique* c, int rank, void* data, size_t bytesPerRank) {
  std::unique_lock<std::mutex> lk(c->m);
  if (c->buf.size() < bytesPerRank * c->n) c->buf.resize(bytesPerRank * c->n);
  memcpy(c->buf.data() + (size_t)rank * bytesPerRank, (char*)data + (size_t)rank * bytesPerRank, bytesPerRank);
  cliqueBarrier(c, lk);
  memcpy(data, c->buf.data(), bytesPerRank * c->n);
  cliqueBarrier(c, lk);
  return ncclSuccess;
}

void bootstrapClose(Bootstrap* b) {
  if (!b) return;
  if (b->fd >= 0) close(b->fd);
  delete b;
}

}  // namespace ncclamd

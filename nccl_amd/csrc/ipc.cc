// ipc.cc — sharing device memory with the other processes of a communicator (staging slabs, flag blocks,
// registered windows).
//
// Reference: src/transport/p2p.cc:220-325 exports each buffer as a cuMem POSIX file descriptor and hands the
// fd to the peer over a UNIX socket (its proxy thread), instead of legacy cudaIpc handles. This is the same
// design on HIP: the exporter turns the allocation into a dma-buf fd (hipMemGetHandleForAddressRange), a
// per-communicator fd server passes it to each importing peer over an abstract UNIX socket (SCM_RIGHTS),
// and the importer maps it with hipImportExternalMemory + hipExternalMemoryGetMappedBuffer.
//
// Why not hipIpcGetMemHandle / hipIpcOpenMemHandle: inside any process that imports torch, this library
// binds to torch's bundled HIP runtime (torch/lib/libamdhip64.so, ROCm 7.0 in this image; same soname,
// loaded first), and there hipIpcOpenMemHandle of an allocation of 2 GiB or more never returns (the
// importing thread spins in user space), for hipMalloc and uncached memory alike. The dma-buf path maps
// 1-3 GiB allocations on both that runtime and /opt/rocm 7.2 (scripts/ipc_paths_torchrt.py,
// tests/native/ipc_paths_probe.hip). NCCL_AMD_IPC=legacy keeps the hipIpc path for
// comparison and refuses allocations of 2 GiB or more on runtimes older than 7.2 instead of hanging.
//
// Every socket operation is bounded (NCCL_AMD_IPC_TIMEOUT_MS): an import whose exporter died or never
// published returns ncclSystemError / ncclRemoteError rather than blocking the caller.
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <string.h>
#include <sys/file.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <thread>

#include "core.h"

namespace ncclamd {

struct FdServer {
  int listenFd = -1;
  int wakePipe[2] = {-1, -1};
  std::thread thread;
  std::mutex mu;
  std::map<uint64_t, int> table;  // key -> exported dma-buf fd
  char name[40] = {};  // fits IpcDesc::server
  int device = 0;      // the communicator's GPU: peers' registered buffers are mapped onto it
  // Peers' registered buffers mapped in this process on their behalf (IMPORT requests; reference: the peer's
  // proxy thread maps a registered buffer for ncclIpcLocalRegisterBuffer, src/transport/p2p.cc ipcRegister):
  // (registering rank, its registration tag) -> mapping. Touched only by the server thread.
  std::map<std::pair<int, uint64_t>, IpcImport> imports;
};

// Releasing a mapping frees its address range and tears the interop mapping down in two runtime calls (hipFree,
// hipDestroyExternalMemory); hipFree also waits for the whole device.
//
// Round 3's fault (gpurun_out/rehearsal_n4_diag/bench_n4.log, bench.py --gpus 4 on one GPU): a helper ("reaper")
// thread of each fd server released peers' deregistered buffers as soon as their RELEASE requests arrived,
// concurrently with whatever the caller's thread did next. In the bench suite the "registered" part deregistered
// its buffers and the next part ("staged_tuning default") created a new communicator at once: its slab was
// allocated, exported and imported by the peers while the reapers were still in hipFree / hipDestroyExternalMemory
// of the old mappings. All four ranks then reported an illegal memory access at the first synchronize after that
// communicator's first collective (no record names the faulting kernel or address; the other two runs of the same
// order failed with a refused dma-buf export and a spin timeout). What the three failures share is a runtime
// allocation / import / export racing a teardown on another thread, which the fix (dea9ffb) removed: no helper
// thread, every import and release of this library under gMapMu.
//
// What the mechanism guarantees since round 4:
//  * the fd server never touches the device for a RELEASE: it moves the mapping to gPending and answers;
//  * gPending is drained on the caller's thread only: at entry points that may block by contract — CommInitRank /
//    InitAll, Finalize, Destroy, (Window)Register and (Window)Deregister — and, since round 6, at a collective's
//    enqueue once none of this library's kernels is in flight in this process (ipcProgressReleases: the unmap then
//    waits for nothing of ours; a collective returns once its work is enqueued, reference nccl.h.in:431-442; the
//    reference unmaps on its proxy thread, src/transport/p2p.cc:762-780), never concurrently with this library's
//    allocations or imports (gMapMu);
//  * a mapping stays valid until drained, so a kernel of this rank still reading the peer's buffer never faults:
//    the dma-buf import keeps the peer's memory referenced even after the peer freed it.
// The cost is memory: a peer's deregistered buffer stays mapped here until this rank's next such point.
static std::mutex gMapMu;
std::mutex& ipcMapMutex() { return gMapMu; }
static void releaseLocked(IpcImport* m);
struct PendingRelease {
  IpcImport map;
  int device;
};
static std::mutex gPendMu;
static std::vector<PendingRelease> gPending;
static std::atomic<bool> gHavePending{false};

// Bytes of released peer mappings waiting to be unmapped (ipcProgressReleases, ipcDrainReleases); past
// NCCL_AMD_PENDING_RELEASE_WARN_BYTES (4 GiB) that is said once per crossing, with the calls that return the memory
// (ADVICE r4).
static uint64_t gPendingBytes = 0;
static bool gPendingWarned = false;

static void releaseLater(int device, const IpcImport& m) {
  std::lock_guard<std::mutex> g(gPendMu);
  gPending.push_back({m, device});
  gPendingBytes += m.size;
  gHavePending.store(true, std::memory_order_release);
  static const uint64_t warnAt = (uint64_t)paramInt("NCCL_AMD_PENDING_RELEASE_WARN_BYTES", (int64_t)4 << 30);
  if (gPendingBytes >= warnAt && !gPendingWarned) {
    gPendingWarned = true;
    WARN("%.2f GiB of peers' deregistered buffers are still mapped in this process (device %d): they are unmapped at "
         "this rank's next collective issued while none of the library's kernels runs here, or its next blocking call "
         "(ncclCommRegister / Deregister / Finalize / Destroy / Init); until then the peers' freed HBM stays allocated",
         gPendingBytes / (double)(1ull << 30), device);
  }
}

void ipcDrainReleases() {
  if (!gHavePending.load(std::memory_order_acquire)) return;
  std::vector<PendingRelease> batch;
  {
    std::lock_guard<std::mutex> g(gPendMu);
    batch.swap(gPending);
    gPendingBytes = 0;
    gPendingWarned = false;
    gHavePending.store(false, std::memory_order_release);
  }
  if (batch.empty()) return;
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;  // another thread may be capturing in global mode
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  for (PendingRelease& r : batch) {
    (void)hipSetDevice(r.device);
    ipcRelease(&r.map);
  }
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  (void)hipSetDevice(dev);
  TRACE("ipc: released %zu peer mapping(s) of deregistered buffers", batch.size());
}

// Every stream this library launched a kernel on in this process, with an event recorded after its latest launch
// (multi-process communicators, outside captures: ipcNoteLaunch). "Every one complete" means no kernel of this library
// is in flight here — the condition for unmapping on the collective path below.
struct StreamTail {
  hipStream_t stream;
  int device;
  hipEvent_t ev;
};
static std::mutex gTailMu;
static std::vector<StreamTail> gTails;
static bool gTailsOverflow = false;  // more streams than tracked: the collective path never unmaps
constexpr size_t kMaxTails = 64;

void ipcNoteLaunch(hipStream_t stream, int device) {
  std::lock_guard<std::mutex> g(gTailMu);
  if (gTailsOverflow) return;
  for (StreamTail& t : gTails)
    if (t.stream == stream && t.device == device) {
      if (hipEventRecord(t.ev, stream) != hipSuccess) (void)hipGetLastError(), gTailsOverflow = true;
      return;
    }
  StreamTail t = {stream, device, nullptr};
  if (gTails.size() >= kMaxTails || hipEventCreateWithFlags(&t.ev, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(t.ev, stream) != hipSuccess) {
    (void)hipGetLastError();
    gTailsOverflow = true;  // (an event created before a failed record stays unused)
    return;
  }
  gTails.push_back(t);
}

static bool libraryIdle() {
  std::lock_guard<std::mutex> g(gTailMu);
  if (gTailsOverflow) return false;
  for (const StreamTail& t : gTails)
    if (hipEventQuery(t.ev) == hipErrorNotReady) return false;
  (void)hipGetLastError();
  return true;
}

// The collective path's share of the drain. A mapping whose owner sent RELEASE is read by no
// kernel any more: the owner sends it only once its own last kernel on the buffer has completed (register.cc
// regProgress, an event query), and every peer kernel reads the buffer before the DONE signal that kernel waits for.
// What keeps it off the collective path is the unmap itself: hipFree of an imported mapping waits for every kernel
// of this process on the device (tests/native/release_probe: 300.0 ms behind a 300 ms kernel; hipDestroyExternalMemory
// 2 us; profiles/r06_release_probe.json). Waiting for one of this library's kernels there could deadlock: it may wait
// on a peer that waits for this rank's next launch (a peer importing a registration from this process's fd server,
// which needs gMapMu; ranks issuing collectives of two communicators in different orders). So the collective path
// unmaps only once every kernel this library launched here has completed (libraryIdle: event queries, never a wait);
// the hipFree then waits at most for the application's own kernels, as any hipFree of the application does. Bounded
// work — two mappings per call — and never contending with this library's allocations and imports: when another thread
// holds gMapMu (a non-blocking init, the fd server importing a peer's registration) they wait for a later call.
// NCCL_AMD_RELEASE_ON_COLL=0 leaves them to the blocking entry points.
bool ipcLibraryIdle() { return libraryIdle(); }

void ipcProgressReleases() {
  if (!gHavePending.load(std::memory_order_acquire)) return;
  static const bool on = paramInt("NCCL_AMD_RELEASE_ON_COLL", 1) != 0;
  static std::atomic<int> said{0};  // why a pending release waits (INFO, the first 16 times in the process)
  if (!on) return;
  if (!libraryIdle()) {
    if (said.fetch_add(1) < 16) INFO("ipc: peers' released mappings wait: a kernel of this library is in flight");
    return;
  }
  std::unique_lock<std::mutex> lk(gMapMu, std::try_to_lock);
  if (!lk.owns_lock()) {
    if (said.fetch_add(1) < 16) INFO("ipc: peers' released mappings wait: the mapping lock is busy");
    return;
  }
  std::vector<PendingRelease> batch;
  {
    std::lock_guard<std::mutex> g(gPendMu);
    while (!gPending.empty() && batch.size() < 2) {
      batch.push_back(gPending.back());
      gPending.pop_back();
      gPendingBytes -= std::min(gPendingBytes, batch.back().map.size);
    }
    if (gPending.empty()) {
      gPendingWarned = false;
      gHavePending.store(false, std::memory_order_release);
    }
  }
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;  // the caller's stream may be capturing
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  for (PendingRelease& r : batch) {
    (void)hipSetDevice(r.device);
    releaseLocked(&r.map);
  }
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  (void)hipSetDevice(dev);
  (void)hipGetLastError();
  INFO("ipc: released %zu peer mapping(s) on the collective path (%zu MiB still pending)", batch.size(),
       (size_t)(gPendingBytes >> 20));
}

// Requests on the fd server's socket (one per connection). FETCH: hand over the fd published under `key`.
// IMPORT: map the dma-buf fd attached to the request (SCM_RIGHTS) on this comm's device on behalf of rank
// `from`, remember it under (from, key) and answer the address it got here. RELEASE: drop that mapping.
enum IpcOp : uint32_t { IPC_FETCH = 1, IPC_IMPORT = 2, IPC_RELEASE = 3 };
struct IpcRequest {
  uint32_t op;
  int32_t from;
  uint64_t key;
  uint64_t size;
  uint32_t legacy;            // IMPORT: map `handle` (a hipIpc handle) instead of an attached dma-buf fd
  uint32_t pad;
  hipIpcMemHandle_t handle;
};
struct IpcReply {
  int32_t status;  // 0 = ok
  int32_t pad;
  uint64_t value;  // IMPORT: the mapped address in the server's process
};

static std::atomic<uint64_t> gServerSerial{0};
static std::atomic<uint64_t> gKeySerial{1};

static int64_t ipcTimeoutMs() { return paramInt("NCCL_AMD_IPC_TIMEOUT_MS", 60000); }

static uint32_t randomNonce() {
  uint32_t v = 0;
  int fd = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
  if (fd >= 0) {
    if (read(fd, &v, sizeof(v)) != (ssize_t)sizeof(v)) v = 0;
    close(fd);
  }
  if (v == 0) v = (uint32_t)std::chrono::steady_clock::now().time_since_epoch().count() ^ (uint32_t)getpid() * 2654435761u;
  return v;
}

bool ipcLegacy() {
  const char* m = paramStr("NCCL_AMD_IPC");
  return m && !strcasecmp(m, "legacy");
}

static socklen_t abstractAddr(const char* name, struct sockaddr_un* a) {
  memset(a, 0, sizeof(*a));
  a->sun_family = AF_UNIX;
  size_t n = strlen(name);
  memcpy(a->sun_path + 1, name, n);  // abstract namespace: leading NUL, nothing on the filesystem
  return (socklen_t)(offsetof(struct sockaddr_un, sun_path) + 1 + n);
}

static void setTimeouts(int fd) {
  int64_t ms = ipcTimeoutMs();
  struct timeval tv = {(time_t)(ms / 1000), (suseconds_t)((ms % 1000) * 1000)};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

static ncclResult_t importFd(int fd, uint64_t size, IpcImport* out);
static ncclResult_t importLegacy(const IpcDesc& d, IpcImport* out);

static int recvWithFd(int c, void* buf, size_t len, int* fd) {
  struct msghdr m = {};
  struct iovec io = {buf, len};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  m.msg_control = ctl;
  m.msg_controllen = sizeof(ctl);
  *fd = -1;
  ssize_t got = recvmsg(c, &m, MSG_WAITALL | MSG_CMSG_CLOEXEC);
  for (struct cmsghdr* h = CMSG_FIRSTHDR(&m); h; h = CMSG_NXTHDR(&m, h))
    if (h->cmsg_level == SOL_SOCKET && h->cmsg_type == SCM_RIGHTS) memcpy(fd, CMSG_DATA(h), sizeof(int));
  return got == (ssize_t)len ? 0 : -1;
}

static int sendWithFd(int c, const void* buf, size_t len, int fd) {
  struct msghdr m = {};
  struct iovec io = {const_cast<void*>(buf), len};
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
  return sendmsg(c, &m, MSG_NOSIGNAL) == (ssize_t)len ? 0 : -1;
}

// One request per connection, from a process of our uid only (SO_PEERCRED).
static void serveOne(FdServer* s, int c) {
  setTimeouts(c);
  struct ucred cred;
  socklen_t cl = sizeof(cred);
  IpcRequest q = {};
  IpcReply reply = {-1, 0, 0};
  int inFd = -1, outFd = -1;
  if (getsockopt(c, SOL_SOCKET, SO_PEERCRED, &cred, &cl) != 0 || cred.uid != getuid() ||
      recvWithFd(c, &q, sizeof(q), &inFd) != 0) {
    if (inFd >= 0) close(inFd);
    close(c);
    return;
  }
  if (q.op == IPC_FETCH) {
    std::lock_guard<std::mutex> g(s->mu);
    auto it = s->table.find(q.key);
    if (it != s->table.end()) {
      outFd = it->second;
      reply.status = 0;
    }
  } else if (q.op == IPC_IMPORT && (inFd >= 0 || q.legacy)) {
    IpcImport m;
    bool mapped = false;
    if (hipSetDevice(s->device) == hipSuccess) {
      if (q.legacy) {  // a registration whose dma-buf export the owner's runtime refused (ipcRemoteImportHandle)
        IpcDesc d;
        memset(&d, 0, sizeof(d));
        d.legacy = 1;
        d.size = q.size;
        d.handle = q.handle;
        memset(&m, 0, sizeof(m));
        m.fd = -1;
        mapped = importLegacy(d, &m) == ncclSuccess;
        m.size = q.size;
      } else {
        mapped = importFd(inFd, q.size, &m) == ncclSuccess;
        if (mapped) inFd = -1;  // owned by the mapping now
      }
    }
    if (mapped) {
      auto key = std::make_pair((int)q.from, q.key);
      // diagnostics: a mapping the runtime placed where an earlier one of ours still lives (live or pending release)
      const uint64_t lo = (uint64_t)m.ptr, hi = lo + m.size;
      auto overlaps = [&](const IpcImport& x) { return lo < (uint64_t)x.ptr + x.size && (uint64_t)x.ptr < hi; };
      for (const auto& kv : s->imports)
        if (overlaps(kv.second))
          WARN("ipc: rank %d tag %lu mapped at %p over the live mapping of rank %d tag %lu (%p, ino %lu / %lu)", q.from,
               (unsigned long)q.key, m.ptr, kv.first.first, (unsigned long)kv.first.second, kv.second.ptr,
               (unsigned long)m.fdIno, (unsigned long)kv.second.fdIno);
      {
        std::lock_guard<std::mutex> g(gPendMu);
        for (const PendingRelease& r : gPending)
          if (overlaps(r.map))
            WARN("ipc: rank %d tag %lu mapped at %p over a mapping pending release (%p, ino %lu / %lu)", q.from,
                 (unsigned long)q.key, m.ptr, r.map.ptr, (unsigned long)m.fdIno, (unsigned long)r.map.fdIno);
      }
      TRACE("ipc: IMPORT rank %d tag %lu: %lu MiB at %p (%s %lu)", q.from, (unsigned long)q.key,
            (unsigned long)(m.size >> 20), m.ptr, q.legacy ? "hipIpc handle" : "dma-buf ino", (unsigned long)m.fdIno);
      auto old = s->imports.find(key);
      if (old != s->imports.end()) releaseLater(s->device, old->second);  // a re-registration replaces its mapping
      s->imports[key] = m;
      reply.status = 0;
      reply.value = (uint64_t)m.ptr;
    } else {
      (void)hipGetLastError();
    }
  } else if (q.op == IPC_RELEASE) {
    auto it = s->imports.find(std::make_pair((int)q.from, q.key));
    if (it != s->imports.end()) {
      TRACE("ipc: RELEASE rank %d tag %lu: %p (ino %lu) pending", q.from, (unsigned long)q.key, it->second.ptr,
            (unsigned long)it->second.fdIno);
      releaseLater(s->device, it->second);  // never block the server on the device (gPending above)
      s->imports.erase(it);
    }
    reply.status = 0;
  }
  if (inFd >= 0) close(inFd);
  (void)sendWithFd(c, &reply, sizeof(reply), outFd);
  close(c);
}

static void serverLoop(FdServer* s) {
  // The server maps peers' registered buffers while this process may be capturing a graph on another thread
  // (NCCL_GRAPH_REGISTER: every rank registers inside its capture): relaxed capture mode keeps this thread's
  // runtime calls out of such a global-mode capture (the reference's proxy thread does the same)
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  while (true) {
    struct pollfd p[2] = {{s->listenFd, POLLIN, 0}, {s->wakePipe[0], POLLIN, 0}};
    int r = poll(p, 2, -1);
    if (r < 0 && errno == EINTR) continue;
    if (r < 0 || (p[1].revents & (POLLIN | POLLHUP))) break;
    if (p[0].revents & POLLIN) {
      int c = accept(s->listenFd, nullptr, nullptr);
      if (c >= 0) serveOne(s, c);
    }
  }
}

ncclResult_t ipcServerStart(ncclComm* comm) {
  if (comm->fdServer || ipcLegacy()) return ncclSuccess;
  FdServer* s = new FdServer();
  s->device = comm->device;
  // pid + a per-process serial + a random nonce: processes of other PID namespaces sharing this network
  // namespace (containers with host networking) may reuse our pid, and the abstract namespace is per netns
  snprintf(s->name, sizeof(s->name), "ncclamd.%d.%llu.%08x", (int)getpid(), (unsigned long long)gServerSerial++,
           (unsigned)randomNonce());
  s->listenFd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  struct sockaddr_un a;
  socklen_t al = abstractAddr(s->name, &a);
  if (s->listenFd < 0 || bind(s->listenFd, (struct sockaddr*)&a, al) != 0 || listen(s->listenFd, 64) != 0 ||
      pipe2(s->wakePipe, O_CLOEXEC) != 0) {
    WARN("ipc: fd server %s: %s", s->name, strerror(errno));
    if (s->listenFd >= 0) close(s->listenFd);
    delete s;
    return ncclSystemError;
  }
  // the server thread's first runtime call must not be the one that initialises the HIP runtime: that init
  // may set environment variables while other threads read theirs (getenv vs setenv), so it happens here first
  int dev = 0;
  (void)hipGetDevice(&dev);
  (void)hipGetLastError();
  s->thread = std::thread(serverLoop, s);
  comm->fdServer = s;
  TRACE("rank %d: fd server %s", comm->rank, s->name);
  return ncclSuccess;
}

const char* ipcServerName(const ncclComm* comm) { return comm->fdServer ? comm->fdServer->name : ""; }

void ipcServerStop(ncclComm* comm) {
  FdServer* s = comm->fdServer;
  if (!s) return;
  if (s->wakePipe[1] >= 0) (void)!write(s->wakePipe[1], "x", 1);
  if (s->thread.joinable()) s->thread.join();
  ipcDrainReleases();  // what RELEASE requests queued (for any communicator of this process)
  for (auto& kv : s->table) close(kv.second);
  if (!s->imports.empty()) (void)hipSetDevice(comm->device);
  for (auto& kv : s->imports) ipcRelease(&kv.second);  // peers' registrations still mapped here
  close(s->listenFd);
  close(s->wakePipe[0]);
  close(s->wakePipe[1]);
  delete s;
  comm->fdServer = nullptr;
}

// The HIP runtime this library is actually bound to. Inside any process that imports torch that is torch's
// bundled libamdhip64 (ROCm 7.0 in this image, same soname, loaded first), not the /opt/rocm 7.2 runtime the
// library was built against: found with dladdr on a runtime entry point, logged once at
// the first communicator init (NCCL_DEBUG=INFO) so a runtime-specific defect is attributable.
const HipRuntimeInfo& hipRuntimeInfo() {
  static HipRuntimeInfo info = [] {
    HipRuntimeInfo r = {};
    (void)hipRuntimeGetVersion(&r.version);  // major * 10000000 + minor * 100000 + patch
    (void)hipDriverGetVersion(&r.driver);
    Dl_info dl;
    if (dladdr((void*)&hipRuntimeGetVersion, &dl) && dl.dli_fname) snprintf(r.path, sizeof(r.path), "%s", dl.dli_fname);
    else snprintf(r.path, sizeof(r.path), "?");
    return r;
  }();
  return info;
}

// NCCL_AMD_IPC=legacy (hipIpc handles): torch's bundled ROCm 7.0 runtime never returns from
// hipIpcOpenMemHandle for allocations of 2 GiB or more, and this engine's slabs, windows and
// registered buffers can reach that size at any time, so legacy handles are refused on runtimes older than
// 7.2 whatever the size. Without NCCL_AMD_IPC=legacy a hipIpc handle only rides along a dma-buf export as the
// importer's fallback, and only where it is known to open: below 2 GiB, or on a 7.2+ runtime.
bool ipcLegacyAllowed(int runtimeVersion, size_t size, bool requested) {
  if (runtimeVersion >= 70200000) return true;
  return !requested && size < ((size_t)2 << 30);
}

// The dma-buf export of [base, +size) (hipMemGetHandleForAddressRange), under gMapMu like every import and release of
// this library. Round 6's eager churn (tests/test_gpu_eager.py, gpurun_out TRACE logs): 2-5 of 16
// exports per rank were refused with "invalid argument", each a re-allocation at the address of a just-freed
// registered allocation whose peers were unmapping the old one; a plain export / import / unmap cycle of the same
// buffers without the library's kernels never failed (scripts/eager_churn_probe.py, tests/native/reuse_probe.hip: 0 of
// 80). `attempts` > 1 retries a refusal 1, 2, 4, 8 ms apart (the lock released meanwhile): kept for the init-time
// exports, whose only alternative is failing the communicator; no retry was ever seen to succeed in the churn, where
// the eager path has the bounce allocation instead and asks for one attempt.
//
// An export can hand back a dma-buf that already exists — another allocation's, exported earlier by this process
// or by another process on the same device — instead of a new one for this allocation. Measured in round 6 (TRACE
// logs): (1) the eager churn inside the full GPU suite, a rank exported its send and then its receive allocation and
// the peer received ONE dma-buf (one inode) for both: the peer's zero-copy kernel read the send buffer as the
// receive one; (2) the n = 8 one-GPU rehearsal, rank 3's export of its 256 MiB output handed back the 512 MiB bounce
// dma-buf rank 2 had created 66 us earlier: the peers mapped it as rank 3's output and pulled rank 2's input from it —
// a silently wrong block on every rank but rank 3, in 1 of 4 runs. Serializing every export and import of the node
// (below) did not remove it (2 such exports in 5 runs, both caught), so it is not a race between concurrent calls
// but stale state in the export path. Two checks, both under the node lock:
//  * the dma-buf's size (its llseek end) must be the allocation's (catches (2));
//  * a node-wide registry of every dma-buf the library's processes exported (/tmp/.ncclamd_dmabuf.<uid>.reg: inode,
//    the exporting process's random id, base, buffer id): a dma-buf exported before for any other allocation is refused
//    (catches (1), and (2) at equal sizes). The same allocation may get its dma-buf back.
// A refused export's descriptor is closed (the API hands it to the caller) and the caller falls back as for any
// refused export (hipIpc handle for explicit registrations, the bounce allocation for eager ones).
// The node lock and the registry are files of this user in /tmp (another user's processes keep their own). The lock is
// waited for at most NCCL_AMD_DMABUF_LOCK_TIMEOUT_MS (5 s; it is held only across one runtime call): a process stuck
// while holding it delays the others that long, then they go on without it (said once).
static std::string nodeFile(const char* what) {
  const char* dir = paramStr("NCCL_AMD_DMABUF_NODE_DIR");  // tests: a directory of their own
  return std::string(dir ? dir : "/tmp") + "/.ncclamd_dmabuf." + std::to_string((unsigned long)getuid()) + "." + what;
}
struct NodeLock {  // every dma-buf export and import of the library's processes on a node, one at a time
  int fd = -1;
  NodeLock() {
    static const int lockFd = paramInt("NCCL_AMD_DMABUF_NODE_LOCK", 1)
                                  ? open(nodeFile("lock").c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600)
                                  : -1;
    static const int64_t waitMs = paramInt("NCCL_AMD_DMABUF_LOCK_TIMEOUT_MS", 5000);
    if (lockFd < 0) return;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(waitMs);
    while (flock(lockFd, LOCK_EX | LOCK_NB) != 0) {
      if (errno != EWOULDBLOCK && errno != EINTR) return;
      if (std::chrono::steady_clock::now() > deadline) {
        static std::atomic<bool> said{false};
        if (!said.exchange(true))
          WARN("ipc: %s held by another process for %lld ms: going on without it", nodeFile("lock").c_str(),
               (long long)waitMs);
        return;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    fd = lockFd;
  }
  ~NodeLock() {
    if (fd >= 0) (void)flock(fd, LOCK_UN);
  }
  bool held() const { return fd >= 0; }
};
struct ExportRec {
  uint64_t dev, ino, proc, base, id;
};
static uint64_t processId() {  // random per process (a forked child draws its own)
  static uint64_t id = 0;
  static pid_t owner = 0;
  if (owner != getpid()) {
    owner = getpid();
    id = ((uint64_t)randomNonce() << 32) ^ (uint64_t)randomNonce() ^ (uint64_t)owner;
  }
  return id;
}
// Looks `rec`'s dma-buf up in the node registry (caller holds the node lock): returns false — refuse — if another
// allocation exported it before; appends it otherwise. Without a readable registry only this process's record counts.
static bool registryAdmit(const ExportRec& rec, ExportRec* prior) {
  static std::vector<ExportRec> local;  // this process's exports (the fallback when the file is unusable)
  static const int regFd = open(nodeFile("reg").c_str(), O_RDWR | O_CREAT | O_APPEND | O_CLOEXEC, 0600);
  auto same = [&](const ExportRec& x) { return x.dev == rec.dev && x.ino == rec.ino; };
  auto mine = [&](const ExportRec& x) { return x.proc == rec.proc && x.base == rec.base && x.id == rec.id; };
  for (const ExportRec& x : local)
    if (same(x) && !mine(x)) return *prior = x, false;
  if (regFd >= 0) {
    ExportRec buf[256];
    off_t off = 0;
    for (;;) {
      const ssize_t got = pread(regFd, buf, sizeof(buf), off);
      if (got <= 0) break;
      for (size_t k = 0; k < (size_t)got / sizeof(ExportRec); k++)
        if (same(buf[k]) && !mine(buf[k])) return *prior = buf[k], false;
      off += got;
    }
    (void)!write(regFd, &rec, sizeof(rec));
  }
  local.push_back(rec);
  return true;
}

static uint64_t allocationId(void* p) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint64_t)id;
}

// The checks above on a descriptor an export handed back for [base, +size) (the caller holds the node lock): true =
// admitted (and recorded); false = refused, `fd` closed. Separate from the export so a CPU test can drive it with
// descriptors of its own (tests/native/export_check_test.cc).
bool ipcAdmitExport(int fd, void* base, size_t size) {
  struct stat st;
  if (fstat(fd, &st) != 0) {
    WARN("ipc: dma-buf export of %p (+%zu MiB) returned fd %d, which fstat refuses: %s", base, size >> 20, fd,
         strerror(errno));
    return false;
  }
  const off_t dsize = lseek(fd, 0, SEEK_END);
  (void)lseek(fd, 0, SEEK_SET);
  if (dsize >= 0 && ((uint64_t)dsize < size || (uint64_t)dsize >= size + ((uint64_t)2 << 20))) {
    WARN("ipc: dma-buf export of %p (+%zu MiB) handed back a dma-buf of %lld bytes (ino %lu): refused (another "
         "allocation's)", base, size >> 20, (long long)dsize, (unsigned long)st.st_ino);
    close(fd);
    return false;
  }
  const ExportRec rec = {(uint64_t)st.st_dev, (uint64_t)st.st_ino, processId(), (uint64_t)base, allocationId(base)};
  ExportRec prior;
  if (!registryAdmit(rec, &prior)) {
    WARN("ipc: dma-buf export of %p (+%zu MiB) handed back dma-buf ino %lu, exported before for %lx%s: refused "
         "(another allocation's)", base, size >> 20, (unsigned long)st.st_ino, (unsigned long)prior.base,
         prior.proc == rec.proc ? "" : " by another process");
    close(fd);
    return false;
  }
  TRACE("ipc: exported %p (+%zu MiB) as fd %d, dma-buf ino %lu", base, size >> 20, fd, (unsigned long)st.st_ino);
  return true;
}

hipError_t ipcExportDmaBuf(void* base, size_t size, int* fd, int attempts) {
  hipError_t e = hipErrorInvalidValue;
  for (int attempt = 0; attempt < attempts; attempt++) {
    if (attempt) std::this_thread::sleep_for(std::chrono::milliseconds(1 << (attempt - 1)));
    std::lock_guard<std::mutex> g(gMapMu);
    NodeLock nl;
    e = hipMemGetHandleForAddressRange(fd, (hipDeviceptr_t)base, size, hipMemRangeHandleTypeDmaBufFd, 0);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    if (!ipcAdmitExport(*fd, base, size)) {
      *fd = -1;
      return hipErrorInvalidValue;
    }
    if (attempt) INFO("ipc: dma-buf export of %p (+%zu MiB) succeeded at attempt %d", base, size >> 20, attempt + 1);
    return e;
  }
  return e;
}

ncclResult_t ipcExport(ncclComm* comm, void* base, size_t size, IpcDesc* d) {
  memset(d, 0, sizeof(*d));
  d->size = size;
  if (ipcLegacy()) {
    const HipRuntimeInfo& rt = hipRuntimeInfo();
    if (!ipcLegacyAllowed(rt.version, size, true)) {
      WARN("ipc: NCCL_AMD_IPC=legacy refused on HIP runtime %d (%s): its hipIpcOpenMemHandle stalls on "
           "allocations of 2 GiB or more; use the default dma-buf path", rt.version, rt.path);
      return ncclSystemError;
    }
    d->legacy = 1;
    HIPCHECK(hipIpcGetMemHandle(&d->handle, base));
    return ncclSuccess;
  }
  if (!comm->fdServer) {
    WARN("ipc: no fd server on rank %d", comm->rank);
    return ncclInternalError;
  }
  int fd = -1;
  hipError_t e = paramInt("NCCL_AMD_IPC_FAIL_EXPORT", 0)  // tests: exercise the fallback below
                     ? hipErrorInvalidValue
                     : ipcExportDmaBuf(base, size, &fd);
  const int err = errno;
  if (e != hipSuccess) {
    // Seen on the one-GPU box after many communicators and registrations in one process (bench.py's N = 4
    // rehearsal): the runtime refuses the dma-buf export of a fresh slab with "invalid argument". The slab then
    // goes to its peers as a hipIpc handle where the runtime can open one (below 2 GiB, or a 7.2+ runtime)
    // instead of failing the communicator; the details are logged for the report.
    (void)hipGetLastError();
    hipDeviceptr_t ab = nullptr;
    size_t as = 0;
    const hipError_t ea = hipMemGetAddressRange(&ab, &as, (hipDeviceptr_t)base);
    (void)hipGetLastError();
    const bool fallback = ipcLegacyAllowed(hipRuntimeInfo().version, size, false) &&
                          hipIpcGetMemHandle(&d->handle, base) == hipSuccess;
    (void)hipGetLastError();
    WARN("ipc: dma-buf export of %p (+%zu MiB) failed: %s (allocation %p +%zu MiB: %s; errno %d %s)%s", base,
         size >> 20, hipGetErrorString(e), (void*)ab, as >> 20, hipGetErrorString(ea), err, strerror(err),
         fallback ? "; peers open a hipIpc handle instead" : "");
    if (!fallback) return ncclUnhandledCudaError;
    d->legacy = 1;
    return ncclSuccess;
  }
  NCCLCHECK(ipcPublish(comm, fd, size, d));
  // A hipIpc handle rides along where the runtime can open it (below 2 GiB, or a 7.2+ runtime): an importer
  // whose runtime cannot map the dma-buf (never seen on one GPU; the first multi-GPU node decides) falls back
  // to it with a warning instead of failing the communicator.
  if (ipcLegacyAllowed(hipRuntimeInfo().version, size, false) && !paramInt("NCCL_AMD_IPC_NO_FALLBACK", 0)) {
    if (hipIpcGetMemHandle(&d->handle, base) == hipSuccess) d->hasHandle = 1;
    else (void)hipGetLastError();
  }
  return ncclSuccess;
}

// Serve fd (owned from here on) under a fresh key until ipcUnexport / ipcServerStop.
ncclResult_t ipcPublish(ncclComm* comm, int fd, size_t size, IpcDesc* d) {
  FdServer* s = comm->fdServer;
  if (!s) {
    close(fd);
    return ncclInternalError;
  }
  d->size = size;
  d->legacy = 0;
  d->hasHandle = 0;
  d->key = gKeySerial++;
  memcpy(d->server, s->name, sizeof(d->server));
  std::lock_guard<std::mutex> g(s->mu);
  s->table[d->key] = fd;
  return ncclSuccess;
}

// Stop serving an export (every peer has imported it: its mapping keeps the memory referenced).
void ipcUnexport(ncclComm* comm, const IpcDesc& d) {
  FdServer* s = comm->fdServer;
  if (d.legacy || !s) return;
  std::lock_guard<std::mutex> g(s->mu);
  auto it = s->table.find(d.key);
  if (it == s->table.end()) return;
  close(it->second);
  s->table.erase(it);
}

// Connect to the fd server named `server` (retrying until the IPC timeout: the peer may still be starting).
static ncclResult_t connectServer(const char* server, int* out, bool retry) {
  struct sockaddr_un a;
  socklen_t al = abstractAddr(server, &a);
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(ipcTimeoutMs());
  while (true) {
    int c = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    SYSCHECK(c >= 0, "socket");
    if (connect(c, (struct sockaddr*)&a, al) == 0) {
      setTimeouts(c);
      *out = c;
      return ncclSuccess;
    }
    int err = errno;
    close(c);
    if (!retry || std::chrono::steady_clock::now() > deadline) {
      if (retry) WARN("ipc: connect to %s failed: %s", server, strerror(err));
      return ncclRemoteError;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

// One request / reply round trip (fd attached to the request and / or received with the reply).
static ncclResult_t ipcCall(const char* server, const IpcRequest& q, int sendFd, IpcReply* r, int* recvFd, bool retry) {
  int c = -1;
  NCCLCHECK(connectServer(server, &c, retry));
  int fd = -1;
  r->status = -1;
  bool ok = sendWithFd(c, &q, sizeof(q), sendFd) == 0 && recvWithFd(c, r, sizeof(*r), &fd) == 0;
  close(c);
  if (recvFd) *recvFd = fd;
  else if (fd >= 0) close(fd);
  return ok ? ncclSuccess : ncclRemoteError;
}

ncclResult_t ipcFetchFd(const IpcDesc& d, int* out) {
  IpcRequest q;
  memset(&q, 0, sizeof(q));
  q.op = IPC_FETCH;
  q.from = -1;
  q.key = d.key;
  IpcReply r;
  int fd = -1;
  ncclResult_t res = ipcCall(d.server, q, -1, &r, &fd, true);
  if (res != ncclSuccess && res != ncclRemoteError) return res;
  if (fd < 0 || r.status != 0) {
    if (fd >= 0) close(fd);
    WARN("ipc: %s did not hand over export %llu (%s)", d.server, (unsigned long long)d.key,
         r.status == 0 ? "no descriptor attached" : "unknown key, timeout or peer gone");
    return ncclRemoteError;
  }
  *out = fd;
  return ncclSuccess;
}

ncclResult_t ipcRemoteImportHandle(const char* server, int rank, uint64_t tag, const hipIpcMemHandle_t& h,
                                   uint64_t size, uint64_t* addr) {
  IpcRequest q;
  memset(&q, 0, sizeof(q));
  q.op = IPC_IMPORT;
  q.from = rank;
  q.key = tag;
  q.size = size;
  q.legacy = 1;
  q.handle = h;
  IpcReply r;
  NCCLCHECK(ipcCall(server, q, -1, &r, nullptr, true));
  if (r.status != 0) {
    WARN("ipc: %s could not open the hipIpc handle of a registered buffer of %zu MiB", server, (size_t)(size >> 20));
    return ncclRemoteError;
  }
  *addr = r.value;
  return ncclSuccess;
}

ncclResult_t ipcRemoteImport(const char* server, int rank, uint64_t tag, int fd, uint64_t size, uint64_t* addr) {
  IpcRequest q;
  memset(&q, 0, sizeof(q));
  q.op = IPC_IMPORT;
  q.from = rank;
  q.key = tag;
  q.size = size;
  IpcReply r;
  NCCLCHECK(ipcCall(server, q, fd, &r, nullptr, true));
  if (r.status != 0) {
    WARN("ipc: %s could not map a registered buffer of %zu MiB", server, (size_t)(size >> 20));
    return ncclRemoteError;
  }
  *addr = r.value;
  return ncclSuccess;
}

void ipcRemoteRelease(const char* server, int rank, uint64_t tag) {
  IpcRequest q;
  memset(&q, 0, sizeof(q));
  q.op = IPC_RELEASE;
  q.from = rank;
  q.key = tag;
  IpcReply r;
  (void)ipcCall(server, q, -1, &r, nullptr, false);  // a peer already gone has released everything itself
}

uint64_t ipcNewTag() { return gKeySerial++; }

// Close an imported descriptor unless the runtime already did: its number may by then name another file of
// this process (opened by another thread meanwhile), so only while it still names the imported dma-buf.
static bool closeIfMine(int fd, uint64_t dev, uint64_t ino) {
  struct stat st;
  const bool mine = fd >= 0 && fstat(fd, &st) == 0 && (uint64_t)st.st_dev == dev && (uint64_t)st.st_ino == ino;
  if (mine) close(fd);
  return mine;
}

static ncclResult_t importLegacy(const IpcDesc& d, IpcImport* out) {
  std::lock_guard<std::mutex> g(gMapMu);
  HIPCHECK(hipIpcOpenMemHandle(&out->ptr, d.handle, hipIpcMemLazyEnablePeerAccess));
  out->legacy = 1;
  return ncclSuccess;
}

// Map a dma-buf fd (owned from here on: kept by the mapping, or closed on failure).
static ncclResult_t importFd(int fd, uint64_t size, IpcImport* out) {
  std::lock_guard<std::mutex> g(gMapMu);
  memset(out, 0, sizeof(*out));
  out->fd = -1;
  // the exporter checked its dma-buf's size against the allocation (ipcExportDmaBuf); the importer checks it against
  // the size it was asked to map, so a descriptor that names another allocation is never mapped in its place
  const off_t dsize = lseek(fd, 0, SEEK_END);
  (void)lseek(fd, 0, SEEK_SET);
  if (dsize >= 0 && ((uint64_t)dsize < size || (uint64_t)dsize >= size + ((uint64_t)2 << 20))) {
    close(fd);
    WARN("ipc: a dma-buf of %lld bytes was handed over for an allocation of %lu: refused", (long long)dsize,
         (unsigned long)size);
    return ncclSystemError;
  }
  hipExternalMemoryHandleDesc hd;
  memset(&hd, 0, sizeof(hd));
  hd.type = hipExternalMemoryHandleTypeOpaqueFd;
  hd.handle.fd = fd;
  hd.size = size;
  hipExternalMemory_t em = nullptr;
  hipError_t e;
  {
    NodeLock nl;
    e = hipImportExternalMemory(&em, &hd);
  }
  if (e != hipSuccess) {
    close(fd);
    WARN("ipc: hipImportExternalMemory(%zu MiB): %s", (size_t)(size >> 20), hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  // Descriptor ownership: kept until the mapping is released (ipcRelease), then closed if the runtime has
  // not closed it itself (the runtime's behaviour is logged at TRACE level)
  TRACE("ipc: imported %zu MiB (fd %d %s after import)", (size_t)(size >> 20), fd,
        fcntl(fd, F_GETFD) != -1 ? "open" : "closed by the runtime");
  out->fd = fd;
  struct stat st;
  if (fstat(fd, &st) == 0) {
    out->fdDev = (uint64_t)st.st_dev;
    out->fdIno = (uint64_t)st.st_ino;
  }
  hipExternalMemoryBufferDesc bd;
  memset(&bd, 0, sizeof(bd));
  bd.offset = 0;
  bd.size = size;
  void* p = nullptr;
  e = hipExternalMemoryGetMappedBuffer(&p, em, &bd);
  if (e != hipSuccess) {
    (void)hipDestroyExternalMemory(em);
    closeIfMine(fd, out->fdDev, out->fdIno);
    out->fd = -1;
    WARN("ipc: hipExternalMemoryGetMappedBuffer: %s", hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  out->ptr = p;
  out->size = size;
  out->ext = em;
  return ncclSuccess;
}

static ncclResult_t importDmaBuf(const IpcDesc& d, IpcImport* out) {
  int fd = -1;
  NCCLCHECK(ipcFetchFd(d, &fd));
  if (paramInt("NCCL_AMD_IPC_FAIL_DMABUF", 0)) {  // tests: exercise the fallback on a box where dma-buf works
    close(fd);
    WARN("ipc: NCCL_AMD_IPC_FAIL_DMABUF=1: refusing the dma-buf import");
    return ncclUnhandledCudaError;
  }
  return importFd(fd, d.size, out);
}

ncclResult_t ipcImport(const IpcDesc& d, IpcImport* out) {
  memset(out, 0, sizeof(*out));
  out->fd = -1;
  if (d.legacy) return importLegacy(d, out);
  ncclResult_t r = importDmaBuf(d, out);
  if (r == ncclSuccess || r == ncclRemoteError || !d.hasHandle) return r;  // exporter gone: nothing to fall back to
  (void)hipGetLastError();
  memset(out, 0, sizeof(*out));
  WARN("ipc: dma-buf import of %zu MiB from %s failed; falling back to its hipIpc handle", (size_t)(d.size >> 20),
       d.server);
  return importLegacy(d, out);
}

ncclResult_t ipcImportHandle(const IpcDesc& d, IpcImport* out) {
  memset(out, 0, sizeof(*out));
  out->fd = -1;
  if (!d.legacy && !d.hasHandle) {
    WARN("ipc: export %llu of %s carries no hipIpc handle to fall back to", (unsigned long long)d.key, d.server);
    return ncclSystemError;
  }
  return importLegacy(d, out);
}

void ipcRelease(IpcImport* m) {
  if (!m->ptr) return;
  std::lock_guard<std::mutex> g(gMapMu);
  releaseLocked(m);
}

static void releaseLocked(IpcImport* m) {  // caller holds gMapMu
  if (!m->ptr) return;
  TRACE("ipc: unmapping %p (%lu MiB, ino %lu)", m->ptr, (unsigned long)(m->size >> 20), (unsigned long)m->fdIno);
  if (m->legacy) {
    (void)hipIpcCloseMemHandle(m->ptr);
  } else {
    (void)hipFree(m->ptr);
    (void)hipDestroyExternalMemory((hipExternalMemory_t)m->ext);
    const bool closed = closeIfMine(m->fd, m->fdDev, m->fdIno);
    TRACE("ipc: released mapping (fd %d %s)", m->fd, closed ? "still open: closed it" : "closed by the runtime");
  }
  memset(m, 0, sizeof(*m));
}

}  // namespace ncclamd

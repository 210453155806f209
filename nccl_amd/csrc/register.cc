// register.cc — buffer registration and symmetric windows.
//
// Reference: src/register/register.cc:154-200 (ncclCommRegister / ncclCommDeregister: local, refcounted
// registration), src/register/coll_reg.cc:326-395 (a ring collective on registered buffers: the buffer is
// IPC-registered with every peer, src/transport/p2p.cc ipcRegisterBuffer, and the kernels exchange the peers'
// addresses of it at run time, src/device/prims_simple.h:748-846 ptrExchange), src/enqueue.cc:283
// (NCCL_GRAPH_REGISTER: buffers of captured collectives are registered automatically),
// src/dev_runtime.cc:1331-1400, 1592-1610 (ncclCommWindowRegister as a group task: every rank maps every
// peer's window; ncclCommWindowDeregister; ncclWinGetUserPtr), src/device/symmetric/* (the window kernels).
//
// ncclCommRegister stays a LOCAL call, as in the reference: the allocation holding the buffer is exported as a
// dma-buf and each peer process maps it through its fd server (ipc.cc IMPORT request — the reference's proxy
// thread does the same for ipcRegisterBuffer), which answers where it landed. A collective whose buffers are
// registered then runs the zero-copy symmetric kernel in "registered" mode (kernels.h symKernel, regMode): each
// rank hands every peer its buffers as mapped in that peer through the flag block before its ENTER signal, so
// ranks need not agree on offsets, and nothing is staged. As in the reference, every rank registers the
// buffers it passes to such a collective (docs/userguide/source/usage/bufferreg.rst:55-56); windows
// (ncclCommWindowRegister) remain the collective, symmetric form.
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>

#include "core.h"

namespace ncclamd {

ncclResult_t commAllGather(ncclComm* comm, void* data, size_t bytesPerRank) {
  if (comm->nRanks == 1) return ncclSuccess;
  if (comm->bootstrap) return bootstrapAllGather(comm->bootstrap, data, bytesPerRank);
  if (comm->clique) return cliqueAllGather(comm->clique.get(), comm->rank, data, bytesPerRank);
  WARN("rank %d: no bootstrap for a collective host exchange", comm->rank);
  return ncclInternalError;
}

struct WinInfo {  // exchanged by ncclCommWindowRegister
  int pid;
  int flags;
  uint64_t ptr;      // user pointer (valid in the owner's process)
  uint64_t base;     // its allocation's base
  uint64_t size;
  IpcDesc desc;      // the whole allocation, exported to other processes (ipc.cc)
};

static ncclResult_t ipcMap(ncclComm* comm, int peer, const WinInfo& w, char** out) {
  for (IpcMapping& m : comm->ipcMaps)
    if (m.peer == peer && m.base == w.base) {
      m.refs++;
      *out = (char*)m.map.ptr + (w.ptr - w.base);
      return ncclSuccess;
    }
  IpcMapping m = {peer, w.base, {}, 1};
  NCCLCHECK(ipcImport(w.desc, &m.map));
  comm->ipcMaps.push_back(m);
  *out = (char*)m.map.ptr + (w.ptr - w.base);
  return ncclSuccess;
}

static void ipcUnmap(ncclComm* comm, int peer, uint64_t base) {
  for (size_t i = 0; i < comm->ipcMaps.size(); i++) {
    IpcMapping& m = comm->ipcMaps[i];
    if (m.peer != peer || m.base != base) continue;
    if (--m.refs == 0) {
      ipcRelease(&m.map);
      comm->ipcMaps.erase(comm->ipcMaps.begin() + i);
    }
    return;
  }
}

static void windowRelease(ncclComm* comm, ncclWindow_vidmem* w);

static ncclResult_t windowRegister(ncclComm* comm, void* buff, size_t size, ncclWindow_t* win, int flags) {
  HIPCHECK(hipSetDevice(comm->device));
  std::vector<WinInfo> all(comm->nRanks);
  WinInfo& me = all[comm->rank];
  memset(&me, 0, sizeof(me));
  me.pid = getpid();
  me.flags = flags;
  me.ptr = (uint64_t)buff;
  me.size = size;
  hipDeviceptr_t base = nullptr;
  size_t allocSize = 0;
  HIPCHECK(hipMemGetAddressRange(&base, &allocSize, (hipDeviceptr_t)buff));
  me.base = (uint64_t)base;
  if ((uint64_t)buff + size > me.base + allocSize) {
    WARN("ncclCommWindowRegister: [%p, +%zu) is not inside one allocation", buff, size);
    return ncclInvalidArgument;
  }
  bool needIpc = false;
  for (const PeerInfo& p : comm->peers) needIpc |= p.pid != me.pid;
  if (needIpc) {
    NCCLCHECK(ipcServerStart(comm));
    NCCLCHECK(ipcExport(comm, (void*)base, allocSize, &me.desc));
  }
  ncclResult_t gres = commAllGather(comm, all.data(), sizeof(WinInfo));
  if (gres != ncclSuccess) {
    if (needIpc) ipcUnexport(comm, me.desc);
    return gres;
  }

  ncclWindow_vidmem* w = new ncclWindow_vidmem();
  ncclResult_t mapRes = ncclSuccess;
  w->comm = comm;
  w->userPtr = buff;
  w->size = size;
  w->flags = flags;
  for (int r = 0; r < comm->nRanks; r++) {
    const WinInfo& p = all[r];
    if ((p.flags & NCCL_WIN_COLL_SYMMETRIC) != (flags & NCCL_WIN_COLL_SYMMETRIC) || p.size != size) {
      if (flags & NCCL_WIN_COLL_SYMMETRIC)
        INFO("window %p: rank %d registered size %lu flags %d (mine %zu / %d): not symmetric", buff, r,
             (unsigned long)p.size, p.flags, size, flags);
      w->flags &= ~NCCL_WIN_COLL_SYMMETRIC;  // every rank sees the same table, so all agree
    }
    if (r == comm->rank || p.pid == me.pid) {
      w->peerPtr[r] = (char*)p.ptr;
      continue;
    }
    ncclResult_t res = ipcMap(comm, r, p, &w->peerPtr[r]);
    if (res != ncclSuccess) {
      mapRes = res;
      break;
    }
    w->peerBase[r] = p.base;
  }
  if (needIpc) {
    // Every rank joins this all-gather whatever its own imports gave: a rank that failed to map
    // a peer must not leave the others waiting in it. It carries each rank's outcome, so all ranks release
    // their mappings and return the same error together; on success every peer has mapped my allocation
    // (its mapping keeps it referenced) and the descriptor is no longer served.
    std::vector<char> sync(comm->nRanks, 0);
    sync[comm->rank] = mapRes == ncclSuccess ? 1 : 0;
    ncclResult_t bres = commAllGather(comm, sync.data(), 1);
    ipcUnexport(comm, me.desc);
    for (int r = 0; r < comm->nRanks && bres == ncclSuccess; r++)
      if (!sync[r]) bres = mapRes != ncclSuccess ? mapRes : ncclRemoteError;
    if (bres != ncclSuccess) {
      if (mapRes == ncclSuccess) WARN("ncclCommWindowRegister: a peer could not map its windows; releasing");
      windowRelease(comm, w);
      return bres;
    }
  } else if (mapRes != ncclSuccess) {
    windowRelease(comm, w);
    return mapRes;
  }
  comm->windows.push_back(w);
  *win = w;
  INFO("rank %d: window %p size %zu flags %d registered", comm->rank, buff, size, w->flags);
  return ncclSuccess;
}

static void windowRelease(ncclComm* comm, ncclWindow_vidmem* w) {
  for (int r = 0; r < comm->nRanks; r++)
    if (w->peerBase[r]) ipcUnmap(comm, r, w->peerBase[r]);
  delete w;
}

ncclWindow_vidmem* findSymWindow(ncclComm* comm, const void* p, size_t bytes) {
  uintptr_t a = (uintptr_t)p;
  for (ncclWindow_vidmem* w : comm->windows) {
    uintptr_t b = (uintptr_t)w->userPtr;
    if ((w->flags & NCCL_WIN_COLL_SYMMETRIC) && a >= b && a + bytes <= b + w->size) return w;
  }
  return nullptr;
}

// ---- registered buffers (ncclCommRegister, NCCL_GRAPH_REGISTER) ----

static uint64_t bufferIdOf(const void* p) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint64_t)id;
}

// Drop the peers' mappings of an allocation (the caller made sure no kernel of this rank still uses it; a
// peer's kernels stop reading it before this rank's kernel passes its DONE handshake).
static void regRelease(ncclComm* comm, RegAlloc* ra) {
  for (int r = 0; r < comm->nRanks; r++)
    if (ra->imported[r]) ipcRemoteRelease(comm->peers[r].fdServer, comm->rank, ra->tag);
  delete ra;
}

// Map the allocation [base, +size) into every peer process (same process: its own pointer).
static ncclResult_t regCreate(ncclComm* comm, uint64_t base, uint64_t size, uint64_t id, RegAlloc** out) {
  RegAlloc* ra = new RegAlloc();
  memset(ra, 0, sizeof(*ra));
  ra->base = base;
  ra->size = size;
  ra->bufferId = id;
  ra->tag = ipcNewTag();
  ra->usable = true;
  const int me = comm->rank, pid = getpid();
  int fd = -1;
  ncclResult_t res = ncclSuccess;
  for (int r = 0; r < comm->nRanks && res == ncclSuccess; r++) {
    if (r == me || comm->peers[r].pid == pid) {  // one address space (peer access enabled at init)
      ra->rmt[r] = base;
      continue;
    }
    if (!comm->regIpcAll) {  // some rank runs no fd server (NCCL_AMD_IPC=legacy): every rank stays staged
      INFO("rank %d: registered buffer %lx stays local (a rank of this communicator has no fd server)", me,
           (unsigned long)base);
      ra->usable = false;
      break;
    }
    if (fd < 0) {
      hipError_t e = paramInt("NCCL_AMD_REG_FAIL_EXPORT", 0)  // tests: a registration that fails on one rank only
                         ? hipErrorInvalidValue
                         : hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)base, size, hipMemRangeHandleTypeDmaBufFd, 0);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        WARN("ncclCommRegister: allocation %lx (+%zu) cannot be exported: %s", (unsigned long)base, (size_t)size,
             hipGetErrorString(e));
        res = ncclUnhandledCudaError;
        break;
      }
    }
    res = ipcRemoteImport(comm->peers[r].fdServer, me, ra->tag, fd, size, &ra->rmt[r]);
    if (res == ncclSuccess) ra->imported[r] = true;
  }
  if (fd >= 0) close(fd);
  if (res != ncclSuccess) {
    regRelease(comm, ra);
    return res;
  }
  TRACE("rank %d: registered allocation %lx +%zu MiB (tag %lu, %s)", me, (unsigned long)base, (size_t)(size >> 20),
        (unsigned long)ra->tag, ra->usable ? "mapped by every peer" : "local only");
  *out = ra;
  return ncclSuccess;
}

// Find or create the registration of the allocation holding [buff, +size) and take a reference on it.
static ncclResult_t regAcquire(ncclComm* comm, const void* buff, size_t size, bool graph, RegAlloc** out) {
  hipDeviceptr_t base = nullptr;
  size_t allocSize = 0;
  HIPCHECK(hipMemGetAddressRange(&base, &allocSize, (hipDeviceptr_t)buff));
  if ((uint64_t)buff + size > (uint64_t)base + allocSize) {
    WARN("ncclCommRegister: [%p, +%zu) is not inside one allocation", buff, size);
    return ncclInvalidArgument;
  }
  const uint64_t id = bufferIdOf(buff);
  RegAlloc* ra = nullptr;
  for (RegAlloc* x : comm->regs)
    if (x->base == (uint64_t)base && x->size == allocSize && x->bufferId == id) ra = x;
  if (!ra) {
    NCCLCHECK(regCreate(comm, (uint64_t)base, allocSize, id, &ra));
    comm->regs.push_back(ra);
  }
  if (graph) ra->graphRefs++;
  else ra->localRefs++;
  *out = ra;
  return ncclSuccess;
}

static void regPut(ncclComm* comm, RegAlloc* ra, bool graph) {
  if (graph) ra->graphRefs--;
  else ra->localRefs--;
  if (ra->localRefs > 0 || ra->graphRefs > 0) return;
  comm->regs.erase(std::find(comm->regs.begin(), comm->regs.end(), ra));
  regRelease(comm, ra);
}

// The usable registration holding [p, +bytes), or nullptr. A registration whose allocation was freed and its
// range handed out again (another buffer id) is never used; an automatic (graph) one is dropped then.
static RegAlloc* regFind(ncclComm* comm, const void* p, size_t bytes, bool capturing) {
  const uint64_t a = (uint64_t)p;
  uint64_t id = 0;
  bool haveId = false;
  for (size_t i = 0; i < comm->regs.size(); i++) {
    RegAlloc* ra = comm->regs[i];
    if (a < ra->base || a + bytes > ra->base + ra->size) continue;
    if (!haveId) {
      id = bufferIdOf(p);
      haveId = true;
    }
    if (id != ra->bufferId) {  // stale: the registered allocation is gone
      if (ra->localRefs == 0) {
        INFO("rank %d: allocation %lx was freed and re-allocated since a captured collective registered it",
             comm->rank, (unsigned long)ra->base);
        ra->graphRefs = 1;
        regPut(comm, ra, true);
        i--;
      }
      continue;
    }
    if (!ra->usable || (ra->localRefs == 0 && !capturing)) return nullptr;  // automatic ones: captures only
    return ra;
  }
  return nullptr;
}

// Graph-held references (NCCL_GRAPH_REGISTER). Every captured use of a registration holds one reference, owned by a
// hipUserObject retained by the capturing graph: the runtime destroys the object when the graph and every executable
// instantiated from it are gone (scripts/user_object_probe.hip: on torch's HIP runtime and on /opt/rocm's, the
// executable keeps it after hipGraphDestroy — PyTorch destroys the hipGraph_t right after instantiating it). The
// destructor makes no HIP call; it queues (comm, tag), and the next blocking call on that communicator drops the
// reference (regDrainGraphReleases) — the last one sends the peers RELEASE, as ncclCommDeregister does (the reference
// ties graph registrations to the graph the same way, src/register/register.cc graph cleanup). Tags are unique in the
// process, so a token that outlives its communicator matches nothing.
struct GraphRelease {
  ncclComm* comm;
  uint64_t tag;
};
// never destroyed: the runtime may destroy a leftover executable graph, and so run graphReleaseFn, while the
// process exits, after this library's static destructors
static std::mutex& graphRelMu() {
  static std::mutex* m = new std::mutex();
  return *m;
}
static std::vector<GraphRelease>& graphRel() {
  static std::vector<GraphRelease>* v = new std::vector<GraphRelease>();
  return *v;
}

static void graphReleaseFn(void* p) {
  GraphRelease* g = (GraphRelease*)p;
  {
    std::lock_guard<std::mutex> lk(graphRelMu());
    graphRel().push_back(*g);
  }
  delete g;
}

// Take a graph reference on `ra` (unless regAcquire just took it: `counted`) for the graph being captured on `stream`.
// Without a user object (a runtime that refuses one) the reference stays until the communicator is destroyed.
static void graphHold(ncclComm* comm, RegAlloc* ra, hipStream_t stream, bool counted) {
  if (!counted) ra->graphRefs++;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nDeps = 0;
  if (hipStreamGetCaptureInfo_v2(stream, &st, &id, &g, &deps, &nDeps) != hipSuccess || st != hipStreamCaptureStatusActive ||
      g == nullptr) {
    (void)hipGetLastError();
    return;
  }
  GraphRelease* tok = new GraphRelease{comm, ra->tag};
  hipUserObject_t obj = nullptr;
  if (hipUserObjectCreate(&obj, tok, graphReleaseFn, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
    (void)hipGetLastError();
    delete tok;
    return;
  }
  if (hipGraphRetainUserObject(g, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipUserObjectRelease(obj, 1);  // its destructor queues the release of the reference taken above
  }
}

void regDrainGraphReleases(ncclComm* comm) {
  std::vector<uint64_t> tags;
  {
    std::lock_guard<std::mutex> lk(graphRelMu());
    std::vector<GraphRelease>& rel = graphRel();
    for (size_t i = 0; i < rel.size();)
      if (rel[i].comm == comm) {
        tags.push_back(rel[i].tag);
        rel[i] = rel.back();
        rel.pop_back();
      } else {
        i++;
      }
  }
  for (uint64_t tag : tags)
    for (RegAlloc* ra : comm->regs)
      if (ra->tag == tag && ra->graphRefs > 0) {
        const bool last = ra->graphRefs == 1 && ra->localRefs == 0;
        if (last)
          INFO("rank %d: automatic registration of allocation %lx released (its graphs are gone)", comm->rank,
               (unsigned long)ra->base);
        regPut(comm, ra, true);
        break;
      }
}

bool regLookup(ncclComm* comm, hipStream_t stream, const void* send, size_t sendBytes, const void* recv,
               size_t recvBytes, const char** rmtSend, char** rmtRecv) {
  if (comm->nRanks == 1) return false;
  bool capturing = false;
  if (comm->tune.graphRegister) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    capturing = hipStreamIsCapturing(stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
    (void)hipGetLastError();
  }
  // graph references whose graphs are gone are dropped BEFORE the lookup: dropping one may free a registration the
  // lookup would otherwise hand back
  if (capturing) regDrainGraphReleases(comm);
  if (comm->regs.empty() && !capturing) return false;
  RegAlloc* rs = send ? regFind(comm, send, sendBytes, capturing) : nullptr;
  RegAlloc* rr = regFind(comm, recv, recvBytes, capturing);
  if (capturing) {
    // NCCL_GRAPH_REGISTER (reference enqueue.cc:283, coll_reg.cc:383-387): a captured collective registers its
    // buffers itself and holds them for the graph's lifetime (graphHold; a registration whose range is freed and
    // re-allocated is dropped earlier, regFind)
    // (relaxed capture mode around the export: the capture of this thread stays valid whatever the runtime
    // deems unsafe among the calls below)
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    RegAlloc* x = nullptr;
    ncclResult_t rsRes = ncclSuccess, rrRes = ncclSuccess;
    if (send && rs) {
      graphHold(comm, rs, stream, false);
    } else if (send && (rsRes = regAcquire(comm, send, sendBytes, true, &x)) == ncclSuccess) {
      graphHold(comm, x, stream, true);
      rs = x->usable ? x : nullptr;
    }
    if (rr) {
      graphHold(comm, rr, stream, false);
    } else if ((rrRes = regAcquire(comm, recv, recvBytes, true, &x)) == ncclSuccess) {
      graphHold(comm, x, stream, true);
      rr = x->usable ? x : nullptr;
    }
    // a rank whose auto-registration failed captures the staged kernel while its peers may capture the zero-copy
    // one: the replay then fails fast on every rank with a kernel-mismatch error (kernels.h WaitProbe) instead of
    // waiting for the spin timeout; said here so the cause is on record
    if (rsRes != ncclSuccess || rrRes != ncclSuccess)
      WARN("rank %d: graph registration of a captured collective's buffers failed (%d): this rank captures the staged "
           "kernel; if its peers registered theirs, the replay stops with a kernel-mismatch error (set "
           "NCCL_GRAPH_REGISTER=0 on every rank to avoid it)", comm->rank, (int)(rsRes != ncclSuccess ? rsRes : rrRes));
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    (void)hipGetLastError();
  }
  if (!rr || (send && !rs)) return false;
  for (int r = 0; r < comm->nRanks; r++) {
    rmtSend[r] = send ? (const char*)(rs->rmt[r] + ((uint64_t)send - rs->base)) : nullptr;
    rmtRecv[r] = (char*)(rr->rmt[r] + ((uint64_t)recv - rr->base));
  }
  return true;
}

void windowsFree(ncclComm* comm, bool notifyPeers) {
  (void)hipSetDevice(comm->device);
  {  // graph releases still queued for this communicator: every registration goes below anyway
    std::lock_guard<std::mutex> lk(graphRelMu());
    std::vector<GraphRelease>& rel = graphRel();
    rel.erase(std::remove_if(rel.begin(), rel.end(), [&](const GraphRelease& g) { return g.comm == comm; }), rel.end());
  }
  for (ncclWindow_vidmem* w : comm->windows) windowRelease(comm, w);
  comm->windows.clear();
  for (IpcMapping& m : comm->ipcMaps) ipcRelease(&m.map);
  comm->ipcMaps.clear();
  for (RegHandle* h : comm->regHandles) delete h;
  comm->regHandles.clear();
  // Destroy (notifyPeers): best-effort RELEASE requests (no retry: a peer already tearing down has no server
  // left, and its ipcServerStop drops every mapping it held for us anyway), so a peer whose communicator lives on
  // does not keep this rank's registered allocations — graph auto-registrations included — mapped until then
  // (the reference drops them with the registration, src/register/register.cc). Abort sends nothing.
  for (RegAlloc* ra : comm->regs) {
    if (notifyPeers) regRelease(comm, ra);
    else delete ra;
  }
  comm->regs.clear();
}

}  // namespace ncclamd

using namespace ncclamd;

#define NCCL_ALIAS(ret, name, ...) extern "C" __attribute__((visibility("default"), alias(#name))) ret p##name(__VA_ARGS__);

NCCL_EXPORT ncclResult_t ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle) {
  NCCLCHECK(commCheck(comm, "ncclCommRegister", "comm"));
  ipcDrainReleases();
  regDrainGraphReleases(comm);
  if (handle == nullptr) {
    WARN("ncclCommRegister : handle argument is NULL");
    return ncclInvalidArgument;
  }
  *handle = nullptr;
  if (buff == nullptr || size == 0) {
    WARN("ncclCommRegister : invalid buffer %p / size %zu", buff, size);
    return ncclInvalidArgument;
  }
  int st = comm->asyncResult.load();
  if (st != ncclSuccess) return st == ncclInProgress ? ncclInProgress : ncclInvalidUsage;
  ROCTX_RANGE("ncclCommRegister comm=%p size=%zu", (void*)comm, size);
  RegHandle* h = new RegHandle{buff, size, nullptr};
  // NCCL_LOCAL_REGISTER=0: the handle only records the buffer (reference register.cc:156-159 returns NULL;
  // a handle is kept here so that ncclCommDeregister of it stays valid)
  if (comm->tune.localRegister && comm->nRanks > 1) {
    DeviceRestore restore;
    HIPCHECK(hipSetDevice(comm->device));
    ncclResult_t res = regAcquire(comm, buff, size, false, &h->ra);
    if (res != ncclSuccess) {
      delete h;
      return res;
    }
  }
  comm->regHandles.push_back(h);
  *handle = h;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommRegister, const ncclComm_t, void*, size_t, void**)

NCCL_EXPORT ncclResult_t ncclCommDeregister(const ncclComm_t comm, void* handle) {
  NCCLCHECK(commCheck(comm, "ncclCommDeregister", "comm"));
  ipcDrainReleases();
  regDrainGraphReleases(comm);
  if (handle == nullptr) return ncclSuccess;  // reference commDeregister: NULL reg is a no-op
  auto it = std::find(comm->regHandles.begin(), comm->regHandles.end(), (RegHandle*)handle);
  if (it == comm->regHandles.end()) {
    WARN("Deregister: Could not find handle");
    return ncclInvalidUsage;
  }
  RegHandle* h = *it;
  comm->regHandles.erase(it);
  if (h->ra) {
    // collectives enqueued on the buffer may still run: wait for them before the peers unmap it
    DeviceRestore restore;
    HIPCHECK(hipSetDevice(comm->device));
    if (h->ra->localRefs == 1 && h->ra->graphRefs == 0) HIPCHECK(hipDeviceSynchronize());
    regPut(comm, h->ra, false);
  }
  delete h;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommDeregister, const ncclComm_t, void*)

NCCL_EXPORT ncclResult_t ncclCommWindowRegister(ncclComm_t comm, void* buff, size_t size, ncclWindow_t* win,
                                                int winFlags) {
  NCCLCHECK(commCheck(comm, "ncclCommWindowRegister", "comm"));
  ipcDrainReleases();
  regDrainGraphReleases(comm);
  if (win == nullptr) {
    WARN("ncclCommWindowRegister : win argument is NULL");
    return ncclInvalidArgument;
  }
  *win = nullptr;
  if (buff == nullptr || size == 0) {
    WARN("invalid pointer %p / size %zu", buff, size);
    return ncclInvalidArgument;
  }
  // a group task in the reference (dev_runtime.cc:1350-1366): inside a group every rank's registration
  // runs concurrently at ncclGroupEnd, so one thread may register the windows of all its ranks
  if (groupActive()) return groupDeferInit([=]() { return windowRegister(comm, buff, size, win, winFlags); });
  DeviceRestore restore;
  return windowRegister(comm, buff, size, win, winFlags);
}
NCCL_ALIAS(ncclResult_t, ncclCommWindowRegister, ncclComm_t, void*, size_t, ncclWindow_t*, int)

NCCL_EXPORT ncclResult_t ncclCommWindowDeregister(ncclComm_t comm, ncclWindow_t win) {
  NCCLCHECK(commCheck(comm, "ncclCommWindowDeregister", "comm"));
  ipcDrainReleases();
  regDrainGraphReleases(comm);
  if (win == nullptr) return ncclSuccess;
  auto it = std::find(comm->windows.begin(), comm->windows.end(), win);
  if (it == comm->windows.end() || win->comm != comm) {
    WARN("ncclCommWindowDeregister: unknown window %p", (void*)win);
    return ncclInvalidArgument;
  }
  // collectives enqueued on this window may still run: wait for the device before unmapping peers
  DeviceRestore restore;
  HIPCHECK(hipSetDevice(comm->device));
  HIPCHECK(hipDeviceSynchronize());
  comm->windows.erase(it);
  windowRelease(comm, win);
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommWindowDeregister, ncclComm_t, ncclWindow_t)

NCCL_EXPORT ncclResult_t ncclWinGetUserPtr(ncclComm_t comm, ncclWindow_t win, void** outUserPtr) {
  NCCLCHECK(commCheck(comm, "ncclWinGetUserPtr", "comm"));
  if (outUserPtr == nullptr || win == nullptr) {
    WARN("ncclWinGetUserPtr : NULL argument");
    return ncclInvalidArgument;
  }
  *outUserPtr = win->userPtr;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclWinGetUserPtr, ncclComm_t, ncclWindow_t, void**)

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
static void regFree(RegAlloc* ra) {
  if (ra->lastEv) (void)hipEventDestroy(ra->lastEv);
  delete ra;
}

static void regRelease(ncclComm* comm, RegAlloc* ra) {
  TRACE("rank %d: RELEASE of allocation %lx (id %lu, tag %lu) to its peers", comm->rank, (unsigned long)ra->base,
        (unsigned long)ra->bufferId, (unsigned long)ra->tag);
  for (int r = 0; r < comm->nRanks; r++)
    if (ra->imported[r]) ipcRemoteRelease(comm->peers[r].fdServer, comm->rank, ra->tag);
  regFree(ra);
}

static thread_local bool tBounceCreate = false;  // regCreate of the bounce allocation (bounceFor)

// Map the allocation [base, +size) into every peer process (same process: its own pointer). `deferRelease` (inside a
// collective): a registration failing after some peers mapped it is retired, not released from here.
static ncclResult_t regCreate(ncclComm* comm, uint64_t base, uint64_t size, uint64_t id, RegAlloc** out,
                              bool deferRelease) {
  RegAlloc* ra = new RegAlloc();
  memset(ra, 0, sizeof(*ra));
  ra->base = base;
  ra->size = size;
  ra->bufferId = id;
  ra->tag = ipcNewTag();
  ra->usable = true;
  const int me = comm->rank, pid = getpid();
  int fd = -1;
  bool useHandle = false;  // the dma-buf export was refused: peers open a hipIpc handle instead (below)
  hipIpcMemHandle_t handle;
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
    if (fd < 0 && !useHandle) {
      // tests: a registration failing on one rank (not the bounce allocation's: bounceFor)
      const bool failAll = !tBounceCreate && paramInt("NCCL_AMD_REG_FAIL_EXPORT", 0) != 0;
      hipError_t e = failAll || paramInt("NCCL_AMD_REG_FAIL_DMABUF", 0)  // tests: the hipIpc fallback below
                         ? hipErrorInvalidValue
                         : ipcExportDmaBuf((void*)base, size, &fd, deferRelease && !tBounceCreate ? 1 : 5);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        // The runtime sometimes refuses the dma-buf export of a fresh allocation ("invalid argument"; round 6's eager
        // churn, DESIGN.md §10.3: a re-allocation at the address of a just-freed registered allocation whose peers were
        // unmapping the old one), or hands back a dma-buf it exported before (refused by ipcExportDmaBuf), as it once
        // refused a fresh slab's (ipc.cc ipcExport). An explicit registration's peers then open a hipIpc handle instead
        // where the runtime gives one (below 2 GiB, or a 7.2+ runtime); the eager path runs the collective on the
        // bounce allocation (bounceFor).
        {
          std::lock_guard<std::mutex> g(ipcMapMutex());
          // not for the eager path's user allocations (deferRelease): those run on the bounce allocation instead,
          // which needs no handle of a range the runtime just refused (§10.3: its exports are not to be trusted); the
          // bounce allocation itself (the library's own) may go by handle
          useHandle = !failAll && (!deferRelease || tBounceCreate) &&
                      ipcLegacyAllowed(hipRuntimeInfo().version, size, false) &&
                      hipIpcGetMemHandle(&handle, (void*)base) == hipSuccess;
        }
        (void)hipGetLastError();
        if (useHandle) {
          INFO("rank %d: allocation %lx (+%zu MiB): dma-buf export refused (%s); its peers open a hipIpc handle", me,
               (unsigned long)base, (size_t)(size >> 20), hipGetErrorString(e));
        } else {
          WARN("ncclCommRegister: allocation %lx (+%zu) cannot be exported: %s", (unsigned long)base, (size_t)size,
               hipGetErrorString(e));
          res = ncclUnhandledCudaError;
          break;
        }
      }
    }
    res = useHandle ? ipcRemoteImportHandle(comm->peers[r].fdServer, me, ra->tag, handle, size, &ra->rmt[r])
                    : ipcRemoteImport(comm->peers[r].fdServer, me, ra->tag, fd, size, &ra->rmt[r]);
    if (res == ncclSuccess) ra->imported[r] = true;
  }
  if (fd >= 0) close(fd);
  if (res != ncclSuccess) {
    if (deferRelease) comm->regRetired.push_back(ra);  // never used by a kernel: released at the next progress call
    else regRelease(comm, ra);
    return res;
  }
  TRACE("rank %d: registered allocation %lx +%zu MiB (id %lu, tag %lu, %s; in rank %d at %lx)", me, (unsigned long)base,
        (size_t)(size >> 20), (unsigned long)id, (unsigned long)ra->tag, ra->usable ? "mapped by every peer" : "local only",
        (me + 1) % comm->nRanks, (unsigned long)ra->rmt[(me + 1) % comm->nRanks]);
  *out = ra;
  return ncclSuccess;
}

// Find or create the registration of the allocation holding [buff, +size) and take a reference of `kind` on it
// (an eager reference is one flag: the cache holds an allocation at most once).
static ncclResult_t regAcquire(ncclComm* comm, const void* buff, size_t size, int kind, RegAlloc** out,
                               bool deferRelease = false) {
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
    NCCLCHECK(regCreate(comm, (uint64_t)base, allocSize, id, &ra, deferRelease));
    comm->regs.push_back(ra);
  }
  if (kind == REF_GRAPH) ra->graphRefs++;
  else if (kind == REF_LOCAL) ra->localRefs++;
  else ra->eagerRef = true;
  *out = ra;
  return ncclSuccess;
}

// No collective may use `ra` any more: unlink it now, send its peers RELEASE at the next blocking entry point
// (regBlockingPoint) — never from inside a collective, where the socket round trips to every peer's fd server do not
// belong.
static void regRetire(ncclComm* comm, RegAlloc* ra) {
  comm->regs.erase(std::find(comm->regs.begin(), comm->regs.end(), ra));
  comm->regRetired.push_back(ra);
}

// Drop a reference of `kind`; the last one releases the registration (deferred: retired instead).
static void regPut(ncclComm* comm, RegAlloc* ra, int kind, bool defer = false) {
  if (kind == REF_GRAPH) ra->graphRefs--;
  else if (kind == REF_LOCAL) ra->localRefs--;
  else ra->eagerRef = false;
  if (ra->localRefs > 0 || ra->graphRefs > 0 || ra->eagerRef) return;
  if (defer) {
    regRetire(comm, ra);
    return;
  }
  comm->regs.erase(std::find(comm->regs.begin(), comm->regs.end(), ra));
  regRelease(comm, ra);
}

// The usable registration holding [p, +bytes), or nullptr. `automatic`: registrations held only by graphs or by
// the eager cache count too (a capture, or an eager collective). A registration whose allocation was freed and its
// range handed out again (another buffer id) is never used; one no ncclCommRegister handle holds is retired then.
static RegAlloc* regFind(ncclComm* comm, const void* p, size_t bytes, bool automatic) {
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
        INFO("rank %d: allocation %lx was freed and re-allocated since it was registered automatically", comm->rank,
             (unsigned long)ra->base);
        regRetire(comm, ra);
        i--;
      }
      continue;
    }
    if (!ra->usable || (ra->localRefs == 0 && !automatic)) return nullptr;
    return ra;
  }
  return nullptr;
}

// Graph-held references (NCCL_GRAPH_REGISTER). Every captured use of a registration holds one reference, owned by a
// hipUserObject retained by the capturing graph: the runtime destroys the object when the graph and every executable
// instantiated from it are gone (scripts/user_object_probe.hip: on torch's HIP runtime and on /opt/rocm's, the
// executable keeps it after hipGraphDestroy — PyTorch destroys the hipGraph_t right after instantiating it). The
// destructor makes no HIP call; it queues (comm, tag), and the next blocking call on that communicator drops the
// reference (regBlockingPoint) — the last one sends the peers RELEASE, as ncclCommDeregister does (the reference
// ties graph registrations to the graph the same way, src/register/register.cc graph cleanup). Tags are unique in the
// process; a token carries its communicator's generation, and a token whose communicator is gone is discarded when
// its graph dies instead of being queued for ever.
struct GraphRelease {
  ncclComm* comm;  // nullptr: inert (the graph never took ownership; the reference stays until comm destroy)
  uint64_t gen;
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
static std::vector<uint64_t>& liveGens() {  // generations of the communicators that hold graph references
  static std::vector<uint64_t>* v = new std::vector<uint64_t>();
  return *v;
}

static void graphReleaseFn(void* p) {
  GraphRelease* g = (GraphRelease*)p;
  {
    std::lock_guard<std::mutex> lk(graphRelMu());
    const std::vector<uint64_t>& live = liveGens();
    if (g->comm && std::find(live.begin(), live.end(), g->gen) != live.end()) graphRel().push_back(*g);
  }
  delete g;
}

size_t regGraphReleasesQueued() {  // tests (register.cc's own): tokens waiting for a drain, every communicator
  std::lock_guard<std::mutex> lk(graphRelMu());
  return graphRel().size();
}

// Take a graph reference on `ra` (unless regAcquire just took it: `counted`) for the graph being captured on `stream`.
// Without a user object (a runtime that refuses one, or refuses to let the graph retain it) the reference stays until
// the communicator is destroyed.
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
  if (comm->regGen == 0) {
    static std::atomic<uint64_t> nextGen{1};
    comm->regGen = nextGen++;
    std::lock_guard<std::mutex> lk(graphRelMu());
    liveGens().push_back(comm->regGen);
  }
  GraphRelease* tok = new GraphRelease{comm, comm->regGen, ra->tag};
  hipUserObject_t obj = nullptr;
  if (hipUserObjectCreate(&obj, tok, graphReleaseFn, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
    (void)hipGetLastError();
    delete tok;
    return;
  }
  const bool failRetain = paramInt("NCCL_AMD_TEST_RETAIN_FAIL", 0) != 0;  // tests: the runtime refuses the retain
  if (failRetain || hipGraphRetainUserObject(g, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
    (void)hipGetLastError();
    // The graph does not own the object, so releasing it runs the destructor now: make the token inert first, or the
    // next drain would drop the reference the captured zero-copy kernel still relies on and a later replay would
    // hand the peers unmapped addresses. The reference then lives until the communicator is destroyed.
    tok->comm = nullptr;
    INFO("rank %d: a graph could not retain the release object of allocation %lx; its registration is kept until the "
         "communicator is destroyed", comm->rank, (unsigned long)ra->base);
    (void)hipUserObjectRelease(obj, 1);
  }
}

// Drop the graph references whose graphs are gone. `defer` (inside a captured collective): a registration whose last
// reference goes is retired, its RELEASE requests sent at the next blocking entry point.
static void regDrainGraphReleases(ncclComm* comm, bool defer) {
  std::vector<uint64_t> tags;
  {
    std::lock_guard<std::mutex> lk(graphRelMu());
    std::vector<GraphRelease>& rel = graphRel();
    for (size_t i = 0; i < rel.size();)
      if (rel[i].comm == comm && rel[i].gen == comm->regGen) {
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
        const bool last = ra->graphRefs == 1 && ra->localRefs == 0 && !ra->eagerRef;
        if (last)
          INFO("rank %d: automatic registration of allocation %lx released (its graphs are gone)", comm->rank,
               (unsigned long)ra->base);
        regPut(comm, ra, REF_GRAPH, defer);
        break;
      }
}

// Eager registration (NCCL_AMD_EAGER_REGISTER=1; reference: IPC registration of a collective's buffers,
// src/register/coll_reg.cc:326-395, which NCCL does on request or under capture): planColl decides which ops qualify
// from what every rank shares (bytes, the size table), so every rank takes the same kernel. At blocking entry points:
static void bounceFree(ncclComm* comm, bool all, bool notifyPeers);

void regBlockingPoint(ncclComm* comm) {
  regDrainGraphReleases(comm, false);
  // eager cache upkeep: registrations whose allocation is gone go first (nothing of ours can use them: the range was
  // freed), then the least recently used beyond NCCL_AMD_EAGER_REGISTER_MAX, after this device's work is done (a
  // queued kernel may still hand the peers their addresses)
  std::vector<RegAlloc*> eager;
  const std::vector<RegAlloc*> regs = comm->regs;  // regPut below may unlink entries
  for (RegAlloc* ra : regs) {
    if (!ra->eagerRef) continue;
    if (bufferIdOf((const void*)ra->base) != ra->bufferId) {
      INFO("rank %d: eager registration of allocation %lx released (the allocation is gone)", comm->rank,
           (unsigned long)ra->base);
      regPut(comm, ra, REF_EAGER, true);
      continue;
    }
    eager.push_back(ra);
  }
  if ((int)eager.size() > comm->tune.eagerMax) {
    std::sort(eager.begin(), eager.end(), [](const RegAlloc* a, const RegAlloc* b) { return a->lastUse < b->lastUse; });
    const size_t drop = eager.size() - (size_t)comm->tune.eagerMax;
    DeviceRestore restore;  // the caller's current device survives the blocking call
    (void)hipSetDevice(comm->device);
    (void)hipDeviceSynchronize();
    for (size_t i = 0; i < drop; i++) regPut(comm, eager[i], REF_EAGER, true);
    INFO("rank %d: %zu eager registrations released (cache bound %d)", comm->rank, drop, comm->tune.eagerMax);
  }
  bounceFree(comm, /*all=*/false, /*notifyPeers=*/true);
  std::vector<RegAlloc*> retired;
  retired.swap(comm->regRetired);
  bool synced = false;
  for (RegAlloc* ra : retired) {
    if (ra->lastEv) (void)hipEventSynchronize(ra->lastEv);  // a blocking call: its last kernel may still run
    if (ra->evMissing && !synced) {
      DeviceRestore restore;
      (void)hipSetDevice(comm->device);
      (void)hipDeviceSynchronize();
      synced = true;
    }
    regRelease(comm, ra);
  }
}

// The upkeep above on the collective path, without waiting for anything: a loop that
// frees and re-allocates buffers and only issues collectives must neither grow the retired list nor keep its peers
// holding freed HBM until some blocking call. Per call, bounded work:
//  * freed allocations: the buffer id of two eager registrations (round robin) is checked; one whose allocation is
//    gone is retired (the lookup of a collective on a re-allocated range retires it too, regFind);
//  * the eager cache's bounds: beyond NCCL_AMD_EAGER_REGISTER_MAX registrations or NCCL_AMD_EAGER_REGISTER_MAX_BYTES,
//    the least recently used eager-only ones are retired (retiring is local: the kernel choice of later collectives,
//    which every rank must share, never depends on it — an evicted allocation is registered again on its next use);
//  * retired registrations whose last zero-copy kernel has completed (hipEventQuery, never a wait) get their peers'
//    RELEASE now, at most four per call (one socket round trip per importing peer each); the peers unmap at their own
//    next collective (ipcProgressReleases). A retired registration still in flight waits for a later call.
void regProgress(ncclComm* comm) {
  if (tPlanOnly || (comm->regs.empty() && comm->regRetired.empty() && comm->bounceOld.empty())) return;
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;  // event queries are not capture-safe in global mode
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  uint64_t eagerBytes = 0;
  int eagerCount = 0;
  for (RegAlloc* ra : comm->regs)
    if (ra->eagerRef && ra->localRefs == 0 && ra->graphRefs == 0) eagerBytes += ra->size, eagerCount++;
  for (int k = 0; k < 2 && !comm->regs.empty(); k++) {
    const size_t i = comm->regScan++ % comm->regs.size();
    RegAlloc* ra = comm->regs[i];
    if (!ra->eagerRef || bufferIdOf((const void*)ra->base) == ra->bufferId) continue;
    INFO("rank %d: eager registration of allocation %lx retired (the allocation is gone)", comm->rank,
         (unsigned long)ra->base);
    if (ra->localRefs == 0 && ra->graphRefs == 0) eagerBytes -= ra->size, eagerCount--;
    regPut(comm, ra, REF_EAGER, /*defer=*/true);
  }
  if (eagerCount > comm->tune.eagerMax || eagerBytes > (uint64_t)comm->tune.eagerMaxBytes) {
    std::vector<RegAlloc*> lru;
    for (RegAlloc* ra : comm->regs)
      if (ra->eagerRef && ra->localRefs == 0 && ra->graphRefs == 0) lru.push_back(ra);
    std::sort(lru.begin(), lru.end(), [](const RegAlloc* a, const RegAlloc* b) { return a->lastUse < b->lastUse; });
    size_t dropped = 0;
    // the most recent registration stays whatever its size (the collective that made it is in flight)
    for (size_t i = 0; i + 1 < lru.size() &&
                       (eagerCount > comm->tune.eagerMax || eagerBytes > (uint64_t)comm->tune.eagerMaxBytes); i++) {
      eagerBytes -= lru[i]->size;
      eagerCount--;
      regPut(comm, lru[i], REF_EAGER, /*defer=*/true);
      dropped++;
    }
    if (dropped)
      INFO("rank %d: %zu eager registrations retired (cache bounds %d / %.1f GiB)", comm->rank, dropped,
           comm->tune.eagerMax, comm->tune.eagerMaxBytes / (double)(1ull << 30));
  }
  // grown-out bounce allocations (bounceFor): once no planned collective still names one, its last copy-out has
  // completed and none of the library's kernels runs here (hipFree would wait for the device otherwise)
  for (size_t i = 0; i < comm->bounceOld.size();) {
    auto& x = comm->bounceOld[i];
    if (x.first->bouncePlans > 0 || hipEventQuery(comm->bounceEv) != hipSuccess || !ipcLibraryIdle()) {
      (void)hipGetLastError();
      break;
    }
    TRACE("rank %d: grown-out bounce allocation %lx freed", comm->rank, (unsigned long)x.first->base);
    regRelease(comm, x.first);
    {
      std::lock_guard<std::mutex> g(ipcMapMutex());
      (void)hipFree(x.second);
    }
    comm->bounceOld.erase(comm->bounceOld.begin() + i);
  }
  int sent = 0;
  for (size_t i = 0; i < comm->regRetired.size() && sent < 4;) {
    RegAlloc* ra = comm->regRetired[i];
    const hipError_t q = ra->evMissing ? hipErrorNotReady : ra->lastEv ? hipEventQuery(ra->lastEv) : hipSuccess;
    if (q == hipErrorNotReady) {
      static std::atomic<int> said{0};
      if (said.fetch_add(1) < 16)
        INFO("rank %d: retired registration %lx waits for its last kernel (%s)", comm->rank, (unsigned long)ra->base,
             ra->evMissing ? "no event" : "event not complete");
      i++;
      continue;
    }
    (void)hipGetLastError();
    comm->regRetired.erase(comm->regRetired.begin() + i);
    regRelease(comm, ra);
    sent++;
  }
  (void)hipThreadExchangeStreamCaptureMode(&mode);
}

void regRecordUse(ncclComm* comm, const SymPlan& sp) {
  if (!sp.args.regMode) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(sp.stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return;  // a capture holds its registrations through the graph's lifetime instead (graphHold)
  }
  for (RegAlloc* ra : sp.regUse) {
    if (!ra) continue;
    if (!ra->lastEv && hipEventCreateWithFlags(&ra->lastEv, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      ra->lastEv = nullptr;
      ra->evMissing = true;
      continue;
    }
    if (hipEventRecord(ra->lastEv, sp.stream) != hipSuccess) (void)hipGetLastError();
  }
  (void)comm;
}

thread_local bool tPlanOnly = false;

// The eager cache's failure memory (ncclComm::eagerFailed): the allocation holding p by (base, buffer id); a pointer
// the runtime knows no allocation of (hipMemGetAddressRange fails: host or managed memory) by (p, its buffer id).
static std::pair<uint64_t, uint64_t> eagerKey(const void* p) {
  hipDeviceptr_t base = nullptr;
  size_t allocSize = 0;
  if (hipMemGetAddressRange(&base, &allocSize, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    base = (hipDeviceptr_t)p;
  }
  return {(uint64_t)base, bufferIdOf(p)};
}
static bool eagerFailedBefore(ncclComm* comm, const void* p) {
  if (comm->eagerFailed.empty()) return false;
  const auto key = eagerKey(p);
  return std::find(comm->eagerFailed.begin(), comm->eagerFailed.end(), key) != comm->eagerFailed.end();
}

// Covered by an ncclCommRegister handle (the user registers the same buffers on every rank, bufferreg.rst:55-56). The
// eager cache does not count: its contents follow this rank's own LRU clock, and the tuner's regBuff must not differ
// between ranks, or a plugin keying on it would pick different kernels on different ranks.
bool regCovers(ncclComm* comm, const void* p, size_t bytes) {
  const uint64_t a = (uint64_t)p;
  for (const RegAlloc* ra : comm->regs)
    if (ra->usable && ra->localRefs > 0 && a >= ra->base && a + bytes <= ra->base + ra->size) return true;
  return false;
}

// ---- the bounce allocation ----
// An eager collective whose buffers this rank cannot register (the runtime refused the export — measured in round 6's
// collective-only churn, DESIGN.md §10.3 — or host memory) would leave this rank on the staged kernel while its peers
// run zero-copy: a kernel-mismatch error on every rank. It runs zero-copy on the bounce allocation instead: one
// allocation of the library per communicator, registered with every peer once, the input copied in before the kernel
// and the output copied out after, on the collective's stream (the kernel's DONE handshake: no peer reads it once this
// rank's kernel has ended). The peers cannot tell. Grown on demand up to NCCL_AMD_EAGER_BOUNCE_MAX_BYTES (4 GiB);
// beyond that, or when the bounce itself cannot be registered, the collective runs staged as before (said once).
static bool bounceFor(ncclComm* comm, const void* send, size_t sendBytes, const void* recv, size_t recvBytes,
                      const char** rmtSend, char** rmtRecv) {
  static const uint64_t maxBytes = (uint64_t)paramInt("NCCL_AMD_EAGER_BOUNCE_MAX_BYTES", (int64_t)4 << 30);
  const uint64_t sendLen = send ? (sendBytes + 4095) / 4096 * 4096 : 0;
  const uint64_t need = sendLen + recvBytes;
  if (comm->bounceFailed) return false;
  if (need > maxBytes) {
    if (!comm->warnedBounceMax) {
      comm->warnedBounceMax = true;
      WARN("rank %d: a collective of %zu + %zu bytes needs more than NCCL_AMD_EAGER_BOUNCE_MAX_BYTES=%lu of bounce "
           "allocation: it runs staged on this rank (a kernel-mismatch error if its peers run zero-copy)", comm->rank,
           sendBytes, recvBytes, (unsigned long)maxBytes);
    }
    return false;
  }
  if (!comm->bounceEv && hipEventCreateWithFlags(&comm->bounceEv, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    comm->bounceEv = nullptr;
    comm->bounceFailed = true;
    WARN("rank %d: no event for the bounce allocation: eager collectives this rank cannot register run staged",
         comm->rank);
    return false;
  }
  if (!comm->bounce || comm->bounce->size < need) {
    const uint64_t mib64 = (uint64_t)64 << 20;  // 64 MiB steps, at least doubling: few re-registrations
    const uint64_t sz = std::min(std::max((need + mib64 - 1) / mib64 * mib64, comm->bounce ? 2 * comm->bounce->size : 0),
                                 maxBytes);
    if (comm->bounce) comm->bounceOld.push_back({comm->bounce, comm->bounceMem});  // planned ops may still use it
    comm->bounce = nullptr;
    comm->bounceMem = nullptr;
    void* mem = nullptr;
    RegAlloc* ra = nullptr;
    hipError_t e;
    {
      std::lock_guard<std::mutex> g(ipcMapMutex());  // the library's allocations, imports and releases: one at a time
      e = hipMalloc(&mem, sz);
    }
    if (e != hipSuccess) {
      (void)hipGetLastError();
      comm->bounceFailed = true;
      WARN("rank %d: bounce allocation of %lu MiB failed: eager collectives this rank cannot register run staged",
           comm->rank, (unsigned long)(sz >> 20));
      return false;
    }
    tBounceCreate = true;
    const ncclResult_t res = regCreate(comm, (uint64_t)mem, sz, bufferIdOf(mem), &ra, /*deferRelease=*/true);
    tBounceCreate = false;
    if (res != ncclSuccess || !ra->usable) {
      if (res == ncclSuccess) regFree(ra);
      std::lock_guard<std::mutex> g(ipcMapMutex());
      (void)hipFree(mem);  // a peer that mapped it before the failure keeps the memory until its RELEASE
      comm->bounceFailed = true;
      WARN("rank %d: the bounce allocation (%lu MiB) could not be registered (%d): eager collectives this rank cannot "
           "register run staged", comm->rank, (unsigned long)(sz >> 20), (int)res);
      return false;
    }
    comm->bounce = ra;
    comm->bounceMem = mem;
    INFO("rank %d: bounce allocation of %lu MiB registered with every peer (eager collectives on buffers this rank "
         "cannot register)", comm->rank, (unsigned long)(sz >> 20));
  }
  RegAlloc* b = comm->bounce;
  b->bouncePlans++;
  BounceCopy& bc = comm->bounceNext;
  bc.ra = b;
  bc.userSend = send;
  bc.userRecv = const_cast<void*>(recv);
  bc.send = send ? (char*)b->base : nullptr;
  bc.recv = (char*)(b->base + sendLen);
  bc.sendBytes = send ? sendBytes : 0;
  bc.recvBytes = recvBytes;
  comm->bounceUsed = true;
  for (int r = 0; r < comm->nRanks; r++) {
    rmtSend[r] = send ? (const char*)b->rmt[r] : nullptr;
    rmtRecv[r] = (char*)(b->rmt[r] + sendLen);
  }
  TRACE("rank %d: bounced zero-copy: send %p recv %p through %lx (+%lu)", comm->rank, send, recv,
        (unsigned long)b->base, (unsigned long)sendLen);
  return true;
}

ncclResult_t bounceLaunch(ncclComm* comm, const SymPlan& sp) {
  const BounceCopy& b = sp.bounce;
  b.ra->bouncePlans--;
  HIPCHECK(hipStreamWaitEvent(sp.stream, comm->bounceEv, 0));  // a use on another stream is done with it
  if (b.userSend) HIPCHECK(hipMemcpyAsync(b.send, b.userSend, b.sendBytes, hipMemcpyDefault, sp.stream));
  NCCLCHECK(launchSymPlan(sp));
  HIPCHECK(hipMemcpyAsync(b.userRecv, b.recv, b.recvBytes, hipMemcpyDefault, sp.stream));
  HIPCHECK(hipEventRecord(comm->bounceEv, sp.stream));
  return ncclSuccess;
}

// Grown-out bounce allocations (their last use done: a blocking point) and, at teardown, the current one.
static void bounceFree(ncclComm* comm, bool all, bool notifyPeers) {
  if (comm->bounceOld.empty() && !(all && comm->bounce)) return;
  if (comm->bounceEv && notifyPeers) (void)hipEventSynchronize(comm->bounceEv);  // (abort: nothing waits)
  if (all && comm->bounce) comm->bounceOld.push_back({comm->bounce, comm->bounceMem});
  if (all) comm->bounce = nullptr, comm->bounceMem = nullptr;
  for (auto& x : comm->bounceOld) {
    if (notifyPeers) regRelease(comm, x.first);
    else regFree(x.first);
    std::lock_guard<std::mutex> g(ipcMapMutex());
    (void)hipFree(x.second);
  }
  comm->bounceOld.clear();
  if (all && comm->bounceEv) (void)hipEventDestroy(comm->bounceEv), comm->bounceEv = nullptr;
}

bool regLookup(ncclComm* comm, hipStream_t stream, const void* send, size_t sendBytes, const void* recv,
               size_t recvBytes, const char** rmtSend, char** rmtRecv, bool eager) {
  comm->regLastUse[0] = comm->regLastUse[1] = nullptr;
  comm->bounceUsed = false;
  if (comm->nRanks == 1) return false;
  bool capturing = false;
  if (comm->tune.graphRegister || eager) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    capturing = hipStreamIsCapturing(stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
    (void)hipGetLastError();
    if (capturing && !comm->tune.graphRegister) return false;  // NCCL_GRAPH_REGISTER=0: captures stay staged
  }
  // graph references whose graphs are gone are dropped BEFORE the lookup: dropping one may free a registration the
  // lookup would otherwise hand back (deferred: no RELEASE round trips inside the collective)
  if (capturing) regDrainGraphReleases(comm, true);
  if (comm->regs.empty() && !capturing && !eager) return false;
  RegAlloc* rs = send ? regFind(comm, send, sendBytes, capturing || eager) : nullptr;
  RegAlloc* rr = regFind(comm, recv, recvBytes, capturing || eager);
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
    } else if (send && (rsRes = regAcquire(comm, send, sendBytes, REF_GRAPH, &x)) == ncclSuccess) {
      graphHold(comm, x, stream, true);
      rs = x->usable ? x : nullptr;
    }
    if (rr) {
      graphHold(comm, rr, stream, false);
    } else if ((rrRes = regAcquire(comm, recv, recvBytes, REF_GRAPH, &x)) == ncclSuccess) {
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
  } else if (eager && tPlanOnly) {
    // ncclGroupSimulateEnd: no registration (no exports, no peer round trips); the real group end would register
    // what is missing and run zero-copy, so the plan says so (the pointers are never used: nothing launches)
    if (!rr || (send && !rs)) {
      if (!comm->regIpcAll) return false;  // registrations would stay local (regCreate): the staged plan
      // an allocation whose eager registration already failed runs staged at the real group end too
      // (unless the bounce allocation takes it, as it does at the real group end: bounceFor)
      if (comm->bounceFailed &&
          ((send && !rs && eagerFailedBefore(comm, send)) || (!rr && eagerFailedBefore(comm, recv))))
        return false;
      for (int r = 0; r < comm->nRanks; r++) rmtSend[r] = nullptr, rmtRecv[r] = nullptr;
      return true;
    }
  } else if (eager) {
    // first use of an unregistered allocation: map it into every peer now (one dma-buf export + one IMPORT request per
    // peer process, once per allocation); later collectives find it in comm->regs. A failure is remembered per
    // allocation (not retried) and the collective runs on the bounce allocation (bounceFor), so the peers, which run
    // zero-copy either way, see no difference.
    auto acquire = [&](const void* b, size_t bytes) -> RegAlloc* {
      if (eagerFailedBefore(comm, b)) return nullptr;
      RegAlloc* y = nullptr;
      // a registration failing half way is retired, its peers' RELEASE sent by regProgress, not from here
      ncclResult_t res = regAcquire(comm, b, bytes, REF_EAGER, &y, /*deferRelease=*/true);
      if (res != ncclSuccess) {
        // not a plain device allocation (host-pinned, managed: hipMemGetAddressRange fails) or the export / an import
        // failed: remembered, said once. Every rank must pass buffers of the same kind.
        const std::pair<uint64_t, uint64_t> key = eagerKey(b);
        // bounded: a loop of fresh allocations the runtime keeps refusing must not grow it for ever (the oldest
        // keys name allocations long gone; forgetting one costs at most a repeated export attempt)
        if (comm->eagerFailed.size() >= 256) comm->eagerFailed.erase(comm->eagerFailed.begin());
        comm->eagerFailed.push_back(key);
        // a WARN the first time on this communicator, INFO after (a churning allocator may see one per iteration)
        if (!comm->warnedEagerRefusal) {
          comm->warnedEagerRefusal = true;
          WARN("rank %d: eager registration of the allocation holding %p failed (%d): its collectives run through "
               "this rank's bounce allocation (copied in and out); later refusals are reported at INFO level",
               comm->rank, b, (int)res);
        } else {
          INFO("rank %d: eager registration of the allocation holding %p failed (%d): bounce allocation", comm->rank,
               b, (int)res);
        }
        return nullptr;
      }
      if ((int)comm->regs.size() > comm->tune.eagerMax && !comm->warnedEagerCap) {
        comm->warnedEagerCap = true;
        INFO("rank %d: %zu registrations exceed NCCL_AMD_EAGER_REGISTER_MAX=%d; the least recently used are retired "
             "at the next collectives (regProgress)", comm->rank, comm->regs.size(), comm->tune.eagerMax);
      }
      return y->usable ? y : nullptr;
    };
    if (send && !rs) rs = acquire(send, sendBytes);
    else if (rs && !rs->eagerRef && rs->localRefs == 0) rs->eagerRef = true;  // a graph's registration, now cached
    if (!rr) rr = acquire(recv, recvBytes);
    else if (!rr->eagerRef && rr->localRefs == 0) rr->eagerRef = true;
    // this rank could not register them: its peers run zero-copy all the same, so this rank does too, on the bounce
    if ((!rr || (send && !rs)) && comm->regIpcAll) return bounceFor(comm, send, sendBytes, recv, recvBytes, rmtSend, rmtRecv);
  }
  if (!rr || (send && !rs)) return false;
  const uint64_t use = ++comm->regClock;
  rr->lastUse = use;
  if (rs) rs->lastUse = use;
  comm->regLastUse[0] = rs;
  comm->regLastUse[1] = rr;
  TRACE("rank %d: zero-copy on send %p (tag %lu) recv %p (tag %lu); in rank %d at %lx / %lx", comm->rank, send,
        rs ? (unsigned long)rs->tag : 0ul, recv, (unsigned long)rr->tag, (comm->rank + 1) % comm->nRanks,
        rs ? (unsigned long)(rs->rmt[(comm->rank + 1) % comm->nRanks] + ((uint64_t)send - rs->base)) : 0ul,
        (unsigned long)(rr->rmt[(comm->rank + 1) % comm->nRanks] + ((uint64_t)recv - rr->base)));
  for (int r = 0; r < comm->nRanks; r++) {
    rmtSend[r] = send ? (const char*)(rs->rmt[r] + ((uint64_t)send - rs->base)) : nullptr;
    rmtRecv[r] = (char*)(rr->rmt[r] + ((uint64_t)recv - rr->base));
  }
  return true;
}

// Eager zero-copy is the default for a communicator spanning processes (enqueue.cc eagerOn), and it maps ordinary
// device allocations — what PyTorch's allocator hands out — into the peers, which the init-time mapping check
// (mapcheck.cc) does not cover: it checks the staging slab and flag block. So at init each rank registers one plain
// hipMalloc allocation with every peer (the eager path: dma-buf export, IMPORT by each peer's fd server) and reads
// every peer's through its own mapping, comparing the bytes. The outcome is all-gathered: if any rank failed any
// part, every rank turns eager zero-copy off for this communicator (the kernel choice stays the same on every rank)
// and the ranks that saw the failure say what failed. A few milliseconds per init; NCCL_AMD_EAGER_PROBE=0 skips it.
static uint64_t probeWord(int rank, size_t i) {
  uint64_t x = 0x9e3779b97f4a7c15ull * (uint64_t)(rank + 1) + 0xd1b54a32d192ed03ull * (uint64_t)(i + 1);
  x ^= x >> 31;
  return x * 0xbf58476d1ce4e5b9ull;
}

ncclResult_t eagerProbe(ncclComm* comm) {
  if (!(comm->tune.eagerRegister < 0 && comm->multiProcess && comm->regIpcAll)) return ncclSuccess;
  if (!paramInt("NCCL_AMD_EAGER_PROBE", 1)) return ncclSuccess;
  const int n = comm->nRanks, me = comm->rank, pid = getpid();
  const size_t bytes = (size_t)2 << 20, words = bytes / sizeof(uint64_t), checkWords = 512;
  char why[160] = "";
  void* mem = nullptr;
  RegAlloc* ra = nullptr;
  hipError_t e;
  {
    std::lock_guard<std::mutex> g(ipcMapMutex());
    e = hipMalloc(&mem, bytes);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    mem = nullptr;
    snprintf(why, sizeof(why), "hipMalloc of the probe: %s", hipGetErrorString(e));
  } else {
    std::vector<uint64_t> pat(words);
    for (size_t i = 0; i < words; i++) pat[i] = probeWord(me, i);
    if ((e = hipMemcpy(mem, pat.data(), bytes, hipMemcpyHostToDevice)) != hipSuccess) {
      (void)hipGetLastError();
      snprintf(why, sizeof(why), "filling the probe: %s", hipGetErrorString(e));
    } else if (regCreate(comm, (uint64_t)mem, bytes, bufferIdOf(mem), &ra, /*deferRelease=*/false) != ncclSuccess) {
      ra = nullptr;  // released by regCreate
      snprintf(why, sizeof(why), "registering the probe with every peer (export or a peer's import)");
    }
  }
  // where each peer mapped my probe: table[q * n + r] = rank q's probe as mapped in rank r's process
  std::vector<uint64_t> table((size_t)n * n, 0);
  if (ra)
    for (int r = 0; r < n; r++) table[(size_t)me * n + r] = ra->rmt[r];
  ncclResult_t res = commAllGather(comm, table.data(), (size_t)n * sizeof(uint64_t));
  if (res == ncclSuccess && !why[0]) {
    std::vector<uint64_t> got(checkWords);
    for (int q = 0; q < n && !why[0]; q++) {
      if (q == me || comm->peers[q].pid == pid) continue;
      const uint64_t addr = table[(size_t)q * n + me];
      if (!addr) continue;  // rank q could not register its probe: it reports that itself
      for (size_t at : {(size_t)0, words - checkWords}) {  // the first and the last 4 KiB
        if ((e = hipMemcpy(got.data(), (const void*)(addr + at * sizeof(uint64_t)), checkWords * sizeof(uint64_t),
                           hipMemcpyDeviceToHost)) != hipSuccess) {
          (void)hipGetLastError();
          snprintf(why, sizeof(why), "reading rank %d's probe through its mapping: %s", q, hipGetErrorString(e));
          break;
        }
        for (size_t i = 0; i < checkWords && !why[0]; i++)
          if (got[i] != probeWord(q, at + i))
            snprintf(why, sizeof(why), "rank %d's probe reads back wrong through its mapping (word %zu)", q, at + i);
      }
    }
  }
  std::vector<int> ok(n, 0);
  ok[me] = res == ncclSuccess && !why[0] ? 1 : 0;
  if (res == ncclSuccess) res = commAllGather(comm, ok.data(), sizeof(int));
  if (ra) regRelease(comm, ra);  // RELEASE to the peers (unmapped at their next blocking call or collective)
  if (mem) {
    std::lock_guard<std::mutex> g(ipcMapMutex());
    (void)hipFree(mem);
  }
  if (res != ncclSuccess) return res;  // the bootstrap itself failed: the init fails
  int bad = -1;
  for (int r = 0; r < n && bad < 0; r++)
    if (!ok[r]) bad = r;
  if (bad >= 0) {
    comm->tune.eagerRegister = 0;  // the same decision on every rank (the all-gathered outcomes)
    if (why[0]) WARN("rank %d: eager zero-copy probe failed: %s; eager zero-copy is off for this communicator", me, why);
    else INFO("rank %d: eager zero-copy is off for this communicator (rank %d's probe failed)", me, bad);
  } else {
    TRACE("rank %d: eager zero-copy probe passed (every peer's plain allocation read back through its mapping)", me);
  }
  return ncclSuccess;
}

void windowsFree(ncclComm* comm, bool notifyPeers) {
  (void)hipSetDevice(comm->device);
  {  // graph releases still queued for this communicator: every registration goes below anyway; tokens of its graphs
     // that die later are discarded (its generation is no longer live)
    std::lock_guard<std::mutex> lk(graphRelMu());
    std::vector<GraphRelease>& rel = graphRel();
    rel.erase(std::remove_if(rel.begin(), rel.end(), [&](const GraphRelease& g) { return g.comm == comm; }), rel.end());
    std::vector<uint64_t>& live = liveGens();
    if (comm->regGen) live.erase(std::remove(live.begin(), live.end(), comm->regGen), live.end());
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
  bounceFree(comm, /*all=*/true, notifyPeers);
  for (RegAlloc* ra : comm->regRetired) comm->regs.push_back(ra);
  comm->regRetired.clear();
  for (RegAlloc* ra : comm->regs) {
    if (notifyPeers) regRelease(comm, ra);
    else regFree(ra);
  }
  comm->regs.clear();
  comm->regLastUse[0] = comm->regLastUse[1] = nullptr;
}

}  // namespace ncclamd

using namespace ncclamd;

#define NCCL_ALIAS(ret, name, ...) extern "C" __attribute__((visibility("default"), alias(#name))) ret p##name(__VA_ARGS__);

NCCL_EXPORT ncclResult_t ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle) {
  NCCLCHECK(commCheck(comm, "ncclCommRegister", "comm"));
  ipcDrainReleases();
  regBlockingPoint(comm);
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
    ncclResult_t res = regAcquire(comm, buff, size, REF_LOCAL, &h->ra);
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
  regBlockingPoint(comm);
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
    if (h->ra->localRefs == 1 && h->ra->graphRefs == 0 && !h->ra->eagerRef) HIPCHECK(hipDeviceSynchronize());
    regPut(comm, h->ra, REF_LOCAL);
  }
  delete h;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommDeregister, const ncclComm_t, void*)

NCCL_EXPORT ncclResult_t ncclCommWindowRegister(ncclComm_t comm, void* buff, size_t size, ncclWindow_t* win,
                                                int winFlags) {
  NCCLCHECK(commCheck(comm, "ncclCommWindowRegister", "comm"));
  ipcDrainReleases();
  regBlockingPoint(comm);
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
  regBlockingPoint(comm);
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

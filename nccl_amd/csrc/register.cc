// register.cc — buffer registration and symmetric windows.
//
// Reference: src/register/register.cc:154-200 (ncclCommRegister / ncclCommDeregister: local, refcounted
// registration used by the reference's SIMPLE-protocol zero-copy paths), src/dev_runtime.cc:1331-1400,
// 1592-1610 (ncclCommWindowRegister as a group task: every rank maps every peer's window;
// ncclCommWindowDeregister; ncclWinGetUserPtr), src/device/symmetric/* (the kernels that use them).
//
// ncclCommRegister: this engine's staged path only ever reads and writes user buffers locally (peers
// exchange data through the comm's own uncached staging), so there is nothing to map: the call
// validates and records the buffer and returns a handle, like the reference does when local
// registration is disabled (register.cc:156-159). Zero-copy is what windows are for:
// ncclCommWindowRegister maps every peer's buffer into this process (a dma-buf fd across processes, ipc.cc;
// the raw pointer inside one process) and collectives whose buffers lie in NCCL_WIN_COLL_SYMMETRIC windows
// run the symmetric kernels (kernels.h symKernel), which read peers' windows directly.
#include <string.h>
#include <unistd.h>

#include <algorithm>

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
      for (int q = 0; q < r; q++)
        if (w->peerBase[q]) ipcUnmap(comm, q, w->peerBase[q]);
      if (needIpc) ipcUnexport(comm, me.desc);
      delete w;
      return res;
    }
    w->peerBase[r] = p.base;
  }
  if (needIpc) {
    // every peer has mapped my allocation (its mapping keeps it referenced): stop serving the descriptor
    std::vector<char> sync(comm->nRanks);
    ncclResult_t bres = commAllGather(comm, sync.data(), 1);
    ipcUnexport(comm, me.desc);
    if (bres != ncclSuccess) {
      windowRelease(comm, w);
      return bres;
    }
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

void windowsFree(ncclComm* comm) {
  (void)hipSetDevice(comm->device);
  for (ncclWindow_vidmem* w : comm->windows) windowRelease(comm, w);
  comm->windows.clear();
  for (IpcMapping& m : comm->ipcMaps) ipcRelease(&m.map);
  comm->ipcMaps.clear();
  for (void* h : comm->regHandles) free(h);
  comm->regHandles.clear();
}

}  // namespace ncclamd

using namespace ncclamd;

#define NCCL_ALIAS(ret, name, ...) extern "C" __attribute__((visibility("default"), alias(#name))) ret p##name(__VA_ARGS__);

struct RegHandle {
  void* buff;
  size_t size;
};

NCCL_EXPORT ncclResult_t ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle) {
  NCCLCHECK(commCheck(comm, "ncclCommRegister", "comm"));
  if (handle == nullptr) {
    WARN("ncclCommRegister : handle argument is NULL");
    return ncclInvalidArgument;
  }
  *handle = nullptr;
  if (buff == nullptr || size == 0) {
    WARN("ncclCommRegister : invalid buffer %p / size %zu", buff, size);
    return ncclInvalidArgument;
  }
  RegHandle* h = (RegHandle*)malloc(sizeof(RegHandle));
  h->buff = buff;
  h->size = size;
  comm->regHandles.push_back(h);
  *handle = h;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommRegister, const ncclComm_t, void*, size_t, void**)

NCCL_EXPORT ncclResult_t ncclCommDeregister(const ncclComm_t comm, void* handle) {
  NCCLCHECK(commCheck(comm, "ncclCommDeregister", "comm"));
  if (handle == nullptr) return ncclSuccess;  // reference commDeregister: NULL reg is a no-op
  auto it = std::find(comm->regHandles.begin(), comm->regHandles.end(), handle);
  if (it == comm->regHandles.end()) {
    WARN("Deregister: Could not find handle");
    return ncclInvalidUsage;
  }
  comm->regHandles.erase(it);
  free(handle);
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommDeregister, const ncclComm_t, void*)

NCCL_EXPORT ncclResult_t ncclCommWindowRegister(ncclComm_t comm, void* buff, size_t size, ncclWindow_t* win,
                                                int winFlags) {
  NCCLCHECK(commCheck(comm, "ncclCommWindowRegister", "comm"));
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

// transport.cc — the xGMI peer-memory transport: staging + flag allocation, HIP IPC export/import.
//
// Reference: src/transport/p2p.cc:130-618 allocates, per ring edge and channel, a receiver-side FIFO
// (ncclRecvMem + buffers) and sender-side head word, shares them through CUDA IPC / cuMem handles
// (p2p.cc:220-325) or a direct pointer inside one process (p2p.cc:345-386), and connects only the
// ring neighbours. On MI355X every GPU of the node has a direct xGMI link to every other GPU, so here
// each rank allocates ONE staging slab and ONE flag block that ALL peers write into (full mesh), and
// maps every peer's slab once at init:
//   - same process (ncclCommInitAll / threads): raw pointer + hipDeviceEnablePeerAccess;
//   - other process: a dma-buf fd handed over by the exporter's fd server and mapped with
//     hipImportExternalMemory (ipc.cc; the reference's cuMem fd path, p2p.cc:220-325).
// Staging and flags are allocated UNCACHED (hipDeviceMallocUncached): they are written by remote
// GPUs over xGMI and read locally, so no L2 anywhere may hold a stale copy.
#include <string.h>
#include <unistd.h>

#include "core.h"

namespace ncclamd {

static size_t stagingBytes(const ncclComm* c) {
  return (size_t)c->maxChannels * STG_KINDS * c->nSlots * c->nRanks * c->slotBytes;
}
static size_t flagWordBytes(const ncclComm* c) {
  return (size_t)c->maxChannels * FLG_KINDS * NCCL_AMD_MAX_RANKS * sizeof(uint64_t);
}
static size_t llOffset(const ncclComm* c) { return (flagWordBytes(c) + 4095) / 4096 * 4096; }
// LL area, then the LL64 area of the same geometry (device_abi.h)
static size_t ll64Offset(const ncclComm* c) { return llOffset(c) + (size_t)c->llChannels * 2 * c->nRanks * c->llBytes; }
// then the mapping-check area (mapcheck.cc): 2 rows x NCCL_AMD_MAX_RANKS x 16 bytes, used once at init
static size_t probeOffset(const ncclComm* c) {
  return (ll64Offset(c) + (size_t)c->llChannels * 2 * c->nRanks * c->llBytes + 255) / 256 * 256;
}
static size_t flagsBytes(const ncclComm* c) { return probeOffset(c) + kMapProbeBytes; }

// Device memory this communicator holds on its GPU (ncclCommMemStats): staging slab, flag/LL lines,
// step counters and the device copy of DevComm. All of it lives as long as the communicator.
// The sizes are the ones recorded when the memory was allocated (llChannels is lowered to the
// co-residency cap AFTER the flag / LL block was allocated at the full count, so recomputing from the comm's
// current shape under-reported it).
size_t commDeviceBytes(const ncclComm* c) {
  size_t b = 0;
  if (c->staging) b += c->stagingAllocBytes;
  if (c->flags) b += c->flagsAllocBytes;
  if (c->counters) b += c->countersAllocBytes;
  if (c->devComm) b += sizeof(DevComm);
  return b;
}

ncclResult_t transportSetup(ncclComm* comm) {
  HIPCHECK(hipSetDevice(comm->device));
  if (comm->nRanks == 1) return ncclSuccess;  // nranks==1 never touches peers (onerank.cu:49-110)
  size_t sb = stagingBytes(comm), fb = flagsBytes(comm);
  {
    // only the allocations themselves are serialized with imports / releases (gMapMu): the fd server thread
    // needs the same lock to map a peer's registration, so it is never held across the device-wide sync below
    // (a peer registering a buffer could otherwise wait behind a sync that waits on that peer)
    std::lock_guard<std::mutex> mapLock(ipcMapMutex());
    if (paramInt("NCCL_AMD_STAGING_PLAIN", 0))  // diagnostics only (scripts/ipc_hang_diag.py): cached staging
      HIPCHECK(hipMalloc(&comm->staging, sb));
    else
      HIPCHECK(hipExtMallocWithFlags(&comm->staging, sb, hipDeviceMallocUncached));
    comm->stagingAllocBytes = sb;
    HIPCHECK(hipExtMallocWithFlags((void**)&comm->flags, fb, hipDeviceMallocUncached));
    comm->flagsAllocBytes = fb;
    comm->probeOffset = probeOffset(comm);  // (llChannels may be lowered later; the layout stays as allocated)
  }
  HIPCHECK(hipMemset(comm->flags, 0, fb));
  HIPCHECK(hipDeviceSynchronize());
  INFO("rank %d dev %d: staging %zu MiB (%d ch x %d slots x %zu KiB), flags %zu KiB", comm->rank, comm->device,
       sb >> 20, comm->maxChannels, comm->nSlots, comm->slotBytes >> 10, fb >> 10);
  return ncclSuccess;
}

ncclResult_t transportConnect(ncclComm* comm) {
  if (comm->nRanks == 1) return ncclSuccess;
  HIPCHECK(hipSetDevice(comm->device));
  // diagnostics (scripts/ipc_hang_diag.py): NCCL_AMD_IMPORT_SERIAL=1 lets one rank at a time import
  const bool serial = comm->bootstrap && paramInt("NCCL_AMD_IMPORT_SERIAL", 0);
  for (int turn = 0; serial && turn < comm->rank; turn++) NCCLCHECK(bootstrapBarrier(comm->bootstrap));
  const PeerInfo& me = comm->peers[comm->rank];
  for (int r = 0; r < comm->nRanks; r++) {
    const PeerInfo& p = comm->peers[r];
    if (r == comm->rank) {
      comm->peerStaging[r] = comm->staging;
      comm->peerFlags[r] = comm->flags;
      continue;
    }
    if (p.hostHash != me.hostHash) {
      WARN("rank %d is on another host: this engine is intra-node only", r);
      return ncclInvalidUsage;
    }
    if (p.pid == me.pid) {
      // Same process: direct pointers (reference p2p.cc:345-386 "P2P/direct pointer").
      if (p.device != comm->device) {
        int can = 0;
        HIPCHECK(hipDeviceCanAccessPeer(&can, comm->device, p.device));
        if (!can) {
          WARN("device %d cannot access peer device %d", comm->device, p.device);
          return ncclSystemError;
        }
        hipError_t e = hipDeviceEnablePeerAccess(p.device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          WARN("hipDeviceEnablePeerAccess(%d->%d): %s", comm->device, p.device, hipGetErrorString(e));
          return ncclUnhandledCudaError;
        }
        (void)hipGetLastError();
      }
      comm->peerStaging[r] = (void*)p.stagingPtr;
      comm->peerFlags[r] = (uint64_t*)p.flagsPtr;
    } else {
      TRACE("rank %d: importing rank %d's staging (%zu MiB)", comm->rank, r, (size_t)(p.stagingDesc.size >> 20));
      NCCLCHECK(ipcImport(p.stagingDesc, &comm->peerStagingMap[r]));
      TRACE("rank %d: importing rank %d's flags", comm->rank, r);
      NCCLCHECK(ipcImport(p.flagsDesc, &comm->peerFlagsMap[r]));
      TRACE("rank %d: rank %d mapped", comm->rank, r);
      comm->peerStaging[r] = comm->peerStagingMap[r].ptr;
      comm->peerFlags[r] = (uint64_t*)comm->peerFlagsMap[r].ptr;
    }
  }
  for (int turn = comm->rank; serial && turn < comm->nRanks; turn++) NCCLCHECK(bootstrapBarrier(comm->bootstrap));
  return ncclSuccess;
}

// The mapping check's second chance (mapcheck.cc): map peer r's slab and flags through the hipIpc handles of their
// exports instead of the dma-buf imports, and give the device the new pointers.
ncclResult_t transportRemapPeer(ncclComm* comm, int r) {
  const PeerInfo& p = comm->peers[r];
  if (p.pid == comm->peers[comm->rank].pid) {
    WARN("rank %d: no other way to map rank %d (same process: a peer pointer)", comm->rank, r);
    return ncclSuccess;  // the second round reports it
  }
  HIPCHECK(hipSetDevice(comm->device));
  IpcImport st, fl;
  if (ipcImportHandle(p.stagingDesc, &st) != ncclSuccess || ipcImportHandle(p.flagsDesc, &fl) != ncclSuccess) {
    ipcRelease(&st);
    WARN("rank %d: rank %d's slab cannot be mapped through a hipIpc handle; keeping the dma-buf mapping", comm->rank, r);
    return ncclSuccess;  // the second round reports it
  }
  ipcRelease(&comm->peerStagingMap[r]);
  ipcRelease(&comm->peerFlagsMap[r]);
  comm->peerStagingMap[r] = st;
  comm->peerFlagsMap[r] = fl;
  comm->peerStaging[r] = st.ptr;
  comm->peerFlags[r] = (uint64_t*)fl.ptr;
  comm->hostDevComm.staging[r] = (char*)st.ptr;
  comm->hostDevComm.flags[r] = (uint64_t*)fl.ptr;
  HIPCHECK(hipMemcpy(comm->devComm, &comm->hostDevComm, sizeof(DevComm), hipMemcpyHostToDevice));
  WARN("rank %d: rank %d (device %d, %s) remapped through hipIpc handles after the dma-buf mapping failed the check",
       comm->rank, r, p.device, p.busId);
  return ncclSuccess;
}

// Before freeing: every slice this rank sent must have been acknowledged (RS_ACK == sendRS and
// AG_ACK == sendAG per channel and peer). Acks are written by peers' kernels after they consumed our
// data, possibly after our own kernels finished; waiting for them (bounded) keeps those stores out of
// freed memory. Returns ncclSuccess or ncclTimeout; the caller frees either way.
ncclResult_t transportDrainCredits(ncclComm* comm) {
  if (comm->nRanks == 1 || !comm->counters || !comm->flags) return ncclSuccess;
  const size_t nc = (size_t)comm->maxChannels * CTR_KINDS * NCCL_AMD_MAX_RANKS;
  const size_t nf = flagWordBytes(comm) / sizeof(uint64_t);
  std::vector<uint64_t> ctr(nc), flg(nf);
  HIPCHECK(hipMemcpy(ctr.data(), comm->counters, nc * sizeof(uint64_t), hipMemcpyDeviceToHost));
  const int64_t limitMs = paramInt("NCCL_AMD_DESTROY_TIMEOUT_MS", 10000);
  for (int64_t waited = 0;; waited++) {
    HIPCHECK(hipMemcpy(flg.data(), comm->flags, nf * sizeof(uint64_t), hipMemcpyDeviceToHost));
    bool done = true;
    for (int c = 0; c < comm->maxChannels && done; c++)
      for (int p = 0; p < comm->nRanks && done; p++) {
        if (p == comm->rank) continue;
        done = flg[flagIndex(c, FLG_RS_ACK, p)] >= ctr[ctrIndex(c, CTR_SEND_RS, p)] &&
               flg[flagIndex(c, FLG_AG_ACK, p)] >= ctr[ctrIndex(c, CTR_SEND_AG, p)] &&
               flg[flagIndex(c, FLG_PULL_ACK, p)] >= ctr[ctrIndex(c, CTR_PULL_PUB, 0)];
      }
    if (done) return ncclSuccess;
    if (waited >= limitMs) {
      WARN("rank %d: peers still owe credits after %ld ms; freeing anyway", comm->rank, (long)limitMs);
      return ncclTimeout;
    }
    usleep(1000);
  }
}

ncclResult_t transportFree(ncclComm* comm) {
  (void)hipSetDevice(comm->device);
  for (int r = 0; r < comm->nRanks && r < NCCL_AMD_MAX_RANKS; r++) {
    ipcRelease(&comm->peerStagingMap[r]);
    ipcRelease(&comm->peerFlagsMap[r]);
    comm->peerStaging[r] = nullptr;
    comm->peerFlags[r] = nullptr;
  }
  ipcServerStop(comm);
  if (comm->staging) (void)hipFree(comm->staging);
  if (comm->flags) (void)hipFree(comm->flags);
  if (comm->counters) (void)hipFree(comm->counters);
  if (comm->devComm) (void)hipFree(comm->devComm);
  if (comm->hostAbort) (void)hipHostFree(comm->hostAbort);
  if (comm->hostError) (void)hipHostFree(comm->hostError);
  comm->staging = nullptr;
  comm->flags = nullptr;
  comm->counters = nullptr;
  comm->devComm = nullptr;
  comm->hostAbort = nullptr;
  comm->hostError = nullptr;
  return ncclSuccess;
}

ncclResult_t commAllocDevState(ncclComm* comm) {
  HIPCHECK(hipSetDevice(comm->device));
  size_t cb = (size_t)comm->maxChannels * CTR_KINDS * NCCL_AMD_MAX_RANKS * sizeof(uint64_t);
  HIPCHECK(hipMalloc((void**)&comm->counters, cb));
  comm->countersAllocBytes = cb;
  HIPCHECK(hipMemset(comm->counters, 0, cb));
  // Test knob (reference TEST_LL_CLEANUP, include/device.h:99-106, shrinks the LL flag space to exercise
  // wraparound): start every channel's LL epoch at NCCL_AMD_LL_EPOCH_BASE, e.g. just below 2^32.
  if (int64_t base = paramInt("NCCL_AMD_LL_EPOCH_BASE", 0)) {
    std::vector<uint64_t> init(cb / sizeof(uint64_t), 0);
    for (int c = 0; c < comm->maxChannels; c++) init[ctrIndex(c, CTR_LL, 0)] = (uint64_t)base;
    HIPCHECK(hipMemcpy(comm->counters, init.data(), cb, hipMemcpyHostToDevice));
  }
  HIPCHECK(hipHostMalloc((void**)&comm->hostAbort, 64, hipHostMallocMapped | hipHostMallocCoherent));
  HIPCHECK(hipHostMalloc((void**)&comm->hostError, 64, hipHostMallocMapped | hipHostMallocCoherent));
  memset(comm->hostAbort, 0, 64);
  memset(comm->hostError, 0, 64);
  DevComm& d = comm->hostDevComm;
  memset(&d, 0, sizeof(d));
  d.rank = comm->rank;
  d.nRanks = comm->nRanks;
  d.nSlots = comm->nSlots;
  d.maxChannels = comm->maxChannels;
  d.slotBytes = comm->slotBytes;
  // s_memrealtime runs at 100 MHz on gfx9 parts.
  d.timeoutTicks = (uint64_t)paramInt("NCCL_AMD_SPIN_TIMEOUT_MS", 120000) * 100000ull;
  for (int r = 0; r < comm->nRanks; r++) {
    d.staging[r] = (char*)comm->peerStaging[r];
    d.flags[r] = comm->peerFlags[r];
  }
  d.counters = comm->counters;
  // the LL channels of a launch must be co-resident like any channel: never more than chanCap (the line
  // area was sized for the full count; host planning and the kernel's batch modulus use this value)
  d.llOffset = llOffset(comm);
  d.ll64Offset = ll64Offset(comm);  // both before the cap below: the areas were sized for the full count
  if (comm->llChannels > comm->chanCap && comm->chanCap > 0) comm->llChannels = comm->chanCap;
  d.llBytes = comm->llBytes;
  d.llChannels = comm->llChannels;
  void* dAbort = nullptr;
  void* dErr = nullptr;
  HIPCHECK(hipHostGetDevicePointer(&dAbort, comm->hostAbort, 0));
  HIPCHECK(hipHostGetDevicePointer(&dErr, comm->hostError, 0));
  d.abortFlag = (uint32_t*)dAbort;
  d.errorWord = (uint32_t*)dErr;
  HIPCHECK(hipMalloc((void**)&comm->devComm, sizeof(DevComm)));
  HIPCHECK(hipMemcpy(comm->devComm, &d, sizeof(DevComm), hipMemcpyHostToDevice));
  const PeerInfo& me = comm->peers[comm->rank];
  for (int r = 0; r < comm->nRanks; r++)
    if (r != comm->rank && comm->peers[r].pid == me.pid && strcmp(comm->peers[r].busId, me.busId) == 0)
      comm->sharedDevInProcess = true;
  // NCCL_AMD_FORK_JOIN=0: the caller guarantees every rank's stream has a hardware queue of its own
  // (e.g. hipExtStreamCreateWithCUMask streams), so launch directly on it and skip the cross-queue
  // event fork/join (tens of microseconds per collective)
  if (!paramInt("NCCL_AMD_FORK_JOIN", 1)) comm->sharedDevInProcess = false;
  if (comm->sharedDevInProcess) {
    std::vector<uint32_t> mask((me.numCUs + 31) / 32, 0u);
    for (int cu = 0; cu < me.numCUs; cu++) mask[cu / 32] |= 1u << (cu % 32);
    HIPCHECK(hipExtStreamCreateWithCUMask(&comm->internalStream, (uint32_t)mask.size(), mask.data()));
    HIPCHECK(hipEventCreateWithFlags(&comm->evIn, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&comm->evOut, hipEventDisableTiming));
  }
  NCCLCHECK(warmKernels());
  return ncclSuccess;
}

// Export the slab and the flag block to other processes (only communicators built by ncclCommInitRank
// can have peers in other processes; ncclCommInitAll clique members share this process).
ncclResult_t exportHandles(ncclComm* comm, PeerInfo* info) {
  memset(&info->stagingDesc, 0, sizeof(info->stagingDesc));
  memset(&info->flagsDesc, 0, sizeof(info->flagsDesc));
  info->stagingPtr = (uint64_t)comm->staging;
  info->flagsPtr = (uint64_t)comm->flags;
  if (comm->nRanks == 1 || !comm->bootstrap) return ncclSuccess;
  NCCLCHECK(ipcServerStart(comm));
  snprintf(info->fdServer, sizeof(info->fdServer), "%s", ipcServerName(comm));
  NCCLCHECK(ipcExport(comm, comm->staging, stagingBytes(comm), &info->stagingDesc));
  NCCLCHECK(ipcExport(comm, comm->flags, flagsBytes(comm), &info->flagsDesc));
  return ncclSuccess;
}

// Every peer has mapped our slab and flags (called after the init barrier): stop serving them.
void unexportHandles(ncclComm* comm) {
  if (comm->peers.empty()) return;
  ipcUnexport(comm, comm->peers[comm->rank].stagingDesc);
  ipcUnexport(comm, comm->peers[comm->rank].flagsDesc);
}

}  // namespace ncclamd

// init.cc — communicator lifecycle: unique id, InitRank(Config), InitAll, Finalize/Destroy/Abort,
// error strings, async error, queries, custom PreMulSum operators, ncclMemAlloc/Free.
//
// Reference: src/init.cc (ncclGetUniqueId :183, ncclCommInitRankFunc :1831-1968,
// initTransportsRank :965-1720, ncclCommInitRank :2562, ncclCommInitAll :2581-2643,
// ncclCommDestroy :2879, ncclCommAbort :3025, ncclGetErrorString :3415, ncclCommGetAsyncError :3449),
// src/enqueue.cc:2479-2583 (user PreMulSum ops), src/allocator.cc (ncclMemAlloc).
// What is NOT rebuilt (out of scope): topology/graph search (single-node full mesh is
// fixed), proxy thread, net/SHM/NVLS transports, split/shrink/grow, windows, suspend/resume.
#include <string.h>
#include <unistd.h>

#include <fstream>
#include <functional>
#include <thread>

#include "core.h"

namespace ncclamd {
ncclResult_t exportHandles(ncclComm* comm, PeerInfo* info);
void unexportHandles(ncclComm* comm);

ncclResult_t commCheck(const ncclComm* comm, const char* opname, const char* what) {
  if (comm == nullptr) {
    WARN("%s : %s argument is NULL", opname, what);
    return ncclInvalidArgument;
  }
  if (comm->startMagic != kCommMagic || comm->endMagic != kCommMagic) {
    WARN("Error: corrupted comm object detected");
    return ncclInvalidArgument;
  }
  return ncclSuccess;
}

static uint64_t hostHash() {
  char host[256] = "";
  gethostname(host, sizeof(host) - 1);
  std::string s(host);
  std::ifstream f("/proc/sys/kernel/random/boot_id");
  std::string boot;
  if (f) std::getline(f, boot);
  s += boot;
  uint64_t h = 1469598103934665603ull;  // FNV-1a
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

// Sanity cap on one rank's staging slab (NCCL_AMD_STAGING_CAP_MIB, default 8 GiB of the 288 GB): slot-size
// overrides beyond it are scaled down with a warning. (Round 1 capped the slab at 1 GiB because importing a
// 2 GiB slab hung; the cause was hipIpcOpenMemHandle in torch's bundled HIP runtime, which the dma-buf
// transport of ipc.cc no longer uses — DESIGN.md §3.) Every rank adopts rank 0's (already capped) shape.
static void clampStaging(ncclComm* c, int nranks) {
  const int64_t cap = paramInt("NCCL_AMD_STAGING_CAP_MIB", 8192) << 20;
  const int64_t per = (int64_t)c->maxChannels * 2 * c->nSlots * (nranks > 1 ? nranks : 2);
  if ((int64_t)c->slotBytes * per <= cap) return;
  int64_t sb = cap / per / 4096 * 4096;
  if (sb < 4096) sb = 4096;
  WARN("staging slab %lld MiB exceeds the %lld MiB cap: slot size %zu -> %lld bytes",
       (long long)(((int64_t)c->slotBytes * per) >> 20), (long long)(cap >> 20), c->slotBytes, (long long)sb);
  c->slotBytes = (size_t)sb;
}

static void commDefaults(ncclComm* c, int rank, int nranks, int dev, const ncclConfig_t* cfg) {
  c->startMagic = c->endMagic = kCommMagic;
  c->rank = rank;
  c->nRanks = nranks;
  c->device = dev;
  c->blocking = true;
  // reference env names (env.rst :884/:901): NCCL_MIN/MAX_CTAS, or the older NCCL_MIN/MAX_NCHANNELS
  c->minCTAs = (int)paramInt("NCCL_MIN_CTAS", paramInt("NCCL_MIN_NCHANNELS", 1));
  c->maxCTAs = (int)paramInt("NCCL_MAX_CTAS", paramInt("NCCL_MAX_NCHANNELS", 256));
  bool userMax = paramStr("NCCL_MAX_CTAS") != nullptr || paramStr("NCCL_MAX_NCHANNELS") != nullptr;
  if (cfg) {
    if (cfg->blocking != NCCL_CONFIG_UNDEF_INT) c->blocking = cfg->blocking != 0;
    if (cfg->minCTAs != NCCL_CONFIG_UNDEF_INT) c->minCTAs = cfg->minCTAs;
    if (cfg->maxCTAs != NCCL_CONFIG_UNDEF_INT) {
      c->maxCTAs = cfg->maxCTAs;
      userMax = true;
    }
    if (cfg->commName) c->commName = cfg->commName;
  }
  if (c->maxCTAs < 1) c->maxCTAs = 1;
  if (c->maxCTAs > NCCL_AMD_MAX_CHANNELS) c->maxCTAs = NCCL_AMD_MAX_CHANNELS;
  if (c->minCTAs < 1) c->minCTAs = 1;
  if (c->minCTAs > c->maxCTAs) c->minCTAs = c->maxCTAs;
  c->maxChannels = c->maxCTAs;
  loadTuning(&c->tune);
  resolveLinkChannels(&c->tune, nranks, userMax);
  c->nSlots = (int)paramInt("NCCL_AMD_NSLOTS", 2);
  if (c->nSlots < 1) c->nSlots = 1;
  // Slot size: the staging slab (maxChannels x 2 kinds x nSlots x nRanks x slot) is sized to a fixed
  // HBM budget (NCCL_AMD_STAGING_MIB, default 1 GiB of the 288 GB), so fewer ranks get bigger slots
  // (fewer handshakes per byte). NCCL_AMD_SLOT_BYTES overrides; so does the reference's NCCL_BUFFSIZE (bytes
  // of one channel's buffer towards one peer, env.rst :857), which here is split into the nSlots slots.
  int64_t budget = paramInt("NCCL_AMD_STAGING_MIB", 1024) << 20;
  int64_t sb = budget / ((int64_t)c->maxChannels * 2 * c->nSlots * (nranks > 1 ? nranks : 2));
  if (sb > (1 << 20)) sb = 1 << 20;
  if (sb < (16 << 10)) sb = 16 << 10;
  if (int64_t buff = paramInt("NCCL_BUFFSIZE", 0)) sb = buff / c->nSlots;
  sb = paramInt("NCCL_AMD_SLOT_BYTES", sb);
  sb = (sb + 4095) / 4096 * 4096;
  if (sb < 4096) sb = 4096;
  c->slotBytes = (size_t)sb;
  clampStaging(c, nranks);
}

static ncclResult_t checkConfig(const ncclConfig_t* cfg) {
  if (!cfg) return ncclSuccess;
  if (cfg->magic != NCCL_API_MAGIC || cfg->size < offsetof(ncclConfig_t, cgaClusterSize)) {
    WARN("ncclConfig_t was not initialized with NCCL_CONFIG_INITIALIZER");
    return ncclInvalidArgument;
  }
  if (cfg->blocking != NCCL_CONFIG_UNDEF_INT && cfg->blocking != 0 && cfg->blocking != 1) {
    WARN("Invalid config blocking attribute value %d", cfg->blocking);
    return ncclInvalidArgument;
  }
  if (cfg->minCTAs != NCCL_CONFIG_UNDEF_INT && cfg->minCTAs <= 0) {
    WARN("Invalid config minCTAs %d", cfg->minCTAs);
    return ncclInvalidArgument;
  }
  if (cfg->maxCTAs != NCCL_CONFIG_UNDEF_INT && cfg->maxCTAs <= 0) {
    WARN("Invalid config maxCTAs %d", cfg->maxCTAs);
    return ncclInvalidArgument;
  }
  return ncclSuccess;
}

static ncclResult_t fillPeerInfo(ncclComm* comm, PeerInfo* p) {
  memset(p, 0, sizeof(*p));
  p->rank = comm->rank;
  p->device = comm->device;
  p->pid = getpid();
  p->hostHash = hostHash();
  HIPCHECK(hipDeviceGetPCIBusId(p->busId, sizeof(p->busId), comm->device));
  HIPCHECK(hipDeviceGetAttribute(&p->numCUs, hipDeviceAttributeMultiprocessorCount, comm->device));
  NCCLCHECK(exportHandles(comm, p));
  return ncclSuccess;
}

// Channels of one launch must all be resident at once on every GPU (a channel spins on the same
// channel of its peers). With several ranks on one GPU (NCCL_MULTI_RANK_GPU_ENABLE / test boxes) the
// launches share the CUs, with half the slots kept free as a margin (enqueue.cc coResidentChannelCap).
// Every rank computes this from the same peer table, so all agree.
static void computeChannelCap(ncclComm* c) {
  int minCU = 1 << 30, maxPer = 1;
  for (size_t i = 0; i < c->peers.size(); i++) {
    int same = 0;
    for (size_t j = 0; j < c->peers.size(); j++) same += strcmp(c->peers[i].busId, c->peers[j].busId) == 0;
    if (same > maxPer) maxPer = same;
    if (c->peers[i].numCUs > 0 && c->peers[i].numCUs < minCU) minCU = c->peers[i].numCUs;
  }
  if (minCU == (1 << 30)) minCU = 256;
  int cap = coResidentChannelCap(minCU, maxPer);
  // diagnostics (set alike on every rank): the shared-GPU cap itself, up to every slot (2 x CUs / ranks per GPU) —
  // the round-5 setting is NCCL_AMD_SHARED_GPU_CHANNELS=64 at 8 ranks per GPU
  const int64_t forced = maxPer > 1 ? paramInt("NCCL_AMD_SHARED_GPU_CHANNELS", 0) : 0;
  if (forced > 0) cap = (int)std::min<int64_t>(forced, 2 * minCU / maxPer);
  c->chanCap = cap < c->maxChannels ? cap : c->maxChannels;
  bool oneDevice = true;
  for (size_t i = 1; i < c->peers.size(); i++) oneDevice = oneDevice && !strcmp(c->peers[i].busId, c->peers[0].busId);
  resolveFence(&c->tune, oneDevice);
  // registered buffers map into every other-process peer through that peer's fd server: usable by every rank
  // only if every such peer runs one — one comm-wide answer from the shared table (register.cc regCreate)
  c->regIpcAll = true;
  for (size_t i = 0; i < c->peers.size(); i++)
    for (size_t j = 0; j < c->peers.size(); j++)
      if (c->peers[i].pid != c->peers[j].pid && c->peers[j].fdServer[0] == 0) c->regIpcAll = false;
  c->multiProcess = false;
  for (size_t i = 1; i < c->peers.size(); i++) c->multiProcess = c->multiProcess || c->peers[i].pid != c->peers[0].pid;
}

// Which HIP runtime this process bound (reference: init-time INFO lines, src/init.cc:1831-1968): in a torch
// process it is torch's bundled libamdhip64, not the one the library was built against (ipc.cc).
static void logRuntimeOnce() {
  static std::once_flag once;
  std::call_once(once, [] {
    const HipRuntimeInfo& rt = hipRuntimeInfo();
    INFO("HIP runtime %d.%d.%d (driver %d) from %s; built against HIP %d.%d", rt.version / 10000000,
         rt.version / 100000 % 100, rt.version % 100000, rt.driver, rt.path, HIP_VERSION_MAJOR, HIP_VERSION_MINOR);
    if (rt.version / 100000 != HIP_VERSION_MAJOR * 100 + HIP_VERSION_MINOR)
      INFO("HIP runtime differs from the build's (%d.%d): dma-buf IPC is used, legacy hipIpc handles only on 7.2+",
           HIP_VERSION_MAJOR, HIP_VERSION_MINOR);
  });
}

// Shape parameters every rank must agree on (exchanged with the PeerInfo block).
struct ShapeInfo {
  int maxChannels, minChannels, nSlots;
  uint64_t slotBytes;
  CommTuning tune;
};

// Initialise `comm` (commDefaults already applied) in place. On failure its device/bootstrap resources
// are released but the object stays (the caller deletes it, or a non-blocking caller keeps it so the
// user can read the error with ncclCommGetAsyncError and then destroy it).
static ncclResult_t commInitRankInto(ncclComm* comm, int nranks, ncclUniqueId id, int rank, int dev) {
  ncclResult_t res = ncclSuccess;
  struct Blob {
    PeerInfo info;
    ShapeInfo shape;
  };
  std::vector<Blob> blobs(nranks);
  if ((res = bootstrapInit(&id, rank, nranks, &comm->bootstrap)) != ncclSuccess) goto fail;
  // Agree on the channel/slot shape and the tuning knobs: rank 0's parameters win (env may differ).
  {
    std::vector<ShapeInfo> shapes(nranks);
    shapes[rank] = {comm->maxChannels, comm->minCTAs, comm->nSlots, comm->slotBytes, comm->tune};
    if ((res = bootstrapAllGather(comm->bootstrap, shapes.data(), sizeof(ShapeInfo))) != ncclSuccess) goto fail;
    // NCCL_ALGO / NCCL_PROTO that did not parse on ANY rank fail every rank's init (reference: parseList's
    // ncclInvalidUsage out of ncclTopoTuneModel, src/graph/tuning.cc:456-461), so no rank is left waiting
    for (int r = 0; r < nranks; r++)
      if (shapes[r].tune.parseError) {
        WARN("rank %d: NCCL_ALGO / NCCL_PROTO could not be parsed on rank %d", rank, r);
        res = ncclInvalidUsage;
        goto fail;
      }
    comm->maxChannels = comm->maxCTAs = shapes[0].maxChannels;
    comm->nSlots = shapes[0].nSlots;
    comm->slotBytes = shapes[0].slotBytes;
    comm->tune = shapes[0].tune;
    // minCTAs raises every plan's channel count (planChannels), so it must agree too: a rank planning more
    // channels than its peers would wait on channels that never arrive
    comm->minCTAs = shapes[0].minChannels;
    if (comm->minCTAs > comm->maxCTAs) comm->minCTAs = comm->maxCTAs;
  }
  if ((res = transportSetup(comm)) != ncclSuccess) goto fail;
  if ((res = fillPeerInfo(comm, &blobs[rank].info)) != ncclSuccess) goto fail;
  TRACE("rank %d: handles exported", rank);
  if ((res = bootstrapAllGather(comm->bootstrap, blobs.data(), sizeof(Blob))) != ncclSuccess) goto fail;
  TRACE("rank %d: peer table gathered", rank);
  comm->peers.resize(nranks);
  for (int r = 0; r < nranks; r++) comm->peers[r] = blobs[r].info;
  computeChannelCap(comm);
  if ((res = transportConnect(comm)) != ncclSuccess) goto fail;
  TRACE("rank %d: peers mapped", rank);
  if ((res = commAllocDevState(comm)) != ncclSuccess) goto fail;
  TRACE("rank %d: device state ready", rank);
  // every peer mapping carries bytes both ways before the first collective (mapcheck.cc; all ranks fail together)
  if ((res = mapCheck({comm})) != ncclSuccess) goto fail;
  // ... and so does a plain device allocation, or eager zero-copy stays off on every rank (register.cc)
  if ((res = eagerProbe(comm)) != ncclSuccess) goto fail;
  if ((res = tunerLoad(comm)) != ncclSuccess) goto fail;
  if ((res = bootstrapBarrier(comm->bootstrap)) != ncclSuccess) goto fail;
  unexportHandles(comm);  // every peer has mapped our slab and flags
  logRuntimeOnce();
  INFO("comm %p rank %d nRanks %d dev %d busId %s - Init COMPLETE", (void*)comm, rank, nranks, dev,
       comm->peers[rank].busId);
  return ncclSuccess;
fail:
  transportFree(comm);
  bootstrapClose(comm->bootstrap);
  comm->bootstrap = nullptr;
  return res;
}

static ncclResult_t commInitRankDev(ncclComm** out, int nranks, ncclUniqueId id, int rank, int dev,
                                    const ncclConfig_t* cfg) {
  ncclComm* comm = new ncclComm();
  commDefaults(comm, rank, nranks, dev, cfg);
  ncclResult_t res = commInitRankInto(comm, nranks, id, rank, dev);
  if (res != ncclSuccess) {
    comm->startMagic = comm->endMagic = 0;
    delete comm;
    *out = nullptr;
    return res;
  }
  *out = comm;
  return ncclSuccess;
}

// Non-blocking communicator (config.blocking = 0; reference init.cc ncclCommInitRankConfig +
// ncclCommGetAsyncError): the handle is returned at once with ncclInProgress and initialisation runs
// on a thread; ncclCommGetAsyncError reports ncclInProgress until it finishes, then its result.
static ncclResult_t commInitRankAsync(ncclComm** out, int nranks, ncclUniqueId id, int rank, int dev,
                                      const ncclConfig_t* cfg) {
  ncclComm* comm = new ncclComm();
  commDefaults(comm, rank, nranks, dev, cfg);
  comm->asyncResult.store(ncclInProgress);
  comm->initThread = std::thread([comm, nranks, id, rank, dev]() {
    ncclResult_t r = hipSetDevice(dev) == hipSuccess ? commInitRankInto(comm, nranks, id, rank, dev)
                                                     : ncclUnhandledCudaError;
    comm->asyncResult.store(r);
  });
  *out = comm;
  return ncclInProgress;
}

}  // namespace ncclamd

using namespace ncclamd;

#define NCCL_ALIAS(ret, name, ...) extern "C" __attribute__((visibility("default"), alias(#name))) ret p##name(__VA_ARGS__);

NCCL_EXPORT ncclResult_t ncclGetVersion(int* version) {
  if (version == nullptr) return ncclInvalidArgument;
  *version = NCCL_VERSION_CODE;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclGetVersion, int*)

NCCL_EXPORT ncclResult_t ncclGetUniqueId(ncclUniqueId* out) {
  logInit();
  if (out == nullptr) {
    WARN("ncclGetUniqueId : out argument is NULL");
    return ncclInvalidArgument;
  }
  return bootstrapGetUniqueId(out);
}
NCCL_ALIAS(ncclResult_t, ncclGetUniqueId, ncclUniqueId*)

static ncclResult_t initRankCommon(ncclComm_t* newcomm, int nranks, ncclUniqueId commId, int myrank,
                                   ncclConfig_t* config) {
  logInit();
  if (newcomm == nullptr) {
    WARN("CommInitRank : comm argument is NULL");
    return ncclInvalidArgument;
  }
  *newcomm = nullptr;
  if (nranks < 1 || nranks > NCCL_AMD_MAX_RANKS) {
    WARN("Invalid number of ranks %d (this engine supports 1..%d intra-node ranks)", nranks, NCCL_AMD_MAX_RANKS);
    return ncclInvalidArgument;
  }
  if (myrank < 0 || myrank >= nranks) {
    WARN("Invalid rank requested : %d/%d", myrank, nranks);
    return ncclInvalidArgument;
  }
  NCCLCHECK(checkConfig(config));
  ipcDrainReleases();
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  ncclConfig_t cfgCopy;
  bool hasCfg = config != nullptr;
  if (hasCfg) cfgCopy = *config;
  if (groupActive()) {
    // Deferred to ncclGroupEnd, where all pending inits run concurrently (reference group.cc:35).
    return groupDeferInit([=]() -> ncclResult_t {
      HIPCHECK(hipSetDevice(dev));
      return commInitRankDev(newcomm, nranks, commId, myrank, dev, hasCfg ? &cfgCopy : nullptr);
    });
  }
  if (hasCfg && cfgCopy.blocking == 0) return commInitRankAsync(newcomm, nranks, commId, myrank, dev, &cfgCopy);
  return commInitRankDev(newcomm, nranks, commId, myrank, dev, hasCfg ? &cfgCopy : nullptr);
}

NCCL_EXPORT ncclResult_t ncclCommInitRankConfig(ncclComm_t* newcomm, int nranks, ncclUniqueId commId, int myrank,
                                                ncclConfig_t* config) {
  return initRankCommon(newcomm, nranks, commId, myrank, config);
}
NCCL_ALIAS(ncclResult_t, ncclCommInitRankConfig, ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*)

NCCL_EXPORT ncclResult_t ncclCommInitRank(ncclComm_t* newcomm, int nranks, ncclUniqueId commId, int myrank) {
  ROCTX_RANGE("ncclCommInitRank nranks=%d rank=%d", nranks, myrank);
  return initRankCommon(newcomm, nranks, commId, myrank, nullptr);
}
NCCL_ALIAS(ncclResult_t, ncclCommInitRank, ncclComm_t*, int, ncclUniqueId, int)

// Several ids (reference init.cc:2695-2728, nccl.h.in:260-264; the number and order of ids are the same on
// every rank). The reference spreads the bootstrap over nId roots; this single-node star rendezvouses at
// commIds[0], and each other id's root is told to exit by one rank (bootstrapReleaseUnused).
NCCL_EXPORT ncclResult_t ncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId,
                                                  ncclUniqueId* commIds, ncclConfig_t* config) {
  logInit();
  if (nId < 1 || commIds == nullptr) {
    WARN("ncclCommInitRankScalable : invalid nId %d or commIds NULL", nId);
    return ncclInvalidArgument;
  }
  if (newcomm != nullptr && nranks >= 1 && nranks <= NCCL_AMD_MAX_RANKS && myrank >= 0 && myrank < nranks &&
      checkConfig(config) == ncclSuccess) {
    NCCLCHECK(bootstrapReleaseUnused(commIds, nId, myrank, nranks));
  }
  return initRankCommon(newcomm, nranks, commIds[0], myrank, config);
}
NCCL_ALIAS(ncclResult_t, ncclCommInitRankScalable, ncclComm_t*, int, int, int, ncclUniqueId*, ncclConfig_t*)

// Single-process clique: every comm lives in this process, so peers are connected by raw pointers and
// no socket rendezvous is needed (reference init.cc:2581-2643 runs the generic path in threads).
NCCL_EXPORT ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
  logInit();
  ROCTX_RANGE("ncclCommInitAll ndev=%d", ndev);
  ipcDrainReleases();
  if (comms == nullptr) {
    WARN("CommInitAll : comms argument is NULL");
    return ncclInvalidArgument;
  }
  if (ndev < 0 || ndev > NCCL_AMD_MAX_RANKS) {
    WARN("Invalid device count requested : %d", ndev);
    return ncclInvalidArgument;
  }
  int total = 0;
  HIPCHECK(hipGetDeviceCount(&total));
  bool multiRank = paramInt("NCCL_MULTI_RANK_GPU_ENABLE", 0) != 0;  // reference init.cc:68
  std::vector<int> seen(total > 0 ? total : 1, 0);
  for (int i = 0; i < ndev; i++) {
    int d = devlist ? devlist[i] : i;
    if (d < 0 || d >= total) {
      WARN("Invalid device %d (totalnDev=%d)", d, total);
      return ncclInvalidArgument;
    }
    if (seen[d] && !multiRank) {
      WARN("Duplicate device %d in devlist (set NCCL_MULTI_RANK_GPU_ENABLE=1 to allow)", d);
      return ncclInvalidUsage;
    }
    seen[d] = 1;
  }
  if (ndev == 0) return ncclSuccess;
  int oldDev = 0;
  HIPCHECK(hipGetDevice(&oldDev));
  std::vector<ncclComm*> cs(ndev, nullptr);
  ncclResult_t res = ncclSuccess;
  std::vector<PeerInfo> infos(ndev);
  for (int i = 0; i < ndev && res == ncclSuccess; i++) {
    int d = devlist ? devlist[i] : i;
    cs[i] = new ncclComm();
    commDefaults(cs[i], i, ndev, d, nullptr);
    if (cs[i]->tune.parseError) {  // NCCL_ALGO / NCCL_PROTO (reference tuning.cc:456-461)
      res = ncclInvalidUsage;
      break;
    }
    res = transportSetup(cs[i]);
    if (res == ncclSuccess) res = fillPeerInfo(cs[i], &infos[i]);
  }
  for (int i = 0; i < ndev && res == ncclSuccess; i++) {
    cs[i]->peers = infos;
    computeChannelCap(cs[i]);
    res = transportConnect(cs[i]);
    if (res == ncclSuccess) res = commAllocDevState(cs[i]);
    if (res == ncclSuccess) res = tunerLoad(cs[i]);
  }
  if (res == ncclSuccess) res = mapCheck(cs);  // every peer pointer carries bytes both ways (mapcheck.cc)
  (void)hipSetDevice(oldDev);
  if (res != ncclSuccess) {
    for (auto* c : cs)
      if (c) {
        transportFree(c);
        delete c;
      }
    return res;
  }
  auto clique = cliqueCreate(ndev);
  for (int i = 0; i < ndev; i++) {
    cs[i]->clique = clique;
    comms[i] = cs[i];
  }
  logRuntimeOnce();
  INFO("ncclCommInitAll COMPLETE: %d ranks", ndev);
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommInitAll, ncclComm_t*, int, const int*)

void ncclamd::commPollAsync(ncclComm* comm) {
  if (comm->hostError && __atomic_load_n(comm->hostError, __ATOMIC_ACQUIRE) != DERR_NONE) {
    uint32_t e = __atomic_load_n(comm->hostError, __ATOMIC_ACQUIRE);
    int cur = ncclSuccess;
    ncclResult_t r = e == DERR_ABORT ? ncclRemoteError : e == DERR_MISMATCH ? ncclInvalidUsage : ncclSystemError;
    if (comm->asyncResult.compare_exchange_strong(cur, r))
      WARN("rank %d: device-side %s in a collective kernel", comm->rank,
           e == DERR_TIMEOUT    ? "spin timeout (peer never arrived)"
           : e == DERR_MISMATCH ? "kernel mismatch (a peer ran the other kernel for this collective: its buffers "
                                  "are registered on some ranks only, e.g. a registration that failed on one rank)"
                                : "abort");
  }
}

NCCL_EXPORT ncclResult_t ncclCommFinalize(ncclComm_t comm) {
  NCCLCHECK(commCheck(comm, "ncclCommFinalize", "comm"));
  if (comm->finalized) return ncclInvalidUsage;
  DeviceRestore restore;
  HIPCHECK(hipSetDevice(comm->device));
  HIPCHECK(hipDeviceSynchronize());
  ipcDrainReleases();  // a blocking entry point: peers' deregistered buffers are unmapped here (ipc.cc)
  regBlockingPoint(comm);  // and this rank's graph-released, stale, surplus eager and retired registrations (register.cc)
  if (comm->bootstrap) NCCLCHECK(bootstrapBarrier(comm->bootstrap));
  comm->finalized = true;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommFinalize, ncclComm_t)

static ncclResult_t commFree(ncclComm* comm, bool notifyPeers) {
  if (comm->initThread.joinable()) comm->initThread.join();  // a non-blocking init still running
  tunerUnload(comm);
  windowsFree(comm, notifyPeers);
  if (comm->internalStream) (void)hipStreamDestroy(comm->internalStream);
  if (comm->evIn) (void)hipEventDestroy(comm->evIn);
  if (comm->evOut) (void)hipEventDestroy(comm->evOut);
  transportFree(comm);
  bootstrapClose(comm->bootstrap);
  comm->bootstrap = nullptr;
  comm->startMagic = comm->endMagic = 0;
  delete comm;
  return ncclSuccess;
}

NCCL_EXPORT ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;  // reference: destroying NULL is a no-op
  NCCLCHECK(commCheck(comm, "ncclCommDestroy", "comm"));
  ipcDrainReleases();
  int old = 0;
  (void)hipGetDevice(&old);
  if (comm->initThread.joinable()) comm->initThread.join();
  (void)hipSetDevice(comm->device);
  // Local, like the reference (init.cc:2879-2911): wait for this rank's kernels, then for the credit
  // words peers still owe us (the only writes a peer can make after our kernels finished), so no
  // peer store lands in freed memory. No bootstrap barrier: one thread may destroy every comm of a
  // clique in turn (the reference's single-process pattern).
  (void)hipDeviceSynchronize();
  if (!comm->finalized) (void)transportDrainCredits(comm);
  commFree(comm, true);
  (void)hipSetDevice(old);
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommDestroy, ncclComm_t)

NCCL_EXPORT ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;
  NCCLCHECK(commCheck(comm, "ncclCommAbort", "comm"));
  if (comm->initThread.joinable()) comm->initThread.join();
  // Kernels poll the abort word inside every bounded spin (reference primitives.h:154-164).
  if (comm->hostAbort) __atomic_store_n(comm->hostAbort, 1u, __ATOMIC_RELEASE);
  DeviceRestore restore;
  (void)hipSetDevice(comm->device);
  (void)hipDeviceSynchronize();
  commFree(comm, false);
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommAbort, ncclComm_t)

NCCL_EXPORT const char* ncclGetErrorString(ncclResult_t code) {
  switch (code) {
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "unhandled hip error (run with NCCL_DEBUG=INFO for details)";
    case ncclSystemError: return "unhandled system error (run with NCCL_DEBUG=INFO for details)";
    case ncclInternalError: return "internal error - please report this issue to the NCCL developers";
    case ncclInvalidArgument: return "invalid argument (run with NCCL_DEBUG=WARN for details)";
    case ncclInvalidUsage: return "invalid usage (run with NCCL_DEBUG=WARN for details)";
    case ncclRemoteError: return "remote process exited or there was a network error";
    case ncclInProgress: return "NCCL operation in progress";
    case ncclTimeout: return "timeout";
    default: return "unknown result code";
  }
}
NCCL_ALIAS(const char*, ncclGetErrorString, ncclResult_t)

NCCL_EXPORT const char* ncclGetLastError(ncclComm_t comm) {
  (void)comm;
  return lastError();
}
NCCL_ALIAS(const char*, ncclGetLastError, ncclComm_t)

NCCL_EXPORT ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
  NCCLCHECK(commCheck(comm, "ncclGetAsyncError", "comm"));
  if (asyncError == nullptr) {
    WARN("ncclGetAsyncError : asyncError argument is NULL");
    return ncclInvalidArgument;
  }
  commPollAsync(comm);
  *asyncError = (ncclResult_t)comm->asyncResult.load();
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommGetAsyncError, ncclComm_t, ncclResult_t*)

NCCL_EXPORT ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  NCCLCHECK(commCheck(comm, "CommCount", "comm"));
  if (!count) return ncclInvalidArgument;
  *count = comm->nRanks;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommCount, const ncclComm_t, int*)

NCCL_EXPORT ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* devid) {
  NCCLCHECK(commCheck(comm, "CommCuDevice", "comm"));
  if (!devid) return ncclInvalidArgument;
  *devid = comm->device;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommCuDevice, const ncclComm_t, int*)

NCCL_EXPORT ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  NCCLCHECK(commCheck(comm, "CommUserRank", "comm"));
  if (!rank) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclCommUserRank, const ncclComm_t, int*)

// Reference mem_manager.cc:1010-1047. Everything this engine allocates for a communicator (staging slab,
// flag and LL lines, counters) is persistent — there is no suspend/resume — so Suspend is 0, Suspended
// is 0 and Total == Persist. A non-blocking communicator still initialising reports ncclInProgress.
NCCL_EXPORT ncclResult_t ncclCommMemStats(ncclComm_t comm, ncclCommMemStat_t stat, uint64_t* value) {
  NCCLCHECK(commCheck(comm, "ncclCommMemStats", "comm"));
  if (value == nullptr) return ncclInvalidArgument;
  int st = comm->asyncResult.load();
  if (st == ncclInProgress) return ncclInProgress;
  if (st != ncclSuccess) return (ncclResult_t)st;
  switch (stat) {
    case ncclStatGpuMemTotal:
    case ncclStatGpuMemPersist: *value = commDeviceBytes(comm); return ncclSuccess;
    case ncclStatGpuMemSuspend:
    case ncclStatGpuMemSuspended: *value = 0; return ncclSuccess;
    default: return ncclInvalidArgument;
  }
}
NCCL_ALIAS(ncclResult_t, ncclCommMemStats, ncclComm_t, ncclCommMemStat_t, uint64_t*)

// ---- custom operators (reference enqueue.cc:2560-2576 user ops, ncclRedOpCreatePreMulSum) ----
NCCL_EXPORT ncclResult_t ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                                  ncclScalarResidence_t residence, ncclComm_t comm) {
  NCCLCHECK(commCheck(comm, "ncclRedOpCreatePreMulSum", "comm"));
  if (op == nullptr || scalar == nullptr || datatype < 0 || datatype >= ncclNumTypes) return ncclInvalidArgument;
  UserRedOp u = {};
  u.used = true;
  u.datatype = datatype;
  u.devOp = DEV_PREMULSUM;
  if (residence == ncclScalarHostImmediate) {
    memcpy(&u.scalarArg, scalar, typeSize(datatype));
    u.scalarPtr = nullptr;
  } else if (residence == ncclScalarDevice) {
    u.scalarPtr = scalar;
  } else {
    return ncclInvalidArgument;
  }
  size_t ix = 0;
  while (ix < comm->userOps.size() && comm->userOps[ix].used) ix++;
  if (ix == comm->userOps.size()) comm->userOps.push_back(u);
  else comm->userOps[ix] = u;
  *op = (ncclRedOp_t)(ncclNumOps + ix);
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclRedOpCreatePreMulSum, ncclRedOp_t*, void*, ncclDataType_t, ncclScalarResidence_t,
           ncclComm_t)

NCCL_EXPORT ncclResult_t ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm) {
  NCCLCHECK(commCheck(comm, "ncclRedOpDestroy", "comm"));
  int ix = (int)op - (int)ncclNumOps;
  if (ix < 0 || ix >= (int)comm->userOps.size() || !comm->userOps[ix].used) {
    WARN("ncclRedOpDestroy : operator %d unknown to this communicator", (int)op);
    return ncclInvalidArgument;
  }
  comm->userOps[ix].used = false;
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclRedOpDestroy, ncclRedOp_t, ncclComm_t)

NCCL_EXPORT ncclResult_t ncclMemAlloc(void** ptr, size_t size) {
  if (ptr == nullptr) return ncclInvalidArgument;
  if (size == 0) {
    *ptr = nullptr;
    return ncclSuccess;
  }
  HIPCHECK(hipMalloc(ptr, size));
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclMemAlloc, void**, size_t)

NCCL_EXPORT ncclResult_t ncclMemFree(void* ptr) {
  if (ptr) HIPCHECK(hipFree(ptr));
  return ncclSuccess;
}
NCCL_ALIAS(ncclResult_t, ncclMemFree, void*)

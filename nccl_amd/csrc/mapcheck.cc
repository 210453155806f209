// mapcheck.cc — verify every peer mapping at communicator init, before the first collective.
//
// Reference: src/transport/p2p.cc:345-386 (p2pMap: a peer's buffer becomes a pointer in this process — a direct
// pointer with peer access in one process, an imported cuMem handle across processes) and :536-618 (the connection
// is set up from it). The reference trusts the mapping once the import returns. Here the mappings are checked with
// the bytes themselves, because this engine's cross-device paths (hipDeviceEnablePeerAccess, dma-buf imports of
// another GPU's memory, the hipIpc fallback, write-through stores and flag loads over xGMI) have run only with every
// rank on one GPU until the first 8-GPU node: a mapping that returns a pointer but does not carry the bytes would
// otherwise show up as a spin timeout (120 s) or silently wrong sums in the first collective.
//
// The check, for the communicator's local ranks (one for ncclCommInitRank, all for ncclCommInitAll):
//   1. every rank writes its own "self" pattern into its staging slab (slot [0][AG][0][me]) and flag block (probe
//      row 1) from the host, so it is in HBM before any peer reads it;
//   2. barrier; one wave per rank (kernels.hip mapCheckKernel) stores, through its mapping of every peer p, the
//      pattern (me -> p) into p's staging slot [0][RS][0][me] and flag probe row 0 [me] — the kernels' own store
//      flavour (16-byte system-scope write-through) — and loads p's self patterns through the same mappings;
//   3. barrier; every rank reads what its peers wrote into its memory and what it read from theirs, and compares
//      with the expected words (mapCheckWord: a function of a nonce every rank derives from the shared peer table);
//   4. the ranks exchange their outcome, so every rank fails the init together (ncclSystemError), each naming the
//      device pairs, allocations, directions and import paths it saw fail.
// A failed first round gets one more try: the ranks whose mappings failed re-import those peers through the hipIpc
// handle that rides along the dma-buf export (ipc.cc; transportRemapPeer) and every rank checks again; only a failure
// that survives it fails the init. NCCL_AMD_MAPCHECK=0 skips the check, NCCL_AMD_MAPCHECK_FALLBACK=0 the second
// round; NCCL_AMD_MAPCHECK_FAULT=1 (tests) makes this rank skip its remote stores, =2 in the first round only, =3
// fails this rank's part of the check before its kernel (the peers must fail with ncclRemoteError at once).
#include <string.h>

#include "core.h"

namespace ncclamd {

static uint64_t mix64(uint64_t x) {  // splitmix64 finalizer
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

uint64_t mapCheckWord(uint64_t nonce, int kind, int src, int dst, int half) {
  uint64_t w = mix64(nonce ^ ((uint64_t)kind << 40) ^ ((uint64_t)src << 24) ^ ((uint64_t)dst << 8) ^ (uint64_t)half);
  return w ? w : 1;  // never 0: fresh (zeroed) memory must not pass
}

static const char* kKind[2] = {"staging slab", "flag block"};

std::string mapCheckVerify(int me, int nRanks, uint64_t nonce, const MapCheckObs& obs, const MapCheckPeer* peers) {
  std::string out;
  char line[640];
  const MapCheckPeer& m = peers[me];
  for (int p = 0; p < nRanks; p++) {
    if (p == me) continue;
    for (int k = 0; k < 2; k++) {
      // direction 0: peer p stored into MY allocation through ITS mapping of it (p -> me); peers[p].pathIn names
      // how p maps this rank's memory
      const uint64_t w0 = mapCheckWord(nonce, k, p, me, 0), w1 = mapCheckWord(nonce, k, p, me, 1);
      if (obs.wrote[k][p][0] != w0 || obs.wrote[k][p][1] != w1) {
        snprintf(line, sizeof(line),
                 "rank %d (device %d, %s) -> rank %d (device %d, %s): 16-byte stores into rank %d's %s through rank "
                 "%d's mapping (%s) did not arrive: found %016llx %016llx, want %016llx %016llx\n",
                 p, peers[p].device, peers[p].busId, me, m.device, m.busId, me, kKind[k], p, peers[p].pathIn,
                 (unsigned long long)obs.wrote[k][p][0], (unsigned long long)obs.wrote[k][p][1], (unsigned long long)w0,
                 (unsigned long long)w1);
        out += line;
      }
      // direction 1: I loaded peer p's self pattern through MY mapping of p's allocation (me <- p)
      const uint64_t r0 = mapCheckWord(nonce, 2 + k, p, p, 0), r1 = mapCheckWord(nonce, 2 + k, p, p, 1);
      if (obs.read[k][p][0] != r0 || obs.read[k][p][1] != r1) {
        snprintf(line, sizeof(line),
                 "rank %d (device %d, %s) <- rank %d (device %d, %s): loads of rank %d's %s through rank %d's mapping "
                 "(%s) returned %016llx %016llx, want %016llx %016llx\n",
                 me, m.device, m.busId, p, peers[p].device, peers[p].busId, p, kKind[k], me, peers[p].path,
                 (unsigned long long)obs.read[k][p][0], (unsigned long long)obs.read[k][p][1], (unsigned long long)r0,
                 (unsigned long long)r1);
        out += line;
      }
    }
  }
  return out;
}

// The nonce: a hash of the peer table every rank holds (pids, devices, export keys, raw slab pointers), so the
// patterns of this communicator differ from anything an earlier one left in the same memory.
static uint64_t mapNonce(const ncclComm* c) {
  uint64_t h = 0x6d617063686b0001ull;
  for (const PeerInfo& p : c->peers) {
    h = mix64(h ^ (uint64_t)p.pid);
    h = mix64(h ^ ((uint64_t)p.device << 32 ^ (uint64_t)p.rank));
    h = mix64(h ^ p.stagingDesc.key ^ (p.flagsDesc.key << 1));
    h = mix64(h ^ p.stagingPtr ^ (p.flagsPtr << 1));
  }
  return h;
}

// How this rank maps rank r's memory (path) and how rank r maps this rank's (pathIn, from what this rank exported).
static const char* pathTo(const ncclComm* c, int r) {
  const PeerInfo& me = c->peers[c->rank];
  const PeerInfo& p = c->peers[r];
  if (p.pid == me.pid) return strcmp(p.busId, me.busId) ? "peer pointer, hipDeviceEnablePeerAccess" : "same-GPU pointer";
  if (c->peerStagingMap[r].legacy || c->peerFlagsMap[r].legacy) return "hipIpc handle, the dma-buf import's fallback";
  return "dma-buf import, hipImportExternalMemory";
}
static const char* pathFrom(const ncclComm* c, int r) {
  const PeerInfo& me = c->peers[c->rank];
  const PeerInfo& p = c->peers[r];
  if (p.pid == me.pid) return strcmp(p.busId, me.busId) ? "peer pointer, hipDeviceEnablePeerAccess" : "same-GPU pointer";
  if (me.stagingDesc.legacy || me.flagsDesc.legacy) return "hipIpc handle: this rank's dma-buf export was refused";
  return "dma-buf import, or its hipIpc fallback if that import failed there";
}

static uint64_t stagingSlot(const ncclComm* c, int kind, int from) {
  return ((((uint64_t)0 * STG_KINDS + kind) * c->nSlots + 0) * c->nRanks + from) * c->slotBytes;
}

// step 1: this rank's self patterns into its own memory, the slots peers will write cleared
static ncclResult_t mapPrepare(ncclComm* c, uint64_t nonce) {
  HIPCHECK(hipSetDevice(c->device));
  const int me = c->rank;
  uint64_t self[2][2];
  for (int k = 0; k < 2; k++)
    for (int h = 0; h < 2; h++) self[k][h] = mapCheckWord(nonce, 2 + k, me, me, h);
  char* st = (char*)c->staging;
  char* fl = (char*)c->flags + c->probeOffset;
  HIPCHECK(hipMemcpy(st + stagingSlot(c, STG_AG, me), self[0], 16, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(fl + NCCL_AMD_MAX_RANKS * 16, self[1], 16, hipMemcpyHostToDevice));
  for (int p = 0; p < c->nRanks; p++) {
    if (p == me) continue;
    HIPCHECK(hipMemset(st + stagingSlot(c, STG_RS, p), 0, 16));
    HIPCHECK(hipMemset(fl + (size_t)p * 16, 0, 16));
  }
  HIPCHECK(hipDeviceSynchronize());
  return ncclSuccess;
}

// step 2: the remote stores and loads (one wave), results into a device buffer
static ncclResult_t mapRun(ncclComm* c, uint64_t nonce, int attempt, uint64_t** outDev) {
  HIPCHECK(hipSetDevice(c->device));
  HIPCHECK(hipMalloc((void**)outDev, (size_t)NCCL_AMD_MAX_RANKS * 4 * sizeof(uint64_t)));
  HIPCHECK(hipMemset(*outDev, 0, (size_t)NCCL_AMD_MAX_RANKS * 4 * sizeof(uint64_t)));
  MapCheckArgs a;
  memset(&a, 0, sizeof(a));
  for (int p = 0; p < c->nRanks; p++)
    for (int k = 0; k < 2; k++)
      for (int h = 0; h < 2; h++) a.w[p][k][h] = mapCheckWord(nonce, k, c->rank, p, h);
  a.probeOff = c->probeOffset;
  // tests: 1 = this rank's stores never arrive; 2 = only in the first round (the remap below then fixes it)
  const int64_t fault = paramInt("NCCL_AMD_MAPCHECK_FAULT", 0);
  a.skip = fault == 1 || (fault == 2 && attempt == 0);
  NCCLCHECK(launchMapCheck(c->devComm, a, *outDev, nullptr));
  return ncclSuccess;
}

// step 3: what arrived here and what was read from the peers
static ncclResult_t mapCollect(ncclComm* c, uint64_t* outDev, MapCheckObs* obs) {
  HIPCHECK(hipSetDevice(c->device));
  memset(obs, 0, sizeof(*obs));
  std::vector<uint64_t> out((size_t)NCCL_AMD_MAX_RANKS * 4);
  HIPCHECK(hipMemcpy(out.data(), outDev, out.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  std::vector<uint64_t> row0(NCCL_AMD_MAX_RANKS * 2);
  HIPCHECK(hipMemcpy(row0.data(), (char*)c->flags + c->probeOffset, row0.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  for (int p = 0; p < c->nRanks; p++) {
    if (p == c->rank) continue;
    HIPCHECK(hipMemcpy(obs->wrote[0][p], (char*)c->staging + stagingSlot(c, STG_RS, p), 16, hipMemcpyDeviceToHost));
    obs->wrote[1][p][0] = row0[2 * p];
    obs->wrote[1][p][1] = row0[2 * p + 1];
    for (int k = 0; k < 2; k++)
      for (int h = 0; h < 2; h++) obs->read[k][p][h] = out[(size_t)p * 4 + 2 * k + h];
  }
  return ncclSuccess;
}

static ncclResult_t localBarrier(ncclComm* c) {
  if (c->bootstrap) return bootstrapBarrier(c->bootstrap);
  return ncclSuccess;  // ncclCommInitAll: one thread drives every rank, the steps run rank by rank
}

// One round of the check for the local comms. fail[r] (every rank of the communicator, filled for the local ones):
// bit p of .load = rank r's loads from p failed, bit p of .store = p's stores into rank r failed; .err = a step of
// the check itself failed on rank r (a HIP call, a remap). A rank whose step fails still joins both barriers and the
// closing all-gather, so its peers learn it at once instead of waiting in a barrier for the bootstrap timeout.
struct MapFail {
  uint32_t load, store;
  int32_t err;
  uint32_t pad;
};
static ncclResult_t mapRound(const std::vector<ncclComm*>& comms, uint64_t nonce, int attempt, ncclResult_t localErr,
                             std::vector<MapFail>& fail, std::string& report) {
  ncclResult_t res = localErr;
  std::vector<uint64_t*> outs(comms.size(), nullptr);
  for (ncclComm* c : comms)
    if (res == ncclSuccess) res = mapPrepare(c, nonce);
  NCCLCHECK(localBarrier(comms[0]));
  for (size_t i = 0; i < comms.size() && res == ncclSuccess; i++) res = mapRun(comms[i], nonce, attempt, &outs[i]);
  for (size_t i = 0; i < comms.size() && res == ncclSuccess; i++) {
    (void)hipSetDevice(comms[i]->device);
    if (hipDeviceSynchronize() != hipSuccess) res = ncclUnhandledCudaError;
  }
  // a failed barrier (the bootstrap is broken) still frees the probe buffers below, and then skips the closing
  // all-gather, which could only fail the same way
  const ncclResult_t bres = localBarrier(comms[0]);
  if (bres != ncclSuccess && res == ncclSuccess) res = bres;
  for (size_t i = 0; i < comms.size() && res == ncclSuccess; i++) {
    ncclComm* c = comms[i];
    MapCheckObs obs;
    res = mapCollect(c, outs[i], &obs);
    if (res != ncclSuccess) break;
    std::vector<MapCheckPeer> peers(c->nRanks);
    for (int r = 0; r < c->nRanks; r++) {
      peers[r].device = c->peers[r].device;
      memcpy(peers[r].busId, c->peers[r].busId, sizeof(peers[r].busId));
      peers[r].path = r == c->rank ? "local" : pathTo(c, r);
      peers[r].pathIn = r == c->rank ? "local" : pathFrom(c, r);
    }
    report += mapCheckVerify(c->rank, c->nRanks, nonce, obs, peers.data());
    MapFail& f = fail[c->rank];
    f.load = f.store = 0;
    for (int p = 0; p < c->nRanks; p++) {
      if (p == c->rank) continue;
      for (int k = 0; k < 2; k++) {
        if (obs.read[k][p][0] != mapCheckWord(nonce, 2 + k, p, p, 0) || obs.read[k][p][1] != mapCheckWord(nonce, 2 + k, p, p, 1))
          f.load |= 1u << p;
        if (obs.wrote[k][p][0] != mapCheckWord(nonce, k, p, c->rank, 0) || obs.wrote[k][p][1] != mapCheckWord(nonce, k, p, c->rank, 1))
          f.store |= 1u << p;
      }
    }
  }
  for (size_t i = 0; i < comms.size(); i++)
    if (outs[i]) {
      (void)hipSetDevice(comms[i]->device);
      (void)hipFree(outs[i]);
    }
  if (bres != ncclSuccess) return bres;
  for (ncclComm* c : comms) fail[c->rank].err = (int32_t)res;
  // every rank learns every rank's row (a rank whose own view is clean still learns that it must remap or fail)
  if (comms[0]->bootstrap) NCCLCHECK(bootstrapAllGather(comms[0]->bootstrap, fail.data(), sizeof(MapFail)));
  if (res != ncclSuccess) return res;
  for (size_t r = 0; r < fail.size(); r++)
    if (fail[r].err != ncclSuccess) {
      WARN("mapping check: rank %zu could not run its part of the check (error %d); failing the init here too", r,
           (int)fail[r].err);
      return ncclRemoteError;
    }
  return ncclSuccess;
}

ncclResult_t mapCheck(const std::vector<ncclComm*>& comms) {
  if (comms.empty() || comms[0]->nRanks == 1 || !paramInt("NCCL_AMD_MAPCHECK", 1)) return ncclSuccess;
  int oldDev = 0;
  (void)hipGetDevice(&oldDev);
  const int n = comms[0]->nRanks;
  const uint64_t nonce = mapNonce(comms[0]);
  std::vector<MapFail> fail(n, MapFail{0, 0, 0, 0});
  std::string report;
  // tests: 3 = this rank's check fails before its kernel (as a HIP error would)
  const ncclResult_t injected = paramInt("NCCL_AMD_MAPCHECK_FAULT", 0) == 3 ? ncclUnhandledCudaError : ncclSuccess;
  ncclResult_t res = mapRound(comms, nonce, 0, injected, fail, report);
  auto anyFail = [&]() {
    for (const MapFail& f : fail)
      if (f.load | f.store) return true;
    return false;
  };
  if (res == ncclSuccess && anyFail() && paramInt("NCCL_AMD_MAPCHECK_FALLBACK", 1)) {
    // Second chance for cross-process mappings: a rank re-imports every peer p whose loads through its mapping
    // failed, or into which its stores did not arrive (p's row), through the hipIpc handle that rides along the
    // dma-buf export where the runtime can open one (ipc.cc) — then every rank runs the check again. Every rank
    // sees the same table, so all take the second round together (a rank whose remap fails joins it with the error).
    if (!report.empty()) INFO("mapping check, first round:\n%s", report.c_str());
    report.clear();
    ncclResult_t remap = ncclSuccess;
    for (ncclComm* c : comms) {
      const int me = c->rank;
      for (int p = 0; p < n && remap == ncclSuccess; p++) {
        if (p == me || !(((fail[me].load >> p) & 1) || ((fail[p].store >> me) & 1))) continue;
        remap = transportRemapPeer(c, p);
      }
    }
    res = mapRound(comms, nonce ^ 0x5eedull, 1, remap, fail, report);
  }
  (void)hipSetDevice(oldDev);
  if (res != ncclSuccess) return res;
  ncclComm* c0 = comms[0];
  if (!anyFail()) {
    INFO("rank %d: peer mappings verified (store and load through every mapping, staging and flags)", c0->rank);
    return ncclSuccess;
  }
  if (!report.empty()) {
    size_t pos = 0;
    while (pos < report.size()) {
      size_t e = report.find('\n', pos);
      WARN("mapping check: %s", report.substr(pos, e - pos).c_str());
      pos = e + 1;
    }
  } else {
    int nbad = 0;
    for (const MapFail& f : fail) nbad += (f.load | f.store) ? 1 : 0;
    WARN("mapping check: rank %d's mappings carried the patterns, but %d rank(s) saw a mapping fail (their logs name "
         "the device pairs)", c0->rank, nbad);
  }
  return ncclSystemError;
}

}  // namespace ncclamd

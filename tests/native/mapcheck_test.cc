// mapcheck_test.cc — CPU test driver of the init-time mapping check (nccl_amd/csrc/mapcheck.cc) with the device and
// the imports stubbed: n "ranks" live in host memory, each rank's DevComm holds its "mappings" of the peers' staging
// slabs and flag blocks as plain pointers, and the check kernel (kernels.hip mapCheckKernel) is emulated on the host.
// Faults are injected where a real mapping could go wrong, and the check must fail the init with messages naming
// the device pair, the allocation, the direction and the import path.
//
//   mapcheck_test NRANKS [wrongmap:R:P:K] [legacy:R:P] [skip:R] [samepid] ...
//     wrongmap:R:P:K  rank R's mapping of rank P's staging (K=0) or flag block (K=1) points at other memory
//     legacy:R:P      rank R maps rank P's memory through a hipIpc handle (the dma-buf import's fallback)
//     skip:R          rank R's stores never arrive (NCCL_AMD_MAPCHECK_FAULT on that rank)
//     samepid         every rank in one process (peer pointers) instead of one process per rank
//     fixable:R:P     rank R's remap of rank P (the second round, transportRemapPeer) repairs its mapping
//     threads         one thread per rank, each calling mapCheck for its own comm (ncclCommInitRank), with the
//                     bootstrap's barrier and all-gather emulated across the threads
//     runfail:R       rank R's check kernel cannot be launched (a HIP error on that rank only)
// prints "result=<ncclResult_t>" (rank 0's) and "results=<r0>,<r1>,..."; the check's WARN lines go to stderr.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../nccl_amd/csrc/core.h"

static std::vector<int> gSkip;
static std::vector<int> gRunFail;

extern "C" {
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipGetDevice(int* d) {
  *d = 0;
  return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "stub"; }
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
  memcpy(d, s, n);
  return hipSuccess;
}
hipError_t hipMemset(void* d, int v, size_t n) {
  memset(d, v, n);
  return hipSuccess;
}
hipError_t hipMalloc(void** p, size_t n) {
  *p = calloc(1, n);
  return hipSuccess;
}
hipError_t hipFree(void* p) {
  free(p);
  return hipSuccess;
}
}

namespace ncclamd {
// "threads" mode: the bootstrap of rank r is the pointer value r + 1; barrier and all-gather across the threads
static int gN = 0;
static std::mutex gMu;
static std::condition_variable gCv;
static int gArrived = 0, gGen = 0;
static std::vector<char> gGather;
static int rankOf(Bootstrap* b) { return (int)(intptr_t)b - 1; }
static void barrier() {
  std::unique_lock<std::mutex> lk(gMu);
  const int gen = gGen;
  if (++gArrived == gN) {
    gArrived = 0;
    gGen++;
    gCv.notify_all();
  } else {
    gCv.wait(lk, [&] { return gGen != gen; });
  }
}
ncclResult_t bootstrapBarrier(Bootstrap*) {
  barrier();
  return ncclSuccess;
}
ncclResult_t bootstrapAllGather(Bootstrap* b, void* data, size_t bytes) {
  const int r = rankOf(b);
  {
    std::lock_guard<std::mutex> lk(gMu);
    if (gGather.size() < bytes * gN) gGather.resize(bytes * gN);
    memcpy(gGather.data() + r * bytes, (char*)data + r * bytes, bytes);
  }
  barrier();
  {
    std::lock_guard<std::mutex> lk(gMu);
    memcpy(data, gGather.data(), bytes * gN);
  }
  barrier();
  return ncclSuccess;
}
// the check kernel, on the host (kernels.hip mapCheckKernel)
ncclResult_t launchMapCheck(const DevComm* dcp, const MapCheckArgs& a, uint64_t* out, hipStream_t) {
  const DevComm& dc = *dcp;
  const int me = dc.rank;
  if (gRunFail[me]) return ncclUnhandledCudaError;
  for (int p = 0; p < dc.nRanks; p++) {
    if (p == me) continue;
    char* fl = (char*)dc.flags[p] + a.probeOff;
    if (!a.skip && !gSkip[me]) {
      memcpy(dc.staging[p] + stagingOffset(dc, 0, STG_RS, 0, me), a.w[p][0], 16);
      memcpy(fl + (size_t)me * 16, a.w[p][1], 16);
    }
    memcpy(out + p * 4, dc.staging[p] + stagingOffset(dc, 0, STG_AG, 0, p), 16);
    memcpy(out + p * 4 + 2, fl + NCCL_AMD_MAX_RANKS * 16, 16);
  }
  return ncclSuccess;
}
// the second round's remap (transport.cc transportRemapPeer): "fixable" faults are repaired by it
static std::vector<std::vector<int>> gFixable;
static std::vector<DevComm>* gDcs = nullptr;
static std::vector<ncclComm*>* gComms = nullptr;
int gRemaps = 0;
ncclResult_t transportRemapPeer(ncclComm* comm, int r) {
  gRemaps++;
  if (gFixable[comm->rank][r]) {
    (*gDcs)[comm->rank].staging[r] = (char*)(*gComms)[r]->staging;
    (*gDcs)[comm->rank].flags[r] = (*gComms)[r]->flags;
    comm->peerStagingMap[r].legacy = 1;
  }
  printf("remap %d<-%d\n", comm->rank, r);
  return ncclSuccess;
}
}  // namespace ncclamd

using namespace ncclamd;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2;
  gSkip.assign(n, 0);
  gRunFail.assign(n, 0);
  gN = n;
  bool threads = false;
  gFixable.assign(n, std::vector<int>(n, 0));
  bool samePid = false;
  const size_t slot = 4096, probe = 8192;
  std::vector<ncclComm*> cs(n);
  std::vector<PeerInfo> peers(n);
  for (int r = 0; r < n; r++) {
    ncclComm* c = new ncclComm();
    c->rank = r;
    c->nRanks = n;
    c->device = r;
    c->nSlots = 2;
    c->slotBytes = slot;
    c->maxChannels = 1;
    c->probeOffset = probe;
    c->staging = calloc(1, (size_t)STG_KINDS * 2 * n * slot);
    c->flags = (uint64_t*)calloc(1, probe + kMapProbeBytes);
    memset(c->staging, 0xEE, (size_t)STG_KINDS * 2 * n * slot);  // fresh memory is not zeroed
    cs[r] = c;
  }
  for (int i = 2; i < argc; i++) {
    if (!strcmp(argv[i], "samepid")) samePid = true;
    if (!strcmp(argv[i], "threads")) threads = true;
  }
  for (int r = 0; r < n; r++) {
    PeerInfo& p = peers[r];
    memset(&p, 0, sizeof(p));
    p.rank = r;
    p.device = r;
    p.pid = samePid ? 1000 : 1000 + r;
    snprintf(p.busId, sizeof(p.busId), "0000:%02x:00.0", 0x10 + r);
    p.stagingDesc.key = 100 + r;
    p.flagsDesc.key = 200 + r;
    p.stagingPtr = (uint64_t)cs[r]->staging;
    p.flagsPtr = (uint64_t)cs[r]->flags;
  }
  std::vector<DevComm> dcs(n);
  std::vector<std::vector<char>> decoys;
  for (int r = 0; r < n; r++) {
    cs[r]->peers = peers;
    DevComm& d = dcs[r];
    memset(&d, 0, sizeof(d));
    d.rank = r;
    d.nRanks = n;
    d.nSlots = 2;
    d.maxChannels = 1;
    d.slotBytes = slot;
    for (int p = 0; p < n; p++) {
      d.staging[p] = (char*)cs[p]->staging;
      d.flags[p] = cs[p]->flags;
    }
    cs[r]->devComm = &d;
  }
  decoys.reserve(64);
  for (int i = 2; i < argc; i++) {
    int R = 0, P = 0, K = 0;
    if (sscanf(argv[i], "wrongmap:%d:%d:%d", &R, &P, &K) == 3) {
      decoys.emplace_back(probe + kMapProbeBytes + (size_t)STG_KINDS * 2 * n * slot, (char)0x5A);
      if (K == 0) dcs[R].staging[P] = decoys.back().data();
      else dcs[R].flags[P] = (uint64_t*)decoys.back().data();
    } else if (sscanf(argv[i], "legacy:%d:%d", &R, &P) == 2) {
      cs[R]->peerStagingMap[P].legacy = 1;
    } else if (sscanf(argv[i], "skip:%d", &R) == 1) {
      gSkip[R] = 1;
    } else if (sscanf(argv[i], "fixable:%d:%d", &R, &P) == 2) {
      gFixable[R][P] = 1;
    } else if (sscanf(argv[i], "runfail:%d", &R) == 1) {
      gRunFail[R] = 1;
    }
  }
  gDcs = &dcs;
  gComms = &cs;
  logInit();
  std::vector<ncclResult_t> res(n, ncclSuccess);
  if (threads) {
    std::vector<std::thread> ts;
    for (int r = 0; r < n; r++) {
      cs[r]->bootstrap = (Bootstrap*)(intptr_t)(r + 1);
      ts.emplace_back([&, r] { res[r] = mapCheck(std::vector<ncclComm*>{cs[r]}); });
    }
    for (std::thread& t : ts) t.join();
  } else {
    res.assign(n, mapCheck(cs));
  }
  printf("result=%d\nresults=", (int)res[0]);
  for (int r = 0; r < n; r++) printf("%s%d", r ? "," : "", (int)res[r]);
  printf("\n");
  return 0;
}

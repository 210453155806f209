// tuner.cc — external tuner plugins (NCCL_TUNER_PLUGIN) over the reference's tuner ABI v4-v6.
//
// Reference: src/plugin/tuner.cc:38-120 (load once per process, refcounted: NCCL_TUNER_PLUGIN names a
// path or `libnccl-tuner-<name>.so`, "none" disables; symbols ncclTunerPlugin_v6 → v5 → v4),
// src/include/plugin/tuner/tuner_v6.h:12-83 (init / getCollInfo / finalize / getChunkSize),
// src/enqueue.cc topoGetAlgoInfo (NCCL fills a [algorithm][protocol] cost table with its model's times,
// the plugin may rewrite it and set nChannels, NCCL then takes the cheapest entry).
//
// Mapping onto this engine (one xGMI node): for AllReduce, (TREE|RING, LL) → the LL
// kernel, (TREE, SIMPLE) → one-shot, (RING, SIMPLE) → direct scatter-reduce-gather; for ReduceScatter,
// AllGather and Reduce only (RING, SIMPLE) exists. Every other entry is NCCL_ALGO_PROTO_IGNORE. A plugin
// that leaves the table unchanged keeps the engine's own size table; nChannels > 0 overrides the channel
// count (clamped to what the chosen kernel supports).
#include <dlfcn.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "../../include/nccl_tuner.h"
#include "core.h"

namespace ncclamd {

namespace {
std::mutex gMu;
int gStatus = 0;  // 0 not tried, 1 loaded, 2 failed / disabled
void* gLib = nullptr;
int gVersion = 0;
const ncclTuner_v6_t* gV6 = nullptr;
const ncclTuner_v5_t* gV5 = nullptr;
const ncclTuner_v4_t* gV4 = nullptr;
int gRefs = 0;

void tunerLog(ncclDebugLogLevel level, unsigned long, const char* file, int line, const char* fmt, ...) {
  if ((int)level > gLogLevel) return;
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  logMessage((int)level, file, line, "TUNER %s", buf);
}

void* openLib(const char* name) {
  std::string tries[3];
  int n = 0;
  if (name) {
    tries[n++] = name;
    tries[n++] = std::string("libnccl-tuner-") + name + ".so";
  } else {
    tries[n++] = "libnccl-tuner.so";
  }
  for (int i = 0; i < n; i++) {
    void* h = dlopen(tries[i].c_str(), RTLD_NOW | RTLD_LOCAL);
    if (h) {
      INFO("TUNER/Plugin: loaded %s", tries[i].c_str());
      return h;
    }
  }
  if (name) WARN("TUNER/Plugin: could not load %s (%s)", name, dlerror());
  return nullptr;
}
}  // namespace

ncclResult_t tunerLoad(ncclComm* comm) {
  std::lock_guard<std::mutex> lk(gMu);
  comm->tunerCtx = nullptr;
  comm->tunerLoaded = false;
  if (gStatus == 2) return ncclSuccess;
  if (gStatus == 0) {
    const char* name = paramStr("NCCL_TUNER_PLUGIN");
    if (name && !strcasecmp(name, "none")) {
      gStatus = 2;
      return ncclSuccess;
    }
    gLib = openLib(name);
    if (gLib) {
      if ((gV6 = (const ncclTuner_v6_t*)dlsym(gLib, "ncclTunerPlugin_v6"))) gVersion = 6;
      else if ((gV5 = (const ncclTuner_v5_t*)dlsym(gLib, "ncclTunerPlugin_v5"))) gVersion = 5;
      else if ((gV4 = (const ncclTuner_v4_t*)dlsym(gLib, "ncclTunerPlugin_v4"))) gVersion = 4;
    }
    if (!gVersion) {
      if (gLib) {
        WARN("TUNER/Plugin: no ncclTunerPlugin_v6/v5/v4 symbol; ignoring the plugin");
        dlclose(gLib);
      }
      gLib = nullptr;
      gStatus = 2;
      return ncclSuccess;
    }
    gStatus = 1;
  }
  ncclNvlDomainInfo_v6_t dom = {1, comm->nRanks, comm->nRanks};  // one xGMI "domain": the node
  ncclTunerConstants_v6_t consts;
  memset(&consts, 0, sizeof(consts));
  uint64_t commId = comm->peers.empty() ? 0 : comm->peers[0].hostHash ^ (uint64_t)(uintptr_t)comm->devComm;
  ncclResult_t r = ncclSuccess;
  if (gVersion == 6) r = gV6->init(&comm->tunerCtx, commId, comm->nRanks, 1, tunerLog, &dom, &consts);
  else if (gVersion == 5) r = gV5->init(&comm->tunerCtx, commId, comm->nRanks, 1, tunerLog, &dom, &consts);
  else r = gV4->init(comm->nRanks, 1, tunerLog, &comm->tunerCtx);
  if (r != ncclSuccess) {
    WARN("TUNER/Plugin: init failed (%d); default tuning for this communicator", (int)r);
    return ncclSuccess;
  }
  comm->tunerLoaded = true;
  gRefs++;
  return ncclSuccess;
}

void tunerUnload(ncclComm* comm) {
  std::lock_guard<std::mutex> lk(gMu);
  if (!comm->tunerLoaded) return;
  if (gVersion == 6) gV6->finalize(comm->tunerCtx);
  else if (gVersion == 5) gV5->finalize(comm->tunerCtx);
  else if (gVersion == 4) gV4->destroy(comm->tunerCtx);
  comm->tunerLoaded = false;
  comm->tunerCtx = nullptr;
  if (--gRefs == 0 && gLib) {
    dlclose(gLib);
    gLib = nullptr;
    gV6 = nullptr;
    gV5 = nullptr;
    gV4 = nullptr;
    gVersion = 0;
    gStatus = 0;
  }
}

// The engine's cost model (µs, the unit of the reference's tuning table, tuning.cc): a fixed launch +
// handshake latency plus the busiest resource's time — a rank's link bytes over its n-1 xGMI links
// (≈50 GB/s per link and direction, ring / chain: over ONE link), or its local HBM bytes at ≈6.3 TB/s
// (MI355X_MICROARCH.md's measured copy rate), whichever is longer; one-shot runs on at most 32 channels and
// one channel's workgroup moves ≈50 GB/s (scripts/wg_rate_probe.hip), so its HBM rate is capped
// at 1.6 TB/s — which puts its n = 2 crossover with direct at ≈2.4 MB, where the one-GPU rehearsal has it
// (2 MiB one-shot 14.1 µs vs direct 16.0, 4 MiB 23.1 vs 17.7). `bytes` is the collective's size as the
// tuner sees it (AllReduce / Reduce: the buffer; ReduceScatter / AllGather: n × the per-rank block).
// Used for the plugin's cost table and by ncclGroupSimulateEnd.
ModelCost modelCost(ModelAlgo a, CollFunc func, int n, size_t bytes) {
  const double S = (double)bytes, link = 5.0e4 /* B/µs per link */, hbm = 6.3e6 /* B/µs */;
  const double oneShotHbm = std::min(hbm, 32 * 5.0e4);  // 32 channels x ≈50 GB/s per workgroup
  if (n <= 1) return {2.0, (a == MODEL_COPY ? 2.0 * S : 0.0) / hbm};  // one rank: a copy or nothing
  const double nl = n - 1.0;
  const bool ar = func == FUNC_ALLREDUCE, red = func == FUNC_REDUCE;
  double lat = 10.0, linkB = 0, hbmB = 0, links = nl;
  switch (a) {
    case MODEL_LL:  // 16-byte lines carry 8 payload bytes, to every peer for AllReduce / Reduce
      lat = 4.0;
      linkB = (ar || red ? 2.0 * nl : 2.0 * nl / n) * S;
      break;
    case MODEL_LL128:  // 64-byte lines carry 56 payload bytes
      lat = 4.5;
      linkB = (64.0 / 56.0) * (ar || red ? nl : nl / n) * S;
      break;
    case MODEL_ONESHOT:  // every rank publishes its buffer to every peer and folds all n
      lat = 7.0;
      linkB = nl * S;
      hbmB = (n + 1.0) * S;
      break;
    case MODEL_DIRECT:  // scatter-reduce-gather: 2(n-1)/n S (AllReduce), (n-1)/n S (RS / AG / Reduce)
    case MODEL_SYM:
      lat = a == MODEL_SYM ? 8.0 : 10.0;
      linkB = (ar ? 2.0 * nl / n : nl / n) * S;
      hbmB = ar ? (2.0 + 4.0 * nl / n) * S : 2.0 * S;
      break;
    case MODEL_RING:  // one link per direction; n-1 (RS / AG) or 2(n-1) (AllReduce) pipelined hops
      lat = 10.0 + 2.0 * (ar ? 2.0 * nl : nl);
      linkB = (ar ? 2.0 * nl / n : nl / n) * S;
      hbmB = ar ? (2.0 + 4.0 * nl / n) * S : 2.0 * S;
      links = 1.0;
      break;
    case MODEL_CHAIN:  // reduce up the chain and broadcast down: S per link and direction, 2(n-1) hops
      lat = 10.0 + 3.0 * 2.0 * nl;
      linkB = S;
      hbmB = 4.0 * S;
      links = 1.0;
      break;
    case MODEL_COPY: break;
  }
  const double t = std::max(linkB / (links * link), hbmB / (a == MODEL_ONESHOT ? oneShotHbm : hbm));
  return {lat, t};
}

// Ask the plugin. `algo` (in: the engine's default choice, out: the plugin's) and `nch` (out: channel
// override or 0). llMask: 1 = the LL kernel can take this collective, 2 = the LL64 (LL128-class) one can.
// regBuff: the reference's (enqueue.cc:2141-2147), computed by the caller.
void tunerPick(ncclComm* comm, CollFunc func, size_t bytes, int numPipeOps, int llMask, int regBuff, int* algo, int* nch) {
  const bool llOk = (llMask & 1) != 0, ll128Ok = (llMask & 2) != 0;
  *nch = 0;
  if (!comm->tunerLoaded) return;
  const int n = comm->nRanks;
  auto us = [&](ModelAlgo a) { return (float)modelCost(a, func, n, bytes).total(); };
  float table[NCCL_NUM_ALGORITHMS][NCCL_NUM_PROTOCOLS];
  for (int a = 0; a < NCCL_NUM_ALGORITHMS; a++)
    for (int p = 0; p < NCCL_NUM_PROTOCOLS; p++) table[a][p] = (float)NCCL_ALGO_PROTO_IGNORE;
  ncclFunc_t f = ncclFuncAllReduce;
  if (func == FUNC_ALLREDUCE) {
    if (llOk) {
      table[NCCL_ALGO_RING][NCCL_PROTO_LL] = us(MODEL_LL);
      table[NCCL_ALGO_TREE][NCCL_PROTO_LL] = table[NCCL_ALGO_RING][NCCL_PROTO_LL];
    }
    if (ll128Ok) table[NCCL_ALGO_RING][NCCL_PROTO_LL128] = us(MODEL_LL128);
    table[NCCL_ALGO_TREE][NCCL_PROTO_SIMPLE] = us(MODEL_ONESHOT);
    table[NCCL_ALGO_RING][NCCL_PROTO_SIMPLE] = us(MODEL_DIRECT);
  } else {
    f = func == FUNC_REDUCESCATTER ? ncclFuncReduceScatter : func == FUNC_ALLGATHER ? ncclFuncAllGather : ncclFuncReduce;
    table[NCCL_ALGO_RING][NCCL_PROTO_SIMPLE] = us(MODEL_DIRECT);
    if (llOk) table[NCCL_ALGO_RING][NCCL_PROTO_LL] = us(MODEL_LL);
    if (ll128Ok) table[NCCL_ALGO_RING][NCCL_PROTO_LL128] = us(MODEL_LL128);
  }
  float before[NCCL_NUM_ALGORITHMS][NCCL_NUM_PROTOCOLS];
  memcpy(before, table, sizeof(table));
  int ch = 0;
  ncclResult_t r;
  if (gVersion == 6) r = gV6->getCollInfo(comm->tunerCtx, f, bytes, numPipeOps, (float**)table, NCCL_NUM_ALGORITHMS, NCCL_NUM_PROTOCOLS, regBuff, &ch);
  else if (gVersion == 5) r = gV5->getCollInfo(comm->tunerCtx, f, bytes, numPipeOps, (float**)table, NCCL_NUM_ALGORITHMS, NCCL_NUM_PROTOCOLS, regBuff, &ch);
  else r = gV4->getCollInfo(comm->tunerCtx, f, bytes, numPipeOps, (float**)table, NCCL_NUM_ALGORITHMS, NCCL_NUM_PROTOCOLS, regBuff, &ch);
  if (r != ncclSuccess) return;  // reference: fall back to the default tuning
  if (ch > 0) *nch = ch;
  if (!memcmp(before, table, sizeof(table))) return;  // table untouched: keep the engine's size table
  int bestA = -1, bestP = -1;
  for (int a = 0; a < NCCL_NUM_ALGORITHMS; a++)
    for (int p = 0; p < NCCL_NUM_PROTOCOLS; p++) {
      if (before[a][p] < 0 || table[a][p] < 0) continue;  // not offered / ignored
      if (bestA < 0 || table[a][p] < table[bestA][bestP]) bestA = a, bestP = p;
    }
  if (bestA < 0) return;
  if (bestP == NCCL_PROTO_LL) *algo = TUNE_LL;
  else if (bestP == NCCL_PROTO_LL128) *algo = TUNE_LL128;
  else if (bestA == NCCL_ALGO_TREE) *algo = TUNE_ONESHOT;
  else *algo = TUNE_DIRECT;
  TRACE("tuner: func %d bytes %zu -> algo %d proto %d (%d) nch %d", (int)func, bytes, bestA, bestP, *algo, *nch);
}

}  // namespace ncclamd

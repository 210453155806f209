// group.cc — ncclGroupStart / ncclGroupEnd.
//
// Reference: src/include/group.h:81-155 (thread-local group depth), src/group.cc:766-887
// (ncclGroupEndInternal), :598-760 (groupLaunch), :35 (ncclAsyncLaunch of deferred inits).
// Semantics kept: group state is thread-local; calls inside a group are only recorded, and nothing
// is enqueued on any stream until the outermost ncclGroupEnd; communicator inits inside a group run
// concurrently at ncclGroupEnd (required when one thread creates several ranks). Kernel launches here
// never block on peers (all connections are made at init), so one thread may drive every device of
// the node even without a group — the group is still honoured for ordering and error reporting.
#include <string.h>

#include <functional>
#include <map>
#include <thread>
#include <vector>

#include "core.h"

namespace ncclamd {

struct GroupState {
  int depth = 0;
  ncclResult_t error = ncclSuccess;
  std::vector<CollInfo> colls;
  std::vector<std::function<ncclResult_t()>> inits;
};
static thread_local GroupState tGroup;

bool groupActive() { return tGroup.depth > 0; }

ncclResult_t groupStartInternal() {
  tGroup.depth++;
  return ncclSuccess;
}

ncclResult_t groupDeferColl(const CollInfo& info) {
  tGroup.colls.push_back(info);
  return ncclSuccess;
}

ncclResult_t groupDeferInit(std::function<ncclResult_t()> job) {
  tGroup.inits.push_back(std::move(job));
  return ncclSuccess;
}

void groupRecordError(ncclResult_t r) {
  if (tGroup.depth > 0 && tGroup.error == ncclSuccess && r != ncclSuccess) tGroup.error = r;
}

// Model time of one planned op (ncclGroupSimulateEnd): which kernel it planned onto and its tuner-sized bytes.
static ModelCost planCost(const PlannedColl& pc) {
  const ncclComm* comm = pc.info.comm;
  const int n = comm->nRanks;
  size_t bytes = pc.info.count * (size_t)typeSize(pc.info.datatype);
  if (pc.info.func == FUNC_REDUCESCATTER || pc.info.func == FUNC_ALLGATHER) bytes *= (size_t)n;
  ModelAlgo a = MODEL_DIRECT;
  if (pc.kind == PLAN_SYM) a = MODEL_SYM;
  else switch (pc.p.algo) {
    case ALGO_COPY:
    case ALGO_ONERANK: a = MODEL_COPY; break;
    case ALGO_LL: a = pc.p.ll.ops[0].proto == LLP_LL64 ? MODEL_LL128 : MODEL_LL; break;
    case ALGO_ONESHOT: a = MODEL_ONESHOT; break;
    case ALGO_PIPE:
      a = pc.p.pipeKind == PIPE_CHAIN_AR || pc.p.pipeKind == PIPE_CHAIN_REDUCE ? MODEL_CHAIN : MODEL_RING;
      break;
    default: a = MODEL_DIRECT; break;
  }
  return modelCost(a, pc.info.func, n, bytes);
}

// ncclGroupSimulateEnd (reference group.cc:116-123, :766-866 with simInfo): the group's collectives are
// planned exactly as ncclGroupEnd would plan them (same batches) and dropped instead of launched; deferred
// communicator inits still run. estimatedTime = the cost model's µs for the group: per communicator, one
// latency per launch plus every op's transfer time, and the slowest communicator (they run concurrently on
// their own GPUs). The reference reports the model time of the last op it planned; for a one-op group the
// two agree.
static ncclResult_t groupSimulate(std::vector<CollInfo>& colls, float* estimatedUs) {
  std::map<ncclComm*, double> perComm;
  std::map<ncclComm*, std::vector<PlannedColl>> open;
  auto flush = [&](ncclComm* c) {
    std::vector<PlannedColl>& run = open[c];
    if (run.empty()) return;
    double t = 0;
    for (size_t k = 0; k < run.size(); k++) {
      if (run[k].kind == PLAN_NONE) continue;
      ModelCost m = planCost(run[k]);
      t += (k == 0 ? m.latUs : 0.0) + m.xferUs;
    }
    perComm[c] += t;
    run.clear();
  };
  for (size_t i = 0; i < colls.size(); i++) {
    PlannedColl pc;
    pc.info = colls[i];
    const uint64_t opCount = pc.info.comm->opCount;  // nothing is launched: keep the op counter as it was
    tPlanOnly = true;  // and nothing is registered (eager registration, register.cc)
    const ncclResult_t r = planColl(pc.info, pc.p, pc.sp, &pc.kind);
    tPlanOnly = false;
    NCCLCHECK(r);
    pc.info.comm->opCount = opCount;
    std::vector<PlannedColl>& run = open[pc.info.comm];
    if (!batchable(run, pc)) flush(pc.info.comm);
    run.push_back(pc);
  }
  for (auto& kv : open) flush(kv.first);
  double worst = 0;
  for (auto& kv : perComm) worst = kv.second > worst ? kv.second : worst;
  *estimatedUs = (float)worst;
  return ncclSuccess;
}

ncclResult_t groupEndInternal(ncclSimInfo_t* simInfo) {
  if (tGroup.depth == 0) {
    WARN("ncclGroupEnd: not in a group call.");
    return ncclInvalidUsage;
  }
  ncclSimInfo_t sim;
  size_t simSize = 0;
  if (simInfo) {  // reference group.cc:792-800: copy what the caller's (possibly older) struct holds
    memcpy(&simSize, &simInfo->size, sizeof(size_t));
    if (simSize > sizeof(ncclSimInfo_t)) simSize = sizeof(ncclSimInfo_t);
    sim = NCCL_SIM_INFO_INITIALIZER;
    memcpy(&sim, simInfo, simSize);
  }
  if (--tGroup.depth > 0) return ncclSuccess;
  ncclResult_t ret = tGroup.error;
  std::vector<CollInfo> colls;
  std::vector<std::function<ncclResult_t()>> inits;
  colls.swap(tGroup.colls);
  inits.swap(tGroup.inits);
  tGroup.error = ncclSuccess;
  if (ret != ncclSuccess) return ret;  // a call inside the group failed its checks: launch nothing
  if (simInfo && sim.magic != 0x74685283) {
    WARN("ncclSimInfo_t argument not initialized via NCCL_SIM_INFO_INITIALIZER");
    return ncclInvalidArgument;
  }

  if (!inits.empty()) {
    std::vector<ncclResult_t> rs(inits.size(), ncclSuccess);
    std::vector<std::thread> ts;
    int dev = 0;
    (void)hipGetDevice(&dev);
    for (size_t i = 0; i < inits.size(); i++) ts.emplace_back([&, i]() { rs[i] = inits[i](); });
    for (auto& t : ts) t.join();
    (void)hipSetDevice(dev);
    for (auto r : rs)
      if (r != ncclSuccess) return r;
  }
  if (simInfo) {
    float us = 0;
    NCCLCHECK(groupSimulate(colls, &us));
    sim.estimatedTime = us;
    memcpy(simInfo, &sim, simSize);
    return ncclSuccess;
  }
  int dev = 0;
  (void)hipGetDevice(&dev);
  // each communicator's upkeep first, before any of the group's kernels is launched (enqueue.cc collProgress; not
  // while any of its streams in this group is being captured)
  for (size_t i = 0; i < colls.size(); i++) {
    bool seen = false;
    for (size_t j = 0; j < i && !seen; j++) seen = colls[j].comm == colls[i].comm;
    if (seen) continue;
    bool capturing = false;
    for (size_t j = i; j < colls.size() && !capturing; j++) {
      if (colls[j].comm != colls[i].comm) continue;
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      capturing = hipStreamIsCapturing(colls[j].stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone;
      (void)hipGetLastError();
    }
    if (capturing) continue;
    (void)hipSetDevice(colls[i].comm->device);
    collProgress(colls[i].comm, colls[i].stream);
  }
  ncclResult_t r = ncclSuccess;
  for (size_t i = 0; i < colls.size() && r == ncclSuccess; i++) r = collFork(colls[i]);
  // launches in group order per comm; consecutive ops that planned onto the same kernel with the same stream,
  // type and operator become one launch (enqueue.cc batchable / launchBatch). Every rank of a comm issues the
  // same op sequence, so every rank forms the same batches.
  std::map<ncclComm*, std::vector<PlannedColl>> open;
  auto flush = [&](ncclComm* c) -> ncclResult_t {
    std::vector<PlannedColl>& run = open[c];
    ncclResult_t res = run.empty() ? ncclSuccess : launchBatch(run);
    run.clear();
    return res;
  };
  for (size_t i = 0; i < colls.size() && r == ncclSuccess; i++) {
    PlannedColl pc;
    pc.info = colls[i];
    (void)hipSetDevice(pc.info.comm->device);
    r = planColl(pc.info, pc.p, pc.sp, &pc.kind);
    if (r != ncclSuccess) break;
    std::vector<PlannedColl>& run = open[pc.info.comm];
    if (!batchable(run, pc)) r = flush(pc.info.comm);
    if (r == ncclSuccess) run.push_back(pc);
  }
  for (auto& kv : open)
    if (r == ncclSuccess) r = flush(kv.first);
  for (size_t i = 0; i < colls.size() && r == ncclSuccess; i++) r = collJoin(colls[i]);
  (void)hipSetDevice(dev);
  return r;
}

}  // namespace ncclamd

using namespace ncclamd;

NCCL_EXPORT ncclResult_t ncclGroupStart() {
  ROCTX_RANGE("ncclGroupStart");
  return groupStartInternal();
}
extern "C" __attribute__((visibility("default"), alias("ncclGroupStart"))) ncclResult_t pncclGroupStart();

NCCL_EXPORT ncclResult_t ncclGroupEnd() {
  ROCTX_RANGE("ncclGroupEnd");
  return groupEndInternal(nullptr);
}
extern "C" __attribute__((visibility("default"), alias("ncclGroupEnd"))) ncclResult_t pncclGroupEnd();

NCCL_EXPORT ncclResult_t ncclGroupSimulateEnd(ncclSimInfo_t* simInfo) { return groupEndInternal(simInfo); }
extern "C" __attribute__((visibility("default"), alias("ncclGroupSimulateEnd"))) ncclResult_t
pncclGroupSimulateEnd(ncclSimInfo_t*);

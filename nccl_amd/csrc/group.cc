// group.cc — ncclGroupStart / ncclGroupEnd.
//
// Reference: src/include/group.h:81-155 (thread-local group depth), src/group.cc:766-887
// (ncclGroupEndInternal), :598-760 (groupLaunch), :35 (ncclAsyncLaunch of deferred inits).
// Semantics kept: group state is thread-local; calls inside a group are only recorded, and nothing
// is enqueued on any stream until the outermost ncclGroupEnd; communicator inits inside a group run
// concurrently at ncclGroupEnd (required when one thread creates several ranks). Kernel launches here
// never block on peers (all connections are made at init), so one thread may drive every device of
// the node even without a group — the group is still honoured for ordering and error reporting.
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

ncclResult_t groupEndInternal() {
  if (tGroup.depth == 0) {
    WARN("ncclGroupEnd: not in a group call.");
    return ncclInvalidUsage;
  }
  if (--tGroup.depth > 0) return ncclSuccess;
  ncclResult_t ret = tGroup.error;
  std::vector<CollInfo> colls;
  std::vector<std::function<ncclResult_t()>> inits;
  colls.swap(tGroup.colls);
  inits.swap(tGroup.inits);
  tGroup.error = ncclSuccess;
  if (ret != ncclSuccess) return ret;  // a call inside the group failed its checks: launch nothing

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
  int dev = 0;
  (void)hipGetDevice(&dev);
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

NCCL_EXPORT ncclResult_t ncclGroupStart() { return groupStartInternal(); }
extern "C" __attribute__((visibility("default"), alias("ncclGroupStart"))) ncclResult_t pncclGroupStart();

NCCL_EXPORT ncclResult_t ncclGroupEnd() { return groupEndInternal(); }
extern "C" __attribute__((visibility("default"), alias("ncclGroupEnd"))) ncclResult_t pncclGroupEnd();

// kern_u64.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernU64(const LaunchPlan& p) {
  return launchIntOp<uint64_t>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernU64() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<uint64_t, 0, COLL_AR>);
}
ncclResult_t launchSymKernU64(const SymPlan& p) {
  return launchSymIntOp<uint64_t>(p);
}
}  // namespace ncclamd

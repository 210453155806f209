// kern_u32.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernU32(const LaunchPlan& p) {
  return launchIntOp<uint32_t>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernU32() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<uint32_t, 0, COLL_AR>);
}
ncclResult_t launchSymKernU32(const SymPlan& p) {
  return launchSymIntOp<uint32_t>(p);
}
}  // namespace ncclamd

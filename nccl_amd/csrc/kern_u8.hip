// kern_u8.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernU8(const LaunchPlan& p) {
  return launchIntOp<uint8_t>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernU8() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<uint8_t, 0, COLL_AR>);
}
ncclResult_t launchSymKernU8(const SymPlan& p) {
  return launchSymIntOp<uint8_t>(p);
}
}  // namespace ncclamd

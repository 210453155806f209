// kern_f16.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernF16(const LaunchPlan& p) {
  return launchOp<half_t>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernF16() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<half_t, 0, COLL_AR>);
}
ncclResult_t launchSymKernF16(const SymPlan& p) {
  return launchSymOp<half_t>(p);
}
}  // namespace ncclamd

// kern_bf16.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernBF16(const LaunchPlan& p) {
  return launchOp<bf16_t>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernBF16() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<bf16_t, 0, COLL_AR>);
}
ncclResult_t launchSymKernBF16(const SymPlan& p) {
  return launchSymOp<bf16_t>(p);
}
}  // namespace ncclamd

// kern_f32.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernF32(const LaunchPlan& p) {
  return launchOp<float>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernF32() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<float, 0, COLL_AR>);
}
ncclResult_t launchSymKernF32(const SymPlan& p) {
  return launchSymOp<float>(p);
}
}  // namespace ncclamd

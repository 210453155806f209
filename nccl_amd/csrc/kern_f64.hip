// kern_f64.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernF64(const LaunchPlan& p) {
  return launchOp<double>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernF64() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<double, 0, COLL_AR>);
}
ncclResult_t launchSymKernF64(const SymPlan& p) {
  return launchSymOp<double>(p);
}
}  // namespace ncclamd

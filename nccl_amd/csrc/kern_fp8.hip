// kern_fp8.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernFp8(const LaunchPlan& p) {
  return p.datatype == ncclFloat8e4m3 ? launchOp<e4m3_t>(p) : launchOp<e5m2_t>(p);
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernFp8() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<e4m3_t, 0, COLL_AR>);
}
ncclResult_t launchSymKernFp8(const SymPlan& p) {
  return p.datatype == ncclFloat8e4m3 ? launchSymOp<e4m3_t>(p) : launchSymOp<e5m2_t>(p);
}
}  // namespace ncclamd

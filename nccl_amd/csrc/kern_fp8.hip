// kern_fp8.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernFp8(const LaunchPlan& p) {
  return p.datatype == ncclFloat8e4m3 ? launchOp<e4m3_t>(p) : launchOp<e5m2_t>(p);
}
}  // namespace ncclamd

// kern_u32.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernU32(const LaunchPlan& p) {
  return launchIntOp<uint32_t>(p);
}
}  // namespace ncclamd

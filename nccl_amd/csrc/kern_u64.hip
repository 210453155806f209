// kern_u64.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernU64(const LaunchPlan& p) {
  return launchIntOp<uint64_t>(p);
}
}  // namespace ncclamd

// kern_f16.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernF16(const LaunchPlan& p) {
  return launchOp<half_t>(p);
}
}  // namespace ncclamd

// kern_bf16.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernBF16(const LaunchPlan& p) {
  return launchOp<bf16_t>(p);
}
}  // namespace ncclamd

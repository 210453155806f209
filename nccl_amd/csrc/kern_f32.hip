// kern_f32.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernF32(const LaunchPlan& p) {
  return launchOp<float>(p);
}
}  // namespace ncclamd

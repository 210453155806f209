// kern_u8.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernU8(const LaunchPlan& p) {
  return launchIntOp<uint8_t>(p);
}
}  // namespace ncclamd

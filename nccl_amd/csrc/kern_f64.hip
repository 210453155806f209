// kern_f64.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernF64(const LaunchPlan& p) {
  return launchOp<double>(p);
}
}  // namespace ncclamd

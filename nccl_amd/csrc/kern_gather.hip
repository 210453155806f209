// kern_gather.hip — instantiation unit of the collective kernels (kernels.h) for one element type.
#include "kernels.h"
namespace ncclamd {
ncclResult_t launchKernGather(const LaunchPlan& p) {
  switch (p.eltSize) {
    case 1: return launchTyped<uint8_t, 0>(p);
    case 2: return launchTyped<uint16_t, 0>(p);
    case 4: return launchTyped<uint32_t, 0>(p);
    default: return launchTyped<uint64_t, 0>(p);
  }
}
// Force this code object to load now (see warmKernels in kernels.hip).
hipError_t warmKernGather() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, (const void*)&collKernel<uint32_t, 0, COLL_AG>);
}
ncclResult_t launchSymKernGather(const SymPlan& p) {
  switch (p.eltSize) {
    case 1: return launchSymTyped<uint8_t, 0>(p);
    case 2: return launchSymTyped<uint16_t, 0>(p);
    case 4: return launchSymTyped<uint32_t, 0>(p);
    default: return launchSymTyped<uint64_t, 0>(p);
  }
}
}  // namespace ncclamd

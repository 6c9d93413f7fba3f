// k_abd.hip — ABD step kernels (BASELINE config 3).
#define PXS_STEP_INSTANCE
#include "abd_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps abd_step_ops(uint32_t N) {
  switch (N) {
    case 3: return StepInstance<3, AbdProto>::ops();
    case 5: return StepInstance<5, AbdProto>::ops();
    default: return StepInstance<0, AbdProto>::ops();
  }
}
}  // namespace pxs

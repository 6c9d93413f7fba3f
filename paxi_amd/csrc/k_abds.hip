// k_abds.hip — ABD serial step kernels (BASELINE config 3).
#define PXS_STEP_INSTANCE
#include "abd_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps abd_serial_step_ops(uint32_t N) {
  switch (N) {
    case 3: return SerialInstance<3, AbdProto>::ops();
    case 5: return SerialInstance<5, AbdProto>::ops();
    default: return SerialInstance<0, AbdProto>::ops();
  }
}
}  // namespace pxs

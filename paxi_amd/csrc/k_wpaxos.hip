// k_wpaxos.hip — WPaxos step kernel for any N without its own instance.
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxos9_step_ops();
StepOps wpaxos_step_ops(uint32_t N) {
  return N == 9 ? wpaxos9_step_ops() : StepInstance<0, WPaxosProto>::ops();
}
}  // namespace pxs

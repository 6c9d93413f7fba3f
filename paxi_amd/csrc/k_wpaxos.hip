// k_wpaxos.hip — WPaxos step kernel for any N without its own instance, and
// the choice between the instance-scalar layouts (LDS when the tile image
// holds them, else HBM).
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxos9_step_ops();
StepOps wpaxos9l_step_ops();
StepOps wpaxosl_step_ops();
StepOps wpaxos_step_ops(uint32_t N, bool lds) {
  if (N == 9) return lds ? wpaxos9l_step_ops() : wpaxos9_step_ops();
  return lds ? wpaxosl_step_ops() : StepInstance<0, WPaxosProto>::ops();
}
}  // namespace pxs

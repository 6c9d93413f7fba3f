// k_paxos.hip — Multi-Paxos step kernel for any N without its own instance.
#define PXS_STEP_INSTANCE
#include "paxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps paxos3_step_ops();
StepOps paxos5_step_ops();
StepOps paxos9_step_ops();
StepOps paxos_step_ops(uint32_t N) {
  switch (N) {
    case 3: return paxos3_step_ops();
    case 5: return paxos5_step_ops();
    case 9: return paxos9_step_ops();
    default: return StepInstance<0, PaxosProto>::ops();
  }
}
}  // namespace pxs

// k_paxos3.hip — Multi-Paxos step kernel, 3 replicas (BASELINE config 1).
#define PXS_STEP_INSTANCE
#include "paxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps paxos3_step_ops() { return StepInstance<3, PaxosProto>::ops(); }
}  // namespace pxs

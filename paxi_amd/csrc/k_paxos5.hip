// k_paxos5.hip — Multi-Paxos step kernel, 5 replicas (BASELINE config 2).
#define PXS_STEP_INSTANCE
#include "paxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps paxos5_step_ops() { return StepInstance<5, PaxosProto>::ops(); }
}  // namespace pxs

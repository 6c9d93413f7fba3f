// k_paxos9.hip — Multi-Paxos step kernel, 9 replicas (BASELINE config 4: FGrid 3x3).
#define PXS_STEP_INSTANCE
#include "paxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps paxos9_step_ops() { return StepInstance<9, PaxosProto>::ops(); }
}  // namespace pxs

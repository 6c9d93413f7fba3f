// k_wpaxos9.hip — WPaxos step kernel, 3 zones x 3 nodes (BASELINE config 5).
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxos9_step_ops() { return StepInstance<9, WPaxosProto>::ops(); }
}  // namespace pxs

// k_wpaxos9l.hip — WPaxos step kernel, 3 zones x 3 nodes, instance scalars in LDS (BASELINE config 5).
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxos9l_step_ops() { return StepInstance<9, WPaxosProtoL>::ops(); }
}  // namespace pxs

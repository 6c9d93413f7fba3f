// k_wpaxosl.hip — WPaxos step kernel for any N, instance scalars in LDS.
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxosl_step_ops() { return StepInstance<0, WPaxosProtoL>::ops(); }
}  // namespace pxs

// k_wpaxos9s.hip — WPaxos serial step kernel, 3 zones x 3 nodes, instance scalars in the HBM table.
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxos9_serial_step_ops() { return SerialInstance<9, WPaxosProto>::ops(); }
}  // namespace pxs

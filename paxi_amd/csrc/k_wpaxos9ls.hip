// k_wpaxos9ls.hip — WPaxos serial step kernel, 3 zones x 3 nodes, instance scalars in the tile image (BASELINE config 5).
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxos9l_serial_step_ops() { return SerialInstance<9, WPaxosProtoL>::ops(); }
}  // namespace pxs

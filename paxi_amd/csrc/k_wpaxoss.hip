// k_wpaxoss.hip — WPaxos serial step kernels for any N, and the choice among
// the serial instances (instance scalars in the tile image or the HBM table).
#define PXS_STEP_INSTANCE
#include "wpaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps wpaxos9_serial_step_ops();
StepOps wpaxos9l_serial_step_ops();
StepOps wpaxos_serial_step_ops(uint32_t N, bool lds) {
  if (N == 9) return lds ? wpaxos9l_serial_step_ops() : wpaxos9_serial_step_ops();
  return lds ? SerialInstance<0, WPaxosProtoL>::ops() : SerialInstance<0, WPaxosProto>::ops();
}
}  // namespace pxs

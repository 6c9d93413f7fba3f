// k_paxoss.hip — Multi-Paxos serial step kernels: 3 replicas, any other N,
// and the choice among the serial instances.
#define PXS_STEP_INSTANCE
#include "paxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps paxos5_serial_step_ops();
StepOps paxos9_serial_step_ops();
StepOps paxos_serial_step_ops(uint32_t N) {
  switch (N) {
    case 3: return SerialInstance<3, PaxosProto>::ops();
    case 5: return paxos5_serial_step_ops();
    case 9: return paxos9_serial_step_ops();
    default: return SerialInstance<0, PaxosProto>::ops();
  }
}
}  // namespace pxs

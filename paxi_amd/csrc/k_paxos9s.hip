// k_paxos9s.hip — Multi-Paxos serial step kernel, 9 replicas (BASELINE config 4: FGrid 3x3).
#define PXS_STEP_INSTANCE
#include "paxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps paxos9_serial_step_ops() { return SerialInstance<9, PaxosProto>::ops(); }
}  // namespace pxs

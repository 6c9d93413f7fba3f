// k_paxos5s.hip — Multi-Paxos serial step kernel, 5 replicas (BASELINE config 2).
#define PXS_STEP_INSTANCE
#include "paxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps paxos5_serial_step_ops() { return SerialInstance<5, PaxosProto>::ops(); }
}  // namespace pxs

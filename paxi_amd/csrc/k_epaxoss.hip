// k_epaxoss.hip — EPaxos serial step kernel (epaxos_kernel.h), any N <= EP_NMAX.
#define PXS_STEP_INSTANCE
#include "epaxos_kernel.h"
#include "step_ops.h"

namespace pxs {
StepOps epaxos_serial_step_ops(uint32_t) { return SerialInstance<0, EPaxosProto>::ops(); }
}  // namespace pxs

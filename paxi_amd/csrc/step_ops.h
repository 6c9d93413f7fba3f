// step_ops.h — host-side launchers of the step kernel instances.
//
// Each protocol's sim_steps<N, Proto> instances are compiled in their own
// translation unit (k_*.hip) so the library builds in parallel; paxisim.hip
// reaches them only through this table of function pointers.
#pragma once
#include <hip/hip_runtime.h>

#include "paxisim_dev.h"

namespace pxs {

struct StepOps {
  // launch grid = P.C / (64 * P.G) workgroups of P.G*N waves, P.G * P.lds_bytes of LDS
  hipError_t (*launch)(const Params& P, hipStream_t s, uint32_t t0, uint32_t n);
  // set the dynamic-LDS ceiling of the instance on the current device
  hipError_t (*set_lds)(int bytes);
  hipError_t (*occupancy)(const Params& P, int* blocks);
  hipError_t (*attrs)(int* vgprs, int* max_threads);
  bool staged;   // the instance carries the LDS-staged merge loop (sim_core.h stage_built)
  bool serial;   // the serial kernel: one wave per tile plays every replica (sim_core.h sim_serial)
  // serial kernels: K chunks of n steps in one launch (sim_core.h sim_serial_pipe)
  hipError_t (*launch_pipe)(const Params& P, hipStream_t s, uint32_t t0, uint32_t n, uint32_t K, uint32_t* q);
};

// defined in k_paxos*.hip, k_abd.hip, k_wpaxos.hip; nullptr launch = not built
// *_serial_step_ops: the serial kernel of the same protocol and N
StepOps paxos_serial_step_ops(uint32_t N);
StepOps abd_serial_step_ops(uint32_t N);
StepOps wpaxos_serial_step_ops(uint32_t N, bool lds);
StepOps epaxos_serial_step_ops(uint32_t N);
StepOps paxos_step_ops(uint32_t N);
StepOps abd_step_ops(uint32_t N);
StepOps wpaxos_step_ops(uint32_t N, bool lds);   // lds: instance scalars in the tile image (Params::wlds)
StepOps epaxos_step_ops(uint32_t N);

#ifdef PXS_STEP_INSTANCE   // included by a kernel translation unit
template <int NT, class Proto>
struct StepInstance {
  static hipError_t launch(const Params& P, hipStream_t s, uint32_t t0, uint32_t n) {
    const unsigned grid = (unsigned)(P.C / (LANES * P.G));
    sim_steps<NT, Proto><<<grid, P.G * P.N * LANES, (size_t)P.G * P.lds_bytes, s>>>(P, t0, n);
    return hipGetLastError();
  }
  // The ceiling is set to what the launch uses, not to the CU's 160 KB: the
  // runtime sizes every workgroup's LDS allocation by it, and a 160 KB ceiling
  // would hold each CU to one resident workgroup.
  static hipError_t set_lds(int bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&sim_steps<NT, Proto>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  }
  static hipError_t occupancy(const Params& P, int* blocks) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, reinterpret_cast<const void*>(&sim_steps<NT, Proto>),
                                                        (int)(P.G * P.N * LANES), (size_t)P.G * P.lds_bytes);
  }
  static hipError_t attrs(int* v, int* maxthr) {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&sim_steps<NT, Proto>));
    if (e == hipSuccess) {
      *v = a.numRegs;
      *maxthr = a.maxThreadsPerBlock;
    }
    return e;
  }
  static StepOps ops() { return StepOps{&launch, &set_lds, &occupancy, &attrs, stage_built<NT, Proto>()}; }
};

// The serial kernel (sim_core.h sim_serial): one wave per tile, P.G = 1,
// P.lds_bytes of LDS per workgroup.
template <int NT, class Proto>
struct SerialInstance {
  static hipError_t launch(const Params& P, hipStream_t s, uint32_t t0, uint32_t n) {
    sim_serial<NT, Proto><<<(unsigned)(P.C / LANES), LANES, (size_t)P.lds_bytes, s>>>(P, t0, n);
    return hipGetLastError();
  }
  static hipError_t occupancy(const Params& P, int* blocks) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, reinterpret_cast<const void*>(&sim_serial<NT, Proto>),
                                                        (int)LANES, (size_t)P.lds_bytes);
  }
  static hipError_t attrs(int* v, int* maxthr) {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&sim_serial<NT, Proto>));
    if (e == hipSuccess) {
      *v = a.numRegs;
      *maxthr = a.maxThreadsPerBlock;
    }
    return e;
  }
  static hipError_t launch_pipe(const Params& P, hipStream_t s, uint32_t t0, uint32_t n, uint32_t K, uint32_t* q) {
    unsigned g = (((unsigned)(P.C / LANES) + 7u) / 8u) * 8u * K;   // one ticket per workgroup
    if (PXS_PIPE_PERSIST) {   // the persistent form: the resident slots, a multiple of 8 (sim_core.h)
      int dev = 0, cus = 0, per = 0;
      hipError_t e = hipGetDevice(&dev);
      if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (e == hipSuccess) e = occupancy(P, &per);
      if (e != hipSuccess) return e;
      const unsigned slots = ((unsigned)(cus * per) + 7u) / 8u * 8u;
      if (slots && slots < g) g = slots;
    }
    sim_serial_pipe<NT, Proto><<<g, LANES, (size_t)P.lds_bytes, s>>>(P, t0, n, K, q);
    return hipGetLastError();
  }
  static hipError_t set_lds(int bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sim_serial<NT, Proto>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sim_serial_pipe<NT, Proto>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    return e;
  }
  static StepOps ops() { return StepOps{&launch, &set_lds, &occupancy, &attrs, false, true, &launch_pipe}; }
};
#endif

}  // namespace pxs

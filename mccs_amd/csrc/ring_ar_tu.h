// ring_ar_tu.h — the ten AllReduce kernels of ONE reduction op: the
// reference-named entry points (collectives.h:43-49, common.h:182-188) and the
// library's multi-rank launch, instantiated in their own translation unit
// (ring_ar_<op>.hip) so the four ops compile in parallel.
#pragma once
#include "ring_kernel.h"

#define MCCS_AR_KERNEL(OPN, OPV, TN, DT)                                                               \
  extern "C" __global__ void __launch_bounds__(MCCS_RING_MAX_THREADS)                                  \
      mccsKernel_AllReduce_RING_SIMPLE_##OPN##_##TN(mccsDevComm* comm, uint64_t channelMask,           \
                                                    mccsDevWork* workHead) {                           \
    mccs::ring_kernel_body<mccsFuncAllReduce, DT, OPV, mccs::kRefUnroll<DT>>(comm, channelMask, workHead,  \
                                                                             blockIdx.x, gridDim.x,       \
                                                                             mccs::kRefCfg);              \
  }

#define MCCS_AR_CASE(OPN, OPV, TN, DT)                                                                       \
  case DT:                                                                                                   \
    return multi ? (const void*)&ring_multi_kernel<mccsFuncAllReduce, DT, OPV>                             \
                 : (const void*)&mccsKernel_AllReduce_RING_SIMPLE_##OPN##_##TN;

#define MCCS_AR_TYPES(X, OPN, OPV)                                                                  \
  X(OPN, OPV, int8_t, mccsInt8) X(OPN, OPV, uint8_t, mccsUint8) X(OPN, OPV, int32_t, mccsInt32)    \
  X(OPN, OPV, uint32_t, mccsUint32) X(OPN, OPV, int64_t, mccsInt64) X(OPN, OPV, uint64_t, mccsUint64) \
  X(OPN, OPV, half, mccsFloat16) X(OPN, OPV, float, mccsFloat32) X(OPN, OPV, double, mccsFloat64)  \
  X(OPN, OPV, bfloat16, mccsBfloat16)

// Defines the kernels and mccs::ring_ar_kernel_<OPN>(dtype, multi).
#define MCCS_AR_TU(OPN, OPV)                                     \
  MCCS_AR_TYPES(MCCS_AR_KERNEL, OPN, OPV)                        \
  namespace mccs {                                               \
  const void* ring_ar_kernel_##OPN(int dtype, bool multi) {      \
    switch (dtype) { MCCS_AR_TYPES(MCCS_AR_CASE, OPN, OPV) }     \
    return nullptr;                                              \
  }                                                              \
  }

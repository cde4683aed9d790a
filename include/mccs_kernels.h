/*
 * mccs_kernels.h — the reference-named ring kernels exported by libmccs_hip.so.
 *
 * Mirrors src/collectives/include/collectives.h:43-49 (DECL_KERNEL /
 * DECL_ALL_KERNELS) so the reference's bindgen allowlist "^mccsKernel.*"
 * (src/collectives-sys/build.rs:31) finds them.  For C / Rust callers each
 * name is the host handle that hipLaunchKernel takes (what plan.rs:142-166
 * stores as KernelPlan.kernel_fn); arguments are (comm, channelMask, workHead)
 * exactly as plan.rs:641-646 passes them.  Not for inclusion in HIP device
 * code (ring.hip defines these as extern "C" __global__).
 *
 * Reference linkage.  The reference declares the kernels with C++ linkage
 * (collectives.h:49 has no extern "C"; collectives-sys/build.rs runs bindgen
 * with "-x c++", so Rust binds the Itanium-mangled names) and names the bf16
 * kernels after CUDA's type (..._<Op>___nv_bfloat16, common.h:182-188).  The
 * library therefore also exports, at the same addresses:
 *   _Z<len><name>P11mccsDevCommmP11mccsDevWork   for every name below, and
 *   mccsKernel_AllReduce_RING_SIMPLE_<Op>___nv_bfloat16 (+ its mangled form)
 * (link-time aliases, mccs_amd/build.py reference_aliases), so the
 * reference's wrapper.h / collectives.h link against libmccs_hip.so as is.
 */
#ifndef MCCS_AMD_KERNELS_H_
#define MCCS_AMD_KERNELS_H_

#include <stdint.h>

#include "mccs_devcomm.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MCCS_KERNEL_SYMBOL(name) \
  void name(struct mccsDevComm *comm, uint64_t channelMask, struct mccsDevWork *workHead)

MCCS_KERNEL_SYMBOL(mccsKernel_AllGather_RING_SIMPLE_Sum_int8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_int8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_uint8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_int32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_uint32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_int64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_uint64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_half);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_float);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_double);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum_bfloat16);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_int8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_uint8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_int32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_uint32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_int64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_uint64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_half);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_float);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_double);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod_bfloat16);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_int8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_uint8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_int32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_uint32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_int64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_uint64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_half);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_float);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_double);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max_bfloat16);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_int8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_uint8_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_int32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_uint32_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_int64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_uint64_t);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_half);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_float);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_double);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min_bfloat16);
/* the reference's bf16 spelling (same handles as the ..._bfloat16 ones) */
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Sum___nv_bfloat16);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Prod___nv_bfloat16);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Max___nv_bfloat16);
MCCS_KERNEL_SYMBOL(mccsKernel_AllReduce_RING_SIMPLE_Min___nv_bfloat16);

#ifdef __cplusplus
}
#endif

#endif /* MCCS_AMD_KERNELS_H_ */

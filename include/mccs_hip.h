/*
 * mccs_hip.h — C-ABI of libmccs_hip.so, the MI355X-native mCCS allreduce path.
 *
 * Plain C: pointers, sizes, ints and opaque handles only (no torch, no HIP C++
 * types beyond the hipStream_t / hipEvent_t handles, which are pointers).
 * Each entry point names the reference interface it replaces.
 */
#ifndef MCCS_AMD_HIP_H_
#define MCCS_AMD_HIP_H_

#include <stddef.h>
#include <stdint.h>

#include "mccs_devcomm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* hipStream_t / hipEvent_t are opaque pointers in the HIP C API. */
#ifndef __HIP_PLATFORM_AMD__
typedef struct ihipStream_t *hipStream_t;
#endif

/* Result codes (NCCL/mCCS convention; the reference surfaces errors as
 * Result<(), Error> in libmccs and logs CUDA errors via cuda_warning!). */
typedef enum {
  mccsSuccess = 0,
  mccsUnhandledCudaError = 1, /* a HIP runtime call failed */
  mccsSystemError = 2,
  mccsInternalError = 3,
  mccsInvalidArgument = 4,
  mccsInvalidUsage = 5,
  mccsRemoteError = 6,
  mccsInProgress = 7,
  mccsTimeout = 8, /* a FIFO spin exceeded the watchdog; abortFlag raised */
  mccsNumResults = 9
} mccsResult_t;

/* ======================================================================
 * Device-resident chunk reduce (north-star kernel; BASELINE config 2).
 * Replaces the reduce/reduce-copy loop of the reference ring kernel,
 * ReduceOrCopyMulti (src/collectives/src/common_kernel.h:624-685), as a
 * standalone full-chip launch: y = src[0] (op) src[1] (op) ... in the element
 * type, written to every dst.  dst may alias src[0] (in-place a += b).
 * dtype: mccsDevDataType_t; op: mccsDevSum/Prod/Max/Min.
 * ====================================================================== */
#define MCCS_REDUCE_MAX_SRCS 8
#define MCCS_REDUCE_MAX_DSTS 4
#define MCCS_REDUCE_VARIANT_REG 1 /* register streaming main loop */
#define MCCS_REDUCE_VARIANT_LDS 2 /* LDS-DMA multi-stage staging main loop */

mccsResult_t mccs_hip_reduce(void *dst, const void *const *srcs, int nsrcs, size_t count, int dtype,
                             int op, hipStream_t stream);
mccsResult_t mccs_hip_reduce_copy(void *const *dsts, int ndsts, const void *const *srcs, int nsrcs,
                                  size_t count, int dtype, int op, hipStream_t stream);
/* Select the main loop (0 = default), unroll = KiB per source per wave tile
 * for LDS / 16-byte packs per lane for REG (1/2/4/8, 0 = default), cache
 * policy (0 plain, 1 non-temporal, -1 default), persistent blocks per CU,
 * LDS ring stages (2..4) and waves per block (4/8); 0 = default for each.
 * Process-wide; for benchmarking and tests. */
mccsResult_t mccs_hip_reduce_tune(int variant, int unroll, int policy, int blocks_per_cu, int stages,
                                  int waves);
void mccs_hip_reduce_get_tune(int *variant, int *unroll, int *policy, int *blocks_per_cu, int *stages,
                              int *waves);

/* Library identification. */
const char *mccs_hip_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MCCS_AMD_HIP_H_ */

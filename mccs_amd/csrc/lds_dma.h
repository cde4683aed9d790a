// lds_dma.h — LDS-DMA (global_load_lds_dwordx4) and counted vmcnt waits for
// gfx950, shared by the full-chip chunk reduce (reduce.hip) and the ring's
// per-workgroup stream (ring_kernel.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "reduce_copy.h"

namespace mccs {

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One lane's 16 bytes of a wave-wide LDS-DMA: LDS dst = M0 + lane*16.
// NT: non-temporal (streaming) policy on the DMA read.
template <int POL>
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_wave_base) {
  uint32_t keep;
#define MCCS_GLDS(MODS)                                                   \
  asm volatile(                                                           \
      "s_mov_b32 %0, m0\n\t"                                              \
      "s_mov_b32 m0, %2\n\t"                                              \
      "s_nop 0\n\t"                                                       \
      "global_load_lds_dwordx4 %1, off " MODS "\n\t"                      \
      "s_mov_b32 m0, %0"                                                  \
      : "=&s"(keep)                                                       \
      : "v"(gsrc), "s"(lds_wave_base)                                     \
      : "memory")
  if constexpr (POL == kNonTemporal) MCCS_GLDS("nt");
  else if constexpr (POL == kNtWriteThrough) MCCS_GLDS("sc1 nt");
  else if constexpr (POL == kSystemNt) MCCS_GLDS("sc0 sc1 nt");
  else MCCS_GLDS("");
#undef MCCS_GLDS
}

}  // namespace mccs

// ring_stream.h — the ring's per-slice stream: dynamic wave units.
//
// A ring slice is cut into wave units of U KiB per source; the data waves of
// the workgroup take units from an LDS counter (reduce_copy_rows_dyn), so
// waves that a SIMD issues at different rates still finish a slice together.
// Same operands and element semantics as reduce_copy_rows (ReduceOrCopyMulti,
// reference common_kernel.h:485-685): v = src0 (op) src1, stored to every
// destination; 16-byte aligned operands (else the typed fallback); typed
// scalar tail past the last whole pack.  (The register double buffer and the
// LDS-DMA ring measured against it live beside their one user,
// tools/wg_stream_rows.h.)
#pragma once
#include <type_traits>

#include "dtypes.h"
#include "reduce_copy.h"

namespace mccs {

// A wave-uniform pointer the compiler cannot prove uniform, moved to SGPRs
// (loads and stores then address saddr + a 32-bit lane offset).  The value
// is rebuilt as a GLOBAL-address-space pointer and only then converted to a
// generic one, so the compiler still sees global memory behind it: rebuilt
// from an integer as a generic pointer it became flat_load / flat_store,
// which count in lgkmcnt as well as vmcnt, so every LDS wait (a dynamic
// unit's grab, the count-out) also waited for all of the wave's memory
// operations in flight (gfx950 assembly of the ring kernels; one workgroup
// streamed 58-63 GB/s that way against 75-89 with global operations).
// Every operand behind it is global memory: device HBM, a peer's HBM or
// host memory mapped for the device; never LDS or scratch.
template <typename P>
__device__ __forceinline__ P uniform_ptr(P p) {
  using E = std::remove_pointer_t<P>;
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  auto* g = (__attribute__((address_space(1))) E*)(((uint64_t)hi << 32) | lo);
  return (P)g;
}

// Dynamic work within a slice.  reduce_copy_rows gives every wave the same
// rows, but waves of one CU stream at very different rates (a slice timeline
// at the reference launch shape: waves of one workgroup took 24-48 us to
// issue the same bytes), and a wave may count itself out of slice t only
// after every wave left t-1, so the fast ones idled at the count-out (the
// ring profile's "drain": 12 of 41 us per slice).  Here a slice is cut into
// wave units of U KiB per source (64 lanes x U packs) and each wave takes the
// next unit from a workgroup counter in LDS until none is left, so the waves
// finish a slice within one unit of each other.
//   ctr   LDS counter shared by the workgroup's data waves for this slice's
//         parity (slices t and t+1 use different counters: waves drift up to
//         one slice apart, and a wave starts t+2 only after every wave left t)
//   base  the counter's value when this slice's grabbing began, which every
//         wave derives alike (the previous slice of this parity advanced it
//         by its units + one failing grab per wave)
// Returns how far this slice advances the counter (0 if no unit was taken:
// an empty slice, or an unaligned one, which takes the typed loop; every wave
// of the workgroup decides alike).  Same operands and results as
// reduce_copy_rows.
template <int DT, int OP, int U, int NS, int ND, int NTMASK, int DP0 = kPlain, int DP1 = kPlain>
__device__ __forceinline__ uint32_t reduce_copy_rows_dyn(const void* s0, const void* s1, void* d0, void* d1,
                                                         int64_t nelem, int tid, int nthr, uint32_t* ctr,
                                                         uint32_t base) {
  constexpr int PACK = kPackElems<DT>;
  constexpr int LP0 = (NTMASK & 1) ? kNonTemporal : kPlain;
  constexpr int LP1 = (NTMASK & 2) ? kNonTemporal : kPlain;
  using T = typename Elem<DT>::T;
  if (nelem <= 0) return 0;
  uintptr_t mis = (uintptr_t)s0 | (uintptr_t)d0;
  if constexpr (NS > 1) mis |= (uintptr_t)s1;
  if constexpr (ND > 1) mis |= (uintptr_t)d1;
  if (mis & 15) {  // unaligned: typed loop over every data thread (reference ReduceCopyMulti)
    for (int64_t e = tid; e < nelem; e += nthr) {
      T v = (NTMASK & 1) ? __builtin_nontemporal_load((const T*)s0 + e) : ((const T*)s0)[e];
      if constexpr (NS > 1)
        v = scalar_op<DT, OP>(v, (NTMASK & 2) ? __builtin_nontemporal_load((const T*)s1 + e) : ((const T*)s1)[e]);
      ((T*)d0)[e] = v;
      if constexpr (ND > 1) ((T*)d1)[e] = v;
    }
    return 0;
  }
  const uint32_t nwaves = (uint32_t)nthr >> 6;
  const uint32_t npack = (uint32_t)(nelem / PACK);
  const uint32_t lane = (uint32_t)tid & 63;
  const u32x4* a = (const u32x4*)s0;
  const u32x4* b = (const u32x4*)s1;
  u32x4* x = (u32x4*)d0;
  u32x4* y = (u32x4*)d1;
  const uint32_t unit = 64u * U;
  const uint32_t nunits = npack / unit;  // whole units; the rest below, by every wave
  uint32_t g = 0;
#pragma unroll 1
  for (;;) {
    if (lane == 0) g = atomicAdd(ctr, 1u);
    const uint32_t k = __builtin_amdgcn_readfirstlane(g) - base;
    if (k >= nunits) break;
    // the unit's bases are uniform: saddr + lane offset addressing
    const size_t ko = (size_t)k * unit;
    const u32x4* ak = uniform_ptr(a + ko);
    const u32x4* bk = NS > 1 ? uniform_ptr(b + ko) : nullptr;
    u32x4* xk = uniform_ptr(x + ko);
    u32x4* yk = ND > 1 ? uniform_ptr(y + ko) : nullptr;
    u32x4 v[U], w[NS > 1 ? U : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<LP0>(ak + lane + 64u * u);
    if constexpr (NS > 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = ld16<LP1>(bk + lane + 64u * u);
    }
    // every load of the unit is issued before the first use (the scheduler
    // would otherwise interleave waits to save registers: fewer bytes in flight)
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NS > 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = pack_op<DT, OP>(v[u], w[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st16<DP0>(xk + lane + 64u * u, v[u]);
    if constexpr (ND > 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) st16<DP1>(yk + lane + 64u * u, v[u]);
    }
  }
  // the packs past the last whole unit (< one unit) and the typed tail (< one
  // pack), over every data thread
  for (uint32_t q = nunits * unit + (uint32_t)tid; q < npack; q += (uint32_t)nthr) {
    u32x4 v = ld16<LP0>(a + q);
    if constexpr (NS > 1) v = pack_op<DT, OP>(v, ld16<LP1>(b + q));
    st16<DP0>(x + q, v);
    if constexpr (ND > 1) st16<DP1>(y + q, v);
  }
  for (int64_t e = (int64_t)npack * PACK + tid; e < nelem; e += nthr) {
    T v = (NTMASK & 1) ? __builtin_nontemporal_load((const T*)s0 + e) : ((const T*)s0)[e];
    if constexpr (NS > 1)
      v = scalar_op<DT, OP>(v, (NTMASK & 2) ? __builtin_nontemporal_load((const T*)s1 + e) : ((const T*)s1)[e]);
    ((T*)d0)[e] = v;
    if constexpr (ND > 1) ((T*)d1)[e] = v;
  }
  return nunits + nwaves;
}

}  // namespace mccs

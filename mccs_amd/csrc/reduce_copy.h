// reduce_copy.h — the chunk reduce / reduce-copy inner loops for gfx950.
//
// Restates ReduceOrCopyMulti (reference src/collectives/src/common_kernel.h:485-685):
//   vals = src[0]; vals = fn(vals, src[i]) for i >= 1; vals stored to every dst.
// but shaped for CDNA4: 64-lane waves, 16-byte global_load_dwordx4 per lane,
// U packs in flight per source per lane, packed VALU ops (dtypes.h), and no
// 32-lane warp arithmetic.  Tails (< 16 bytes) and unaligned buffers fall back
// to a typed scalar loop, like the reference's ReduceCopyMulti fallback.
#pragma once
#include "dtypes.h"

namespace mccs {

// Cache policy for a stream of 16-byte accesses.
enum Policy : int { kPlain = 0, kNonTemporal = 1 };

template <int POL>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (POL == kNonTemporal) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int POL>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (POL == kNonTemporal) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Block-cooperative reduce-copy of nelem elements, srcs/dsts already offset.
// Runtime nsrcs in [1, MAXS], ndsts in [1, MAXD]. Threads [tid, nthr) of the
// calling group participate. Used by the ring primitives (one workgroup per
// channel lane) where nsrcs/ndsts vary per primitive call.
// NTMASK: bit s set -> source s is read with non-temporal loads, which bypass
// the CU's L1 (used for FIFO slots another workgroup rewrites between reads).
template <int DT, int OP, int U, int MAXS, int MAXD, int LDPOL = kPlain, int STPOL = kPlain, int NTMASK = 0>
__device__ __forceinline__ void reduce_copy_group(const void* const* srcs, int nsrcs,
                                                  void* const* dsts, int ndsts, int64_t nelem,
                                                  int tid, int nthr) {
  using T = typename Elem<DT>::T;
  constexpr int PACK = kPackElems<DT>;
  if (nelem <= 0) return;
  uintptr_t mis = 0;
#pragma unroll
  for (int s = 0; s < MAXS; ++s)
    if (s < nsrcs) mis |= (uintptr_t)srcs[s];
#pragma unroll
  for (int d = 0; d < MAXD; ++d)
    if (d < ndsts) mis |= (uintptr_t)dsts[d];
  int64_t done = 0;
  if ((mis & 15) == 0) {
    const int64_t npack = nelem / PACK;
    const int64_t step = (int64_t)nthr * U;
    int64_t p = tid;
    // full U-deep iterations: no bounds checks inside
    for (; p + (int64_t)(U - 1) * nthr < npack; p += step) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = ld16<(NTMASK & 1) ? kNonTemporal : LDPOL>((const u32x4*)srcs[0] + p + (int64_t)u * nthr);
#pragma unroll
      for (int s = 1; s < MAXS; ++s) {
        if (s < nsrcs) {
          u32x4 w[U];
#pragma unroll
          for (int u = 0; u < U; ++u)
            w[u] = ((NTMASK >> s) & 1) ? ld16<kNonTemporal>((const u32x4*)srcs[s] + p + (int64_t)u * nthr)
                                       : ld16<LDPOL>((const u32x4*)srcs[s] + p + (int64_t)u * nthr);
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = pack_op<DT, OP>(v[u], w[u]);
        }
      }
#pragma unroll
      for (int d = 0; d < MAXD; ++d) {
        if (d < ndsts) {
#pragma unroll
          for (int u = 0; u < U; ++u) st16<STPOL>((u32x4*)dsts[d] + p + (int64_t)u * nthr, v[u]);
        }
      }
    }
    // remainder packs, one at a time
    for (; p < npack; p += nthr) {
      u32x4 v = ld16<(NTMASK & 1) ? kNonTemporal : LDPOL>((const u32x4*)srcs[0] + p);
#pragma unroll
      for (int s = 1; s < MAXS; ++s)
        if (s < nsrcs)
          v = pack_op<DT, OP>(v, ((NTMASK >> s) & 1) ? ld16<kNonTemporal>((const u32x4*)srcs[s] + p)
                                                     : ld16<LDPOL>((const u32x4*)srcs[s] + p));
#pragma unroll
      for (int d = 0; d < MAXD; ++d)
        if (d < ndsts) st16<STPOL>((u32x4*)dsts[d] + p, v);
    }
    done = npack * PACK;
  }
  // typed scalar tail / unaligned fallback
  for (int64_t e = done + tid; e < nelem; e += nthr) {
    T v = (NTMASK & 1) ? __builtin_nontemporal_load((const T*)srcs[0] + e) : ((const T*)srcs[0])[e];
#pragma unroll
    for (int s = 1; s < MAXS; ++s)
      if (s < nsrcs)
        v = scalar_op<DT, OP>(v, ((NTMASK >> s) & 1) ? __builtin_nontemporal_load((const T*)srcs[s] + e)
                                                     : ((const T*)srcs[s])[e]);
#pragma unroll
    for (int d = 0; d < MAXD; ++d)
      if (d < ndsts) ((T*)dsts[d])[e] = v;
  }
}

}  // namespace mccs

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

// Cache policy for a stream of 16-byte accesses.  The write-through forms
// (sc1: the store goes through this XCD's L2 to memory instead of staying
// dirty there until the end-of-kernel writeback) are store-only.
enum Policy : int { kPlain = 0, kNonTemporal = 1, kNtWriteThrough = 2, kWriteThrough = 3, kSystemNt = 4 };

template <int POL>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (POL == kNonTemporal) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int POL>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (POL == kNonTemporal) __builtin_nontemporal_store(v, p);
  else if constexpr (POL == kNtWriteThrough)
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == kWriteThrough)
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == kSystemNt)
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  else *p = v;
}

// Ring-step reduce-copy with the operand shape fixed at compile time (the
// ring primitive knows it: NS sources, ND destinations) and a wave-contiguous
// layout: wave w of the group owns U consecutive 1 KiB rows of each U*W KiB
// iteration, lane l reads 16 bytes at row offset 16*l, so every load/store
// instruction moves 1 KiB contiguous and the U rows of a wave sit at constant
// 1 KiB strides from one 32-bit per-lane offset (uniform 64-bit bases stay in
// SGPRs; no per-pack 64-bit address registers).  All U x NS loads of an
// iteration are issued before the first use; the partial last iteration is a
// single predicated pass.  Every pointer must be 16-byte aligned when
// ALIGNED; otherwise a typed element loop runs (reference ReduceCopyMulti).
// DP0 / DP1: store policy of destination 0 / 1.
template <int DT, int OP, int U, int NS, int ND, int NTMASK, int DP0 = kPlain, int DP1 = kPlain>
__device__ __forceinline__ void reduce_copy_rows(const void* s0, const void* s1, void* d0, void* d1, int64_t nelem,
                                                 int tid, int nthr) {
  static_assert(NS >= 1 && NS <= 2 && ND >= 1 && ND <= 2, "ring primitives move 1-2 sources to 1-2 destinations");
  using T = typename Elem<DT>::T;
  constexpr int PACK = kPackElems<DT>;
  if (nelem <= 0) return;
  uintptr_t mis = (uintptr_t)s0 | (uintptr_t)d0;
  if constexpr (NS > 1) mis |= (uintptr_t)s1;
  if constexpr (ND > 1) mis |= (uintptr_t)d1;
  int64_t done = 0;
  if ((mis & 15) == 0) {
    const u32x4* a = (const u32x4*)s0;
    const u32x4* b = (const u32x4*)s1;
    u32x4* x = (u32x4*)d0;
    u32x4* y = (u32x4*)d1;
    const uint32_t npack = (uint32_t)(nelem / PACK);
    const uint32_t wave = (uint32_t)tid >> 6, lane = (uint32_t)tid & 63;
    // rows need whole waves: a partial last wave (e.g. the reference's 544 =
    // 8.5 x 64 threads) sits out the vector loop and joins the scalar tail
    const uint32_t nwaves = (uint32_t)nthr >> 6;
    const uint32_t per_iter = nwaves * 64u * U;     // packs
    const uint32_t mine = wave * (64u * U) + lane;  // first pack of this lane in an iteration
    uint32_t base = wave < nwaves ? 0u : npack;  // npack: skip both vector passes
    for (; wave < nwaves && base + per_iter <= npack; base += per_iter) {
      const uint32_t q = base + mine;
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld16<(NTMASK & 1) ? kNonTemporal : kPlain>(a + q + 64u * u);
      if constexpr (NS > 1) {
        u32x4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = ld16<(NTMASK & 2) ? kNonTemporal : kPlain>(b + q + 64u * u);
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = pack_op<DT, OP>(v[u], w[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) st16<DP0>(x + q + 64u * u, v[u]);
      if constexpr (ND > 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) st16<DP1>(y + q + 64u * u, v[u]);
      }
    }
    if (base < npack) {  // partial iteration: same layout, predicated
      const uint32_t q = base + mine;
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (q + 64u * u < npack) v[u] = ld16<(NTMASK & 1) ? kNonTemporal : kPlain>(a + q + 64u * u);
      if constexpr (NS > 1) {
        u32x4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (q + 64u * u < npack) w[u] = ld16<(NTMASK & 2) ? kNonTemporal : kPlain>(b + q + 64u * u);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (q + 64u * u < npack) v[u] = pack_op<DT, OP>(v[u], w[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (q + 64u * u < npack) {
          st16<DP0>(x + q + 64u * u, v[u]);
          if constexpr (ND > 1) st16<DP1>(y + q + 64u * u, v[u]);
        }
    }
    done = (int64_t)npack * PACK;
  }
  // typed scalar tail / unaligned fallback
  for (int64_t e = done + tid; e < nelem; e += nthr) {
    T v = (NTMASK & 1) ? __builtin_nontemporal_load((const T*)s0 + e) : ((const T*)s0)[e];
    if constexpr (NS > 1)
      v = scalar_op<DT, OP>(v, (NTMASK & 2) ? __builtin_nontemporal_load((const T*)s1 + e) : ((const T*)s1)[e]);
    ((T*)d0)[e] = v;
    if constexpr (ND > 1) ((T*)d1)[e] = v;
  }
}

}  // namespace mccs

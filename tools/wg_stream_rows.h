// wg_stream_rows.h — the two per-workgroup slice streams tools/wg_stream.hip
// measures against the ring's dynamic wave units (ring_stream.h), kept here
// beside their one user (no A/B-only code in the shipped
// kernel headers).
// reduce_copy_rows (reduce_copy.h) keeps U packs per source per lane in
// flight only while a pass is loading: a wave loads, waits, reduces, stores,
// and only then issues the next pass.  These two loops keep the next tile
// loading while the current one is reduced and stored:
//   reduce_copy_rows_pp  register double buffer (two passes of U packs)
//   lds_stream_rows      per-wave LDS-DMA ring (global_load_lds_dwordx4):
//                        S stages of U KiB per source, S-1 tiles in flight,
//                        counted vmcnt waits; no VGPRs hold loads in flight
#pragma once
#include <utility>

#include "dtypes.h"
#include "lds_dma.h"
#include "reduce_copy.h"

namespace mccs {

// Register double buffer.  Full passes alternate between two register sets
// so the loads of pass p+1 are in flight while pass p is reduced and stored;
// the partial last pass and the tail go through reduce_copy_rows.
template <int DT, int OP, int U, int NS, int ND, int NTMASK, int DP0 = kPlain, int DP1 = kPlain>
__device__ __forceinline__ void reduce_copy_rows_pp(const void* s0, const void* s1, void* d0, void* d1, int64_t nelem,
                                                    int tid, int nthr) {
  constexpr int PACK = kPackElems<DT>;
  constexpr int LP0 = (NTMASK & 1) ? kNonTemporal : kPlain;
  constexpr int LP1 = (NTMASK & 2) ? kNonTemporal : kPlain;
  if (nelem <= 0) return;
  uintptr_t mis = (uintptr_t)s0 | (uintptr_t)d0;
  if constexpr (NS > 1) mis |= (uintptr_t)s1;
  if constexpr (ND > 1) mis |= (uintptr_t)d1;
  const uint32_t nwaves = (uint32_t)nthr >> 6;
  const uint32_t wave = (uint32_t)tid >> 6, lane = (uint32_t)tid & 63;
  int64_t done = 0;
  if ((mis & 15) == 0 && wave < nwaves) {
    const u32x4* a = (const u32x4*)s0;
    const u32x4* b = (const u32x4*)s1;
    u32x4* x = (u32x4*)d0;
    u32x4* y = (u32x4*)d1;
    const uint32_t npack = (uint32_t)(nelem / PACK);
    const uint32_t per_iter = nwaves * 64u * U;
    const uint32_t nfull = npack / per_iter;
    const uint32_t mine = wave * (64u * U) + lane;
    u32x4 va[U], wa[U], vb[U], wb[U];
    auto load = [&](uint32_t p, u32x4(&v)[U], u32x4(&w)[U]) {
      const uint32_t q = p * per_iter + mine;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld16<LP0>(a + q + 64u * u);
      if constexpr (NS > 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = ld16<LP1>(b + q + 64u * u);
      }
    };
    auto finish = [&](uint32_t p, u32x4(&v)[U], u32x4(&w)[U]) {
      const uint32_t q = p * per_iter + mine;
      if constexpr (NS > 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = pack_op<DT, OP>(v[u], w[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) st16<DP0>(x + q + 64u * u, v[u]);
      if constexpr (ND > 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) st16<DP1>(y + q + 64u * u, v[u]);
      }
    };
    if (nfull > 0) load(0, va, wa);
#pragma unroll 1
    for (uint32_t p = 0; p < nfull; p += 2) {
      if (p + 1 < nfull) load(p + 1, vb, wb);
      finish(p, va, wa);
      if (p + 1 < nfull) {
        if (p + 2 < nfull) load(p + 2, va, wa);
        finish(p + 1, vb, wb);
      }
    }
    done = (int64_t)nfull * per_iter * PACK;
  }
  using T = typename Elem<DT>::T;
  // the partial pass, the scalar tail (and an unaligned slice) as before
  reduce_copy_rows<DT, OP, U, NS, ND, NTMASK, DP0, DP1>((const T*)s0 + done, NS > 1 ? (const T*)s1 + done : nullptr,
                                                       (T*)d0 + done, ND > 1 ? (T*)d1 + done : nullptr, nelem - done,
                                                       tid, nthr);
}

// s_waitcnt vmcnt(nd * G + ns * SD) with nd, ns < S chosen at run time
// (vmcnt takes an immediate): one uniform compare per candidate.
template <int G, int SD, int S, int... I>
__device__ __forceinline__ void wait_younger_impl(int idx, std::integer_sequence<int, I...>) {
  static_assert((S - 1) * (G + SD) < 64, "vmcnt range");
  bool hit = false;
  ((hit = hit || (idx == I ? (wait_vmcnt<(I / S) * G + (I % S) * SD>(), true) : false)), ...);
  if (!hit) wait_vmcnt<0>();
}
template <int G, int SD, int S>
__device__ __forceinline__ void wait_younger_ops(int nd, int ns) {
  wait_younger_impl<G, SD, S>(nd * S + ns, std::make_integer_sequence<int, S * S>{});
}

// LDS-DMA ring per wave.  The slice's packs are cut into tiles of U KiB per
// source (64 lanes x U packs); wave w takes tiles w, w + W, ...  A tile's
// sources land in the wave's stage (k mod S) of lds_wave_base (S x NS x U KiB
// per wave) by global_load_lds_dwordx4; tile k is read back with ds_read_b128
// once vmcnt says it landed (everything younger than its DMA: the DMA of the
// tiles after it and the stores of the tiles before it), reduced and stored
// while tiles k+1 .. k+S-1 are loading.  Lanes past the end of the last tile
// load and store the slice's last pack again (same bytes, same value), so
// every tile issues the same number of operations and the counts stay exact.
template <int DT, int OP, int U, int S, int NS, int ND, int NTMASK, int DP0 = kPlain, int DP1 = kPlain>
__device__ __forceinline__ void lds_stream_rows(const void* s0, const void* s1, void* d0, void* d1, int64_t nelem,
                                                int tid, int nthr, uint32_t lds_wave_base) {
  static_assert(S >= 2 && S <= 4, "stages");
  constexpr int PACK = kPackElems<DT>;
  constexpr int LP0 = (NTMASK & 1) ? kNonTemporal : kPlain;
  constexpr int LP1 = (NTMASK & 2) ? kNonTemporal : kPlain;
  constexpr int G = NS * U;   // DMA instructions per tile
  constexpr int SD = ND * U;  // store instructions per tile
  constexpr uint32_t STAGE = NS * U * 1024;
  if (nelem <= 0) return;
  uintptr_t mis = (uintptr_t)s0 | (uintptr_t)d0;
  if constexpr (NS > 1) mis |= (uintptr_t)s1;
  if constexpr (ND > 1) mis |= (uintptr_t)d1;
  if (mis & 15) {
    reduce_copy_rows<DT, OP, (U < 8 ? U : 8), NS, ND, NTMASK, DP0, DP1>(s0, s1, d0, d1, nelem, tid, nthr);
    return;
  }
  const uint32_t nwaves = (uint32_t)nthr >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6), lane = (uint32_t)tid & 63;
  const u32x4* a = (const u32x4*)s0;
  const u32x4* b = (const u32x4*)s1;
  u32x4* x = (u32x4*)d0;
  u32x4* y = (u32x4*)d1;
  const int64_t npack = nelem / PACK;
  if (npack > 0 && wave < nwaves) {
    const int64_t tile = 64 * U;
    const int64_t ntiles = (npack + tile - 1) / tile;
    const int64_t nmine = (int64_t)wave < ntiles ? (ntiles - wave + nwaves - 1) / nwaves : 0;
    auto issue = [&](int64_t k) {
      // M0 takes a scalar: the stage base is wave-uniform
      const uint32_t st = __builtin_amdgcn_readfirstlane(lds_wave_base + (uint32_t)(k % S) * STAGE);
      const int64_t t0 = ((int64_t)wave + k * nwaves) * tile + lane;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int64_t p = t0 + 64 * u;
        p = p < npack ? p : npack - 1;
        glds16<LP0>(a + p, st + u * 1024);
        if constexpr (NS > 1) glds16<LP1>(b + p, st + (U + u) * 1024);
      }
    };
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (s < nmine) issue(s);
#pragma unroll 1
    for (int64_t k = 0; k < nmine; ++k) {
      if (k + S - 1 < nmine) issue(k + S - 1);
      const int nd = (int)((nmine - 1 - k) < (S - 1) ? (nmine - 1 - k) : (S - 1));
      const int ns = (int)(k < (S - 1) ? k : (S - 1));
      wait_younger_ops<G, SD, S>(nd, ns);
      using lds_cptr = const __attribute__((address_space(3))) char*;
      using lds_vptr = const __attribute__((address_space(3))) u32x4*;
      const lds_cptr lst = (lds_cptr)(uintptr_t)(lds_wave_base + (uint32_t)(k % S) * STAGE);
      const int64_t t0 = ((int64_t)wave + k * nwaves) * tile + lane;
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *(lds_vptr)(lst + u * 1024 + lane * 16);
      if constexpr (NS > 1) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = pack_op<DT, OP>(v[u], *(lds_vptr)(lst + (U + u) * 1024 + lane * 16));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int64_t p = t0 + 64 * u;
        p = p < npack ? p : npack - 1;
        st16<DP0>(x + p, v[u]);
        if constexpr (ND > 1) st16<DP1>(y + p, v[u]);
      }
    }
  }
  // typed scalar tail (< one pack) over every data thread
  using T = typename Elem<DT>::T;
  for (int64_t e = npack * PACK + tid; e < nelem; e += nthr) {
    T v = (NTMASK & 1) ? __builtin_nontemporal_load((const T*)s0 + e) : ((const T*)s0)[e];
    if constexpr (NS > 1)
      v = scalar_op<DT, OP>(v, (NTMASK & 2) ? __builtin_nontemporal_load((const T*)s1 + e) : ((const T*)s1)[e]);
    ((T*)d0)[e] = v;
    if constexpr (ND > 1) ((T*)d1)[e] = v;
  }
}

}  // namespace mccs

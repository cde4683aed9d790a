// direct_kernel.h — two-shot ("direct") AllReduce for a fully connected node.
//
// The ring (ring_kernel.h, all_reduce.h) moves a bucket through 2(n-1)
// neighbour hops.  On an MI355X node every GPU has a link to every other, so
// here a bucket takes two (ring_cfg.h, "Direct"): scatter every chunk to its
// owner, reduce, and broadcast the result.  What it keeps from the reference
// is everything that decides a result bit for bit: the ring's chunk walk
// (all_reduce.h:28-42: chunkSize, loopSize, realChunkSize rounding, chunk k of
// channel bid at gridOffset + (bid*n + k)*realChunkSize), chunk k's owner (the
// rank at ring index k of channel bid's ring) and its summation order
// (acc = x[idx k+1]; acc = fn(x[idx k+j], acc) for j = 2..n, rounded in T at
// every step, all_reduce.h:46-70 + prims_simple.h:174-177), so the output
// equals the ring's (and the oracle's) for the same channels and rings.
//
// One launch per device (blockIdx.y = rank slot when ranks share a GPU), G
// workgroups per rank of MCCS_DIRECT_THREADS threads; sub-tiles of every
// chunk are dealt to the workgroups round-robin.  Phases, per workgroup:
//   1. copy its sub-tiles of chunks owned by others into the owner's in slot
//      (remote stores over xGMI); drain; count itself out per owner -- the
//      workgroup that completes an owner's count posts that owner's in flag;
//   2. for its sub-tiles of chunks it owns: wait for every in flag, reduce the
//      n sources in the ring's order (own input read locally, the others from
//      its own in slots), store to the output and to every peer's out slot;
//      drain; count out per peer -- the last posts the peer's out flag;
//   3. for its sub-tiles of chunks owned by others: wait for that owner's out
//      flag, copy the result from its out slot to the output.
// Flags hold the launch sequence number (>= seq = ready; ring_cfg.h has why
// one set of slots is safe across back-to-back launches).  The hand-off
// policy follows the ring's (mccsRingKernelCfg fence modes): drains only for
// uncached arenas, a system-scope release before counting out and an acquire
// after a wait otherwise (each workgroup fences its own writes: a release only
// writes back the issuing XCD's L2).
#pragma once
#include "ring_kernel.h"

namespace mccs {

constexpr int64_t kDirectSubBytes = 64 * 1024;  // sub-tile of a chunk dealt to one workgroup
constexpr int kDirectUnroll = 2;                 // packs per lane per source in flight (x up to 8 sources)

struct DirectWalk {
  int64_t size, chunkSize, loopSize, gran, sub;
  int n, nch;
};

template <int DT>
__device__ __forceinline__ DirectWalk direct_walk(const mccsDirectArgs& a) {
  using T = typename Elem<DT>::T;
  DirectWalk w;
  w.n = (int)a.nranks;
  w.nch = (int)a.nch;
  w.size = (int64_t)a.count;
  // all_reduce.h:17-21 with the ring kernel's arithmetic (ring_kernel.h run_elem)
  const int64_t stepSize = (int64_t)((int)a.buff_size / MCCS_BUFFER_SLOTS / (int)sizeof(T));
  w.chunkSize = (int64_t)(int)(stepSize * ALLREDUCE_CHUNKSTEPS);
  w.loopSize = (int64_t)w.nch * w.n * w.chunkSize;
  w.gran = (int64_t)((int)a.nthr_ref - WARP_SIZE) * 8 / (int64_t)sizeof(T);
  if (w.gran < 1) w.gran = 1;
  w.sub = kDirectSubBytes / (int64_t)sizeof(T);
  return w;
}

// Calls f(item, off, nelem, bid, k) for every sub-tile of every chunk in the
// ring's walk order; `item` numbers them 0, 1, ... identically in every
// workgroup and on every rank.
template <typename F>
__device__ __forceinline__ void direct_items(const DirectWalk& w, F&& f) {
  uint32_t item = 0;
  for (int64_t g = 0; g < w.size; g += w.loopSize) {
    int64_t rcs = div_up(w.size - g, (int64_t)w.nch * w.n);  // realChunkSize, all_reduce.h:30-36
    rcs = w.chunkSize < rcs ? w.chunkSize : rcs;
    rcs = (int64_t)(int)round_up(rcs, w.gran);
    for (int bid = 0; bid < w.nch; ++bid)
      for (int k = 0; k < w.n; ++k) {
        const int64_t off = g + ((int64_t)bid * w.n + k) * rcs;
        const int64_t ne = rcs < w.size - off ? rcs : w.size - off;
        for (int64_t s = 0; s < ne; s += w.sub) f(item++, off + s, ne - s < w.sub ? ne - s : w.sub, bid, k);
      }
  }
}

struct DirectShm {
  uint64_t seq;
  int ok;  // 0 after an abort / watchdog (written by thread 0 inside direct_wait only)
};

// Thread 0 spins until *flag >= seq; the whole workgroup then agrees.
__device__ __forceinline__ bool direct_wait(DirectShm& sh, const uint64_t* flag, uint64_t seq,
                                            volatile uint32_t* abortFlag, const mccsDirectArgs& a,
                                            const mccsRingKernelCfg& ecfg) {
  if (threadIdx.x == 0 && sh.ok) {
    const bool uncached = a.fence_mode != MCCS_FENCE_SYSTEM;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t attempt = 0, spins = 0;
    while (ld_poll(flag, uncached, attempt++) < seq) {
      if (++spins >= 64) {
        spins = 0;
        if (abort_raised(abortFlag)) {
          raise_error(abortFlag, ecfg, MCCS_ERR_ABORTED);
          sh.ok = 0;
          break;
        }
        if (a.timeout_ticks && __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
          raise_error(abortFlag, ecfg, MCCS_ERR_TIMEOUT);
          sh.ok = 0;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(MCCS_POLL_SLEEP);
    }
    if (sh.ok && !uncached) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  const bool ok = sh.ok != 0;
  __syncthreads();  // every thread has read ok before thread 0 can write it again
  return ok;
}

// This workgroup's writes of the phase are complete (and, for cached arenas,
// written back); count it out for every target rank.  The workgroup that
// completes a target's count resets it (for the next launch) and posts
// `seq` into the target's flag line.
__device__ __forceinline__ void direct_count_out(DirectShm& sh, const mccsDirectArgs& a, const mccsDirectRank& me,
                                                 char* ctrl, int cnt_base, int flag_base, uint64_t seq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && sh.ok) {
    if (a.fence_mode != MCCS_FENCE_UNCACHED) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (uint32_t t = 0; t < a.nranks; ++t) {
      if (t == me.rank) continue;
      uint32_t* cnt = (uint32_t*)(ctrl + cnt_base + (int)t * MCCS_FLAG_LINE_BYTES);
      const uint32_t old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == gridDim.x) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_flag((uint64_t*)(me.region[t] + flag_base + (int)me.rank * MCCS_FLAG_LINE_BYTES), seq);
      }
    }
  }
}

// Phase 2 of one sub-tile: acc = x[q1]; acc = fn(x[qj], acc) (j = 2..n) over
// the sources in ring order, stored to the output and every peer's out slot.
template <int DT, int OP>
__device__ __forceinline__ void direct_reduce(const void* const* src, int n, void* const* dst, int ndst, int64_t ne) {
  using T = typename Elem<DT>::T;
  constexpr int PACK = kPackElems<DT>;
  constexpr int U = kElemBytes<DT> == 1 ? 1 : kDirectUnroll;  // byte types unpack 16 lanes per pack
  const int tid = threadIdx.x, nthr = blockDim.x;
  uintptr_t mis = 0;
#pragma unroll
  for (int j = 0; j < MCCS_DIRECT_MAX_RANKS; ++j) {
    if (j < n) mis |= (uintptr_t)src[j];
    if (j < ndst) mis |= (uintptr_t)dst[j];
  }
  int64_t done = 0;
  if ((mis & 15) == 0) {
    const int64_t npack = ne / PACK;
    for (int64_t base = tid; base < npack; base += (int64_t)nthr * U) {
      u32x4 v[MCCS_DIRECT_MAX_RANKS][U];
#pragma unroll
      for (int j = 0; j < MCCS_DIRECT_MAX_RANKS; ++j)
        if (j < n) {
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (base + (int64_t)u * nthr < npack)
              v[j][u] = __builtin_nontemporal_load((const u32x4*)src[j] + base + (int64_t)u * nthr);
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (base + (int64_t)u * nthr >= npack) continue;
        u32x4 acc = v[0][u];
#pragma unroll
        for (int j = 1; j < MCCS_DIRECT_MAX_RANKS; ++j)
          if (j < n) acc = pack_op<DT, OP>(v[j][u], acc);
#pragma unroll
        for (int d = 0; d < MCCS_DIRECT_MAX_RANKS; ++d)
          if (d < ndst) ((u32x4*)dst[d])[base + (int64_t)u * nthr] = acc;
      }
    }
    done = npack * PACK;
  }
  for (int64_t e = done + tid; e < ne; e += nthr) {
    T acc = __builtin_nontemporal_load((const T*)src[0] + e);
#pragma unroll
    for (int j = 1; j < MCCS_DIRECT_MAX_RANKS; ++j)
      if (j < n) acc = scalar_op<DT, OP>(__builtin_nontemporal_load((const T*)src[j] + e), acc);
#pragma unroll
    for (int d = 0; d < MCCS_DIRECT_MAX_RANKS; ++d)
      if (d < ndst) ((T*)dst[d])[e] = acc;
  }
}

template <int DT, int OP>
__device__ __forceinline__ void direct_body(const mccsDirectArgs& a) {
  using T = typename Elem<DT>::T;
  __shared__ DirectShm sh;
  const mccsDirectRank& me = a.r[blockIdx.y];
  const int n = (int)a.nranks;
  char* const mine = me.region[me.rank];
  volatile uint32_t* abortFlag = me.comm ? me.comm->abortFlag : nullptr;
  mccsRingKernelCfg ecfg{};
  ecfg.err_line = me.err_line;
  if (threadIdx.x == 0) {
    sh.seq = __hip_atomic_load((uint64_t*)(mine + MCCS_DIRECT_LAUNCHES), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) + 1;
    sh.ok = !abort_raised(abortFlag);
  }
  __syncthreads();
  const uint64_t seq = sh.seq;
  const int64_t esz = (int64_t)sizeof(T);
  const int64_t slot = (int64_t)a.slot_bytes;
  auto in_slot = [&](char* region, uint32_t sender) {
    return region + MCCS_DIRECT_CTRL_BYTES + (int64_t)sender * slot;
  };
  auto out_slot = [&](char* region) {
    return region + MCCS_DIRECT_CTRL_BYTES + (int64_t)MCCS_DIRECT_MAX_RANKS * slot;
  };
  const DirectWalk w = direct_walk<DT>(a);
  const uint32_t G = gridDim.x, bx = blockIdx.x;
  u32x4 nopre[1];

  // 1. scatter: every chunk owned by another rank goes to its owner's in slot
  direct_items(w, [&](uint32_t item, int64_t off, int64_t ne, int bid, int k) {
    if (item % G != bx || !sh.ok) return;
    const uint32_t owner = a.idx2rank[bid][k];
    if (owner == me.rank) return;
    reduce_copy_rows<DT, OpSum, MCCS_RING_UNROLL, 1, 1, MCCS_RING_INPUT_NT, kPlain>(
        (const T*)me.send + off, nullptr, in_slot(me.region[owner], me.rank) + off * esz, nullptr, ne, threadIdx.x,
        blockDim.x, false, nopre);
  });
  direct_count_out(sh, a, me, mine, MCCS_DIRECT_CNT_IN(0), MCCS_DIRECT_IN_FLAG(0), seq);

  // 2. reduce the chunks this rank owns, in the ring's order
  bool in_seen = false;  // uniform across the workgroup, like `seen` below
  direct_items(w, [&](uint32_t item, int64_t off, int64_t ne, int bid, int k) {
    if (item % G != bx || !sh.ok) return;
    if (a.idx2rank[bid][k] != me.rank) return;
    if (!in_seen) {
      for (int s = 0; s < n; ++s)
        if (s != (int)me.rank &&
            !direct_wait(sh, (const uint64_t*)(mine + MCCS_DIRECT_IN_FLAG(s)), seq, abortFlag, a, ecfg))
          return;
      in_seen = true;
    }
    // sources in the ring's order from ring index k+1; destinations: the
    // output, then every peer's out slot
    const void* src[MCCS_DIRECT_MAX_RANKS];
    void* dst[MCCS_DIRECT_MAX_RANKS];
#pragma unroll
    for (int j = 0; j < MCCS_DIRECT_MAX_RANKS; ++j) {
      src[j] = nullptr;
      dst[j] = nullptr;
      if (j < n) {
        int idx = k + 1 + j;
        idx = idx >= n ? idx - n : idx;
        const uint32_t q = a.idx2rank[bid][idx];
        src[j] = q == me.rank ? (const void*)((const T*)me.send + off) : (const void*)(in_slot(mine, q) + off * esz);
        // slot j of dst: rank j (own -> the output)
        dst[j] = j == (int)me.rank ? (void*)((T*)me.recv + off) : (void*)(out_slot(me.region[j]) + off * esz);
      }
    }
    direct_reduce<DT, OP>(src, n, dst, n, ne);
  });
  direct_count_out(sh, a, me, mine, MCCS_DIRECT_CNT_OUT(0), MCCS_DIRECT_OUT_FLAG(0), seq);

  // 3. gather: results of the chunks owned by others, from this rank's out slot
  uint32_t seen = 0;  // owners whose out flag this workgroup has seen
  direct_items(w, [&](uint32_t item, int64_t off, int64_t ne, int bid, int k) {
    if (item % G != bx || !sh.ok) return;
    const uint32_t owner = a.idx2rank[bid][k];
    if (owner == me.rank) return;
    if (!(seen & (1u << owner))) {
      if (!direct_wait(sh, (const uint64_t*)(mine + MCCS_DIRECT_OUT_FLAG(owner)), seq, abortFlag, a, ecfg))
        return;
      seen |= 1u << owner;
    }
    reduce_copy_rows<DT, OpSum, MCCS_RING_UNROLL, 1, 1, 1, MCCS_RING_OUT_POLICY>(
        out_slot(mine) + off * esz, nullptr, (T*)me.recv + off, nullptr, ne, threadIdx.x, blockDim.x, false, nopre);
  });

  // the launch is over for this workgroup: the last one advances the sequence
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && sh.ok) {
    uint32_t* done = (uint32_t*)(mine + MCCS_DIRECT_DONE);
    if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == G) {
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((uint64_t*)(mine + MCCS_DIRECT_LAUNCHES), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int DT, int OP>
__global__ void __launch_bounds__(MCCS_DIRECT_THREADS) direct_kernel(mccsDirectArgs a) {
  direct_body<DT, OP>(a);
}

}  // namespace mccs

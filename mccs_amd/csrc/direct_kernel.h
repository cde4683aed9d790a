// direct_kernel.h — direct AllReduce (two-shot / one-shot) for a fully
// connected node.
//
// The ring (ring_kernel.h, all_reduce.h) moves a bucket through 2(n-1)
// neighbour hops.  On an MI355X node every GPU has a link to every other, so
// here a bucket takes two (two-shot) or one (one-shot) -- ring_cfg.h,
// "Direct AllReduce", has the region layout and the reuse argument.  What it
// keeps from the reference is everything that decides a result bit for bit:
// the ring's chunk walk (all_reduce.h:28-42: chunkSize, loopSize,
// realChunkSize rounding, chunk k of channel bid at gridOffset +
// (bid*n + k)*realChunkSize), chunk k's owner (the rank at ring index k of
// channel bid's ring) and its summation order (acc = x[idx k+1];
// acc = fn(x[idx k+j], acc) for j = 2..n, rounded in T at every step,
// all_reduce.h:46-70 + prims_simple.h:174-177), so the output equals the
// ring's (and the oracle's) for the same channels and rings.
//
// One launch per device (blockIdx.y = rank slot when ranks share a GPU), G
// workgroups per rank of MCCS_DIRECT_THREADS threads.  Each phase cuts the
// chunks it touches into pieces and deals them to the G workgroups
// round-robin, so every phase is spread over all of them.
//   two-shot
//     1. scatter: pieces of chunks owned by others -> the owner's in slot
//        (remote stores over xGMI); drain; add the elements written to each
//        owner's IN_CNT line;
//     2. reduce: wait until every peer has sent this rank its chunks; for
//        pieces of the chunks this rank owns, reduce the n sources in the
//        ring's order (own input local, the others from its in slots), store
//        to the output and every peer's out slot; drain; add to every peer's
//        OUT_CNT line;
//     3. gather: wait for every owner's broadcast; copy the results of
//        chunks owned by others from the out slot to the output.
//     Phases 1 and 3 deal the same chunks with the same pieces, so a
//     workgroup rewrites in phase 3 exactly what it read in phase 1 (an
//     in-place call is safe).
//   one-shot (small buckets)
//     1. broadcast: pieces of the whole input -> every peer's one-shot slot
//        of this launch's parity; drain; add to every peer's IN_CNT line;
//     2. reduce: wait for every peer's input; every chunk, in the ring's
//        order, straight into the output.
//   AllGather one-shot (all_gather.h's result, byte for byte)
//     1. this rank's segment -> every peer's one-shot slot and its own place
//        in the output; drain; count out;
//     2. wait; every peer's segment from its slot to its place.
// The hand-off policy follows the ring's (mccsRingKernelCfg fence modes):
// drains only for uncached arenas, a system-scope release before the count
// and an acquire after a wait otherwise (each workgroup fences its own
// writes: a release only writes back the issuing XCD's L2).
#pragma once
#include "ring_kernel.h"

namespace mccs {

#ifndef MCCS_DIRECT_UNROLL
#define MCCS_DIRECT_UNROLL 2
#endif
constexpr int kDirectUnroll = MCCS_DIRECT_UNROLL;  // packs per lane per source in flight (x up to 8 sources)

// Phase timeline of workgroup 0 of every rank slot (A/B builds only:
// -DMCCS_DIRECT_TRACE, read with mccs_direct_trace; tools/direct_trace.py):
// s_memrealtime (100 MHz) stored with plain vector stores, last launch wins.
enum : int {
  kDtStart = 0, kDtPhase1 = 1, kDtCounted1 = 2, kDtWait2 = 3, kDtPhase2 = 4, kDtCounted2 = 5, kDtWait3 = 6,
  kDtEnd = 7, kDtPrologue = 8, kDtPiece1 = 9, kDtPiece3 = 10, kDtEvents = 12
};
#ifdef MCCS_DIRECT_TRACE
namespace {
__device__ unsigned long long g_dtrace[MCCS_MULTI_MAX_RANKS][kDtEvents];
}  // namespace
#define MCCS_DTRACE(ev)                                                                              \
  do {                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_dtrace[blockIdx.y][ev] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define MCCS_DTRACE(ev) ((void)0)
#endif

// The walk in 32-bit arithmetic: a direct bucket holds < 2^31 elements
// (direct_bytes <= 1 GiB), and 64-bit divisions are long software sequences
// that a per-chunk loop run by every thread cannot afford.
struct DirectWalk {
  uint32_t size, chunkSize, loopSize, gran;
  uint32_t n, nch;
};

template <int DT>
__device__ __forceinline__ DirectWalk direct_walk(const mccsDirectArgs& a) {
  using T = typename Elem<DT>::T;
  DirectWalk w;
  w.n = a.nranks;
  w.nch = a.nch;
  w.size = (uint32_t)a.count;
  // all_reduce.h:17-21 with the ring kernel's arithmetic (ring_kernel.h run_elem)
  const uint32_t stepSize = (uint32_t)((int)a.buff_size / MCCS_BUFFER_SLOTS / (int)sizeof(T));
  w.chunkSize = stepSize * ALLREDUCE_CHUNKSTEPS;
  const uint64_t loop = (uint64_t)w.nch * w.n * w.chunkSize;
  w.loopSize = loop > 0x7fffffffu ? 0x7fffffffu : (uint32_t)loop;  // >= size: one loop
  w.gran = ((a.nthr_ref - WARP_SIZE) * 8) / (uint32_t)sizeof(T);
  if (w.gran < 1) w.gran = 1;
  return w;
}

// This workgroup's pieces (pc elements) of the ring chunks `want(owner)`
// selects, in walk order (all_reduce.h:28-42: loop, realChunkSize, chunk k
// of channel bid at gridOffset + (bid*n + k)*realChunkSize): the selected
// chunks' pieces are numbered 0, 1, ... and piece p goes to workgroup p % G.
// Calls f(off, nelem, bid, k, owner).  Divisions: two per loop and one for
// the walk's last, partial chunk; the piece numbering is kept mod G by
// subtraction.
template <typename W, typename F>
__device__ __forceinline__ void direct_pieces(const DirectWalk& w, const uint8_t (*idx2rank)[MCCS_DIRECT_MAX_RANKS],
                                              uint32_t pc, uint32_t G, uint32_t bx, W&& want, F&& f) {
  uint32_t base = 0;  // (pieces of selected chunks before this one) mod G
  const uint32_t parts = w.nch * w.n;
  for (uint32_t g = 0; g < w.size; g += w.loopSize) {
    uint32_t rcs = (w.size - g + parts - 1) / parts;  // realChunkSize, all_reduce.h:30-36
    rcs = w.chunkSize < rcs ? w.chunkSize : rcs;
    rcs = (rcs + w.gran - 1) / w.gran * w.gran;
    const uint32_t np_full = (rcs + pc - 1) / pc;
    for (uint32_t c = 0, bid = 0, k = 0; c < parts; ++c, k = k + 1 == w.n ? 0 : k + 1, bid += k == 0) {
      const uint32_t off = g + c * rcs;
      if (off >= w.size) return;  // every later chunk of the walk is empty
      const uint32_t owner = idx2rank[bid][k];
      if (!want(owner)) continue;
      const uint32_t ne = rcs < w.size - off ? rcs : w.size - off;
      const uint32_t np = ne == rcs ? np_full : (ne + pc - 1) / pc;
      for (uint32_t j = bx >= base ? bx - base : bx + G - base; j < np; j += G) {
        const uint32_t s = j * pc;
        f((int64_t)(off + s), (int64_t)(ne - s < pc ? ne - s : pc), (int)bid, (int)k, owner);
      }
      base += np;
      while (base >= G) base -= G;
    }
  }
}

struct DirectShm {
  uint8_t idx2rank[MCCS_MAX_NCHANNELS][MCCS_DIRECT_MAX_RANKS];  // a.idx2rank (walk lookups stay in LDS)
  char* region[MCCS_DIRECT_MAX_RANKS];                          // a.region
  uint64_t seq;
  uint64_t e_in;                            // E_IN at launch start
  uint64_t e_self;                          // E_SELF at launch start
  uint64_t e_out[MCCS_DIRECT_MAX_RANKS];    // E_OUT at launch start
  uint64_t owned[MCCS_DIRECT_MAX_RANKS];    // elements of this launch's chunks each rank owns
  uint64_t sent[MCCS_DIRECT_MAX_RANKS];     // elements this workgroup wrote into each rank's slots (this phase)
  int ok;  // 0 after an abort / watchdog (written by thread 0 inside direct_wait only)
};

// Wave 0 spins until, for every rank t in `mask`, the u64 count at
// ctrl + cnt_base + t x line reaches need[t]; lane t polls rank t, so all
// counts cost one round trip per poll.  The whole workgroup then agrees.
__device__ __forceinline__ bool direct_wait(DirectShm& sh, const char* ctrl, int cnt_base, uint32_t mask,
                                            const uint64_t* need_sh, volatile uint32_t* abortFlag,
                                            const mccsDirectArgs& a, const mccsRingKernelCfg& ecfg) {
  if (threadIdx.x < 64 && sh.ok) {
    const uint32_t lane = threadIdx.x;
    const bool poll = lane < MCCS_DIRECT_MAX_RANKS && ((mask >> lane) & 1u);
    const uint64_t need = poll ? need_sh[lane] : 0;
    const uint64_t* cnt = (const uint64_t*)(ctrl + cnt_base + (poll ? lane : 0) * MCCS_FLAG_LINE_BYTES);
    const bool uncached = a.fence_mode != MCCS_FENCE_SYSTEM;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t attempt = 0, spins = 0;
    int failed = 0;
    while (!__all(!poll || ld_poll(cnt, uncached, attempt) >= need)) {
      ++attempt;
      if (++spins >= 64) {
        spins = 0;
        int why = 0;  // decided by lane 0, taken by every lane
        if (lane == 0) {
          if (abort_raised(abortFlag)) why = 1;
          else if (a.timeout_ticks && __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) why = 2;
          if (why) raise_error(abortFlag, ecfg, why == 1 ? MCCS_ERR_ABORTED : MCCS_ERR_TIMEOUT);
        }
        why = __builtin_amdgcn_readfirstlane(why);
        if (why) {
          failed = 1;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(MCCS_POLL_SLEEP);
    }
    if (lane == 0) {
      if (failed) sh.ok = 0;
      else if (!uncached) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
  }
  __syncthreads();
  const bool ok = sh.ok != 0;
  __syncthreads();  // every thread has read ok before thread 0 can write it again
  return ok;
}

// This workgroup's writes of the phase are complete (and, for cached arenas,
// written back): add what it wrote into each rank's slots (sh.sent) to that
// rank's count line for this rank (lane t of wave 0 for rank t: one remote
// atomic each, no return value awaited), then clear sh.sent.  self: also
// count sh.sent[me] into this rank's own line (its reads of the input done).
__device__ __forceinline__ void direct_count_out(DirectShm& sh, const mccsDirectArgs& a, const mccsDirectRank& me,
                                                 int cnt_base, bool self = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64 && sh.ok) {
    if (a.fence_mode != MCCS_FENCE_UNCACHED) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint32_t t = threadIdx.x;
    if (t < a.nranks && (t != me.rank || self) && sh.sent[t])
      __hip_atomic_fetch_add((uint64_t*)(sh.region[t] + cnt_base + (int)me.rank * MCCS_FLAG_LINE_BYTES), sh.sent[t],
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (threadIdx.x < MCCS_DIRECT_MAX_RANKS) sh.sent[threadIdx.x] = 0;
  __syncthreads();
}

// acc = x[src0]; acc = fn(x[srcj], acc) (j = 1..n-1) over the sources in
// ring order, stored to every non-null destination among dst[0 .. ndst)
// (n = 1: a copy to several places).
// (Forcing the uniform pointers into scalar registers with readfirstlane
// cut VGPRs from ~160 to ~113 and ran 3-7 % slower on the virtual node: the
// second resident workgroup per CU it allows costs more than it gives.)
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
          if (d < ndst && dst[d]) ((u32x4*)dst[d])[base + (int64_t)u * nthr] = acc;
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
      if (d < ndst && dst[d]) ((T*)dst[d])[e] = acc;
  }
}

template <int DT, int OP>
__device__ __forceinline__ void direct_body(const mccsDirectArgs& a) {
  using T = typename Elem<DT>::T;
  __shared__ DirectShm sh;
  const mccsDirectRank& me = a.r[blockIdx.y];
  const int n = (int)a.nranks;
  char* const mine = a.region[me.rank];
  volatile uint32_t* abortFlag = me.abort_flag;
  mccsRingKernelCfg ecfg{};
  ecfg.err_line = me.err_line;
  const DirectWalk w = direct_walk<DT>(a);
  const bool ag = a.mode == MCCS_DIRECT_AG_ONE_SHOT;  // AllGather: bytes, no reduction
  const bool one_shot = a.mode == MCCS_DIRECT_ONE_SHOT || ag;
  // In-place one-shot AllReduce: phase 2 overwrites the input that other
  // workgroups of this rank may still be reading in phase 1 (their pieces
  // differ), so phase 2 also waits for this rank's own workgroups to have
  // counted their reads (IN_CNT(me), E_SELF).  AllGather in place writes
  // only the other ranks' segments in phase 2; two-shot pieces keep a
  // workgroup on the same bytes in phases 1 and 3.
  const bool self_wait = a.mode == MCCS_DIRECT_ONE_SHOT && me.send == me.recv;
  MCCS_DTRACE(kDtStart);
  // Prologue: lanes of wave 0 load the state words in one round trip.  The
  // abort flag is not read here: it is host memory (comm.cpp
  // place_abort_line), and a read from every workgroup at once cost 1.2 us at
  // 32 KiB and 22 us at 512 KiB per call; the waits below check it.
  if (threadIdx.x < 64) {
    const uint32_t lane = threadIdx.x;
    uint64_t v = 0;
    if (lane < MCCS_DIRECT_ST_WORDS)
      v = __hip_atomic_load((uint64_t*)(mine + MCCS_DIRECT_STATE) + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == MCCS_DIRECT_ST_LAUNCHES) sh.seq = v + 1;
    if (lane == MCCS_DIRECT_ST_E_IN) sh.e_in = v;
    if (lane >= 2 && lane < 2 + MCCS_DIRECT_MAX_RANKS) sh.e_out[lane - 2] = v;
    if (lane == MCCS_DIRECT_ST_E_SELF) sh.e_self = v;
    if (lane == MCCS_DIRECT_ST_WORDS) sh.ok = v == 0;
    if (lane < MCCS_DIRECT_MAX_RANKS) {
      sh.owned[lane] = a.owned[lane];
      sh.sent[lane] = 0;
      sh.region[lane] = a.region[lane];
    }
    // the walk's table, 4 bytes per lane
    ((uint32_t*)sh.idx2rank)[lane] = ((const uint32_t*)a.idx2rank)[lane];
  }
  // Arrival: once every workgroup of the launch has read the start values
  // above, the last to arrive may advance them for the next launch.  The
  // count is issued now and its result consumed after phase 1 (its round
  // trip overlaps the scatter); the loads above complete first.
  uint32_t arrived = 0;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    arrived = __hip_atomic_fetch_add((uint32_t*)(mine + MCCS_DIRECT_DONE), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  MCCS_DTRACE(kDtPrologue);
  const uint64_t seq = sh.seq;
  const int64_t esz = (int64_t)sizeof(T);
  const uint32_t G = gridDim.x, bx = blockIdx.x;
  const uint32_t peers = ((1u << n) - 1u) & ~(1u << me.rank);
  const uint32_t piece = a.piece > 0 ? a.piece : 1;
  const uint32_t piece2 = a.piece2 > 0 ? a.piece2 : 1;
  __shared__ uint64_t need[MCCS_DIRECT_MAX_RANKS];
  // The last workgroup to arrive advances the running totals and the launch
  // count for the next launch (every workgroup of this one has its copies).
  auto advance = [&]() {
    if (threadIdx.x == 0 && arrived + 1 == G) {
      uint64_t* st = (uint64_t*)(mine + MCCS_DIRECT_STATE);
      __hip_atomic_store((uint32_t*)(mine + MCCS_DIRECT_DONE), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(st + MCCS_DIRECT_ST_E_IN, sh.e_in + (one_shot ? (uint64_t)w.size : sh.owned[me.rank]),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!one_shot)
        for (int t = 0; t < n; ++t)
          __hip_atomic_store(st + MCCS_DIRECT_ST_E_OUT(t), sh.e_out[t] + sh.owned[t], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      if (self_wait)
        __hip_atomic_store(st + MCCS_DIRECT_ST_E_SELF, sh.e_self + (uint64_t)w.size, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(st + MCCS_DIRECT_ST_LAUNCHES, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };

  if (one_shot) {
    const int64_t oslot = (int64_t)a.oslot_bytes;
    const int64_t obase = MCCS_DIRECT_CTRL_BYTES + (int64_t)MCCS_DIRECT_SLOTS * (int64_t)a.slot_bytes +
                          (int64_t)(seq & 1) * MCCS_DIRECT_MAX_RANKS * oslot;
    // 1. broadcast the whole input: pieces of [0, count) to every peer's slot
    const uint32_t np = (w.size + piece - 1) / piece;
    for (uint32_t j = bx; j < np && sh.ok; j += G) {
      const int64_t off = (int64_t)j * piece;
      const int64_t ne = (int64_t)w.size - off < (int64_t)piece ? (int64_t)w.size - off : (int64_t)piece;
      const void* src[MCCS_DIRECT_MAX_RANKS] = {(const T*)me.send + off};
      // slot t: rank t's one-shot slot; this rank: nothing, or (AllGather)
      // its own segment of the output
      void* dst[MCCS_DIRECT_MAX_RANKS];
#pragma unroll
      for (int t = 0; t < MCCS_DIRECT_MAX_RANKS; ++t)
        dst[t] = t >= n                 ? nullptr
                 : t != (int)me.rank    ? (void*)(sh.region[t] + obase + (int64_t)me.rank * oslot + off * esz)
                 : ag                   ? (void*)((T*)me.recv + (int64_t)me.rank * w.size + off)
                                        : nullptr;
      direct_reduce<DT, OpSum>(src, 1, dst, n, ne);
      if (threadIdx.x == 0)
        for (int t = 0; t < n; ++t) sh.sent[t] += (uint64_t)ne;
    }
    MCCS_DTRACE(kDtPhase1);
    direct_count_out(sh, a, me, MCCS_DIRECT_IN_CNT(0), self_wait);
    MCCS_DTRACE(kDtCounted1);
    advance();
    if (threadIdx.x < MCCS_DIRECT_MAX_RANKS)
      need[threadIdx.x] = (threadIdx.x == me.rank ? sh.e_self : sh.e_in) + (uint64_t)w.size;
    __syncthreads();
    const uint32_t waitmask = self_wait ? peers | (1u << me.rank) : peers;
    bool in_seen = false;  // uniform across the workgroup
    if (ag) {
      // 2. (AllGather) every peer's segment, from its slot to the output;
      // pieces of the n-1 segments dealt round-robin
      uint32_t base = 0;
      const uint32_t nps = (w.size + piece2 - 1) / piece2;
      for (uint32_t t = 0; t < (uint32_t)n; ++t) {
        if (t == me.rank) continue;
        for (uint32_t j = bx >= base ? bx - base : bx + G - base; j < nps && sh.ok; j += G) {
          if (!in_seen) {
            if (!direct_wait(sh, mine, MCCS_DIRECT_IN_CNT(0), peers, need, abortFlag, a, ecfg)) break;
            in_seen = true;
            MCCS_DTRACE(kDtWait2);
          }
          const int64_t off = (int64_t)j * piece2;
          const int64_t ne = (int64_t)w.size - off < (int64_t)piece2 ? (int64_t)w.size - off : (int64_t)piece2;
          const void* src[MCCS_DIRECT_MAX_RANKS] = {mine + obase + (int64_t)t * oslot + off * esz};
          void* dst[MCCS_DIRECT_MAX_RANKS] = {(T*)me.recv + (int64_t)t * w.size + off};
          direct_reduce<DT, OpSum>(src, 1, dst, 1, ne);
        }
        base += nps;
        while (base >= G) base -= G;
      }
    } else
    // 2. every chunk, reduced in the ring's order into the output
    direct_pieces(w, sh.idx2rank, piece2, G, bx, [](uint32_t) { return true; },
                  [&](int64_t off, int64_t ne, int bid, int k, uint32_t) {
                    if (!sh.ok) return;
                    if (!in_seen) {
                      if (!direct_wait(sh, mine, MCCS_DIRECT_IN_CNT(0), waitmask, need, abortFlag, a, ecfg)) return;
                      in_seen = true;
                      MCCS_DTRACE(kDtWait2);
                    }
                    const void* src[MCCS_DIRECT_MAX_RANKS];
                    void* dst[MCCS_DIRECT_MAX_RANKS] = {(T*)me.recv + off};
#pragma unroll
                    for (int j = 0; j < MCCS_DIRECT_MAX_RANKS; ++j) {
                      src[j] = nullptr;
                      if (j < n) {
                        int idx = k + 1 + j;
                        idx = idx >= n ? idx - n : idx;
                        const uint32_t q = sh.idx2rank[bid][idx];
                        src[j] = q == me.rank ? (const void*)((const T*)me.send + off)
                                              : (const void*)(mine + obase + (int64_t)q * oslot + off * esz);
                      }
                    }
                    direct_reduce<DT, OP>(src, n, dst, 1, ne);
                  });
  } else {
    const int64_t slot = (int64_t)a.slot_bytes;
    auto in_slot = [&](char* region, uint32_t sender) {
      return region + MCCS_DIRECT_CTRL_BYTES + (int64_t)sender * slot;
    };
    auto out_slot = [&](char* region) {
      return region + MCCS_DIRECT_CTRL_BYTES + (int64_t)MCCS_DIRECT_MAX_RANKS * slot;
    };
    auto others = [&](uint32_t owner) { return owner != me.rank; };
    auto own = [&](uint32_t owner) { return owner == me.rank; };

    // 1. scatter: every chunk owned by another rank goes to its owner's in slot
    direct_pieces(w, sh.idx2rank, piece, G, bx, others, [&](int64_t off, int64_t ne, int, int, uint32_t owner) {
      if (!sh.ok) return;
      const void* src[MCCS_DIRECT_MAX_RANKS] = {(const T*)me.send + off};
      void* dst[MCCS_DIRECT_MAX_RANKS] = {in_slot(sh.region[owner], me.rank) + off * esz};
      direct_reduce<DT, OpSum>(src, 1, dst, 1, ne);
      MCCS_DTRACE(kDtPiece1);
      if (threadIdx.x == 0) sh.sent[owner] += (uint64_t)ne;
    });
    MCCS_DTRACE(kDtPhase1);
    direct_count_out(sh, a, me, MCCS_DIRECT_IN_CNT(0));
    MCCS_DTRACE(kDtCounted1);
    advance();

    // 2. reduce the chunks this rank owns, in the ring's order; broadcast
    if (threadIdx.x < MCCS_DIRECT_MAX_RANKS) need[threadIdx.x] = sh.e_in + sh.owned[me.rank];
    __syncthreads();
    bool in_seen = false;  // uniform across the workgroup, like out_seen below
    direct_pieces(w, sh.idx2rank, piece2, G, bx, own, [&](int64_t off, int64_t ne, int bid, int k, uint32_t) {
      if (!sh.ok) return;
      if (!in_seen) {
        if (!direct_wait(sh, mine, MCCS_DIRECT_IN_CNT(0), peers, need, abortFlag, a, ecfg)) return;
        in_seen = true;
        MCCS_DTRACE(kDtWait2);
      }
      // sources in the ring's order from ring index k+1; destination slot t:
      // rank t's out slot (own: the output)
      const void* src[MCCS_DIRECT_MAX_RANKS];
      void* dst[MCCS_DIRECT_MAX_RANKS];
#pragma unroll
      for (int j = 0; j < MCCS_DIRECT_MAX_RANKS; ++j) {
        src[j] = nullptr;
        dst[j] = nullptr;
        if (j < n) {
          int idx = k + 1 + j;
          idx = idx >= n ? idx - n : idx;
          const uint32_t q = sh.idx2rank[bid][idx];
          src[j] = q == me.rank ? (const void*)((const T*)me.send + off) : (const void*)(in_slot(mine, q) + off * esz);
          dst[j] = j == (int)me.rank ? (void*)((T*)me.recv + off) : (void*)(out_slot(sh.region[j]) + off * esz);
        }
      }
      direct_reduce<DT, OP>(src, n, dst, n, ne);
      if (threadIdx.x == 0)
        for (int t = 0; t < n; ++t) sh.sent[t] += (uint64_t)ne;
    });
    MCCS_DTRACE(kDtPhase2);
    direct_count_out(sh, a, me, MCCS_DIRECT_OUT_CNT(0));
    MCCS_DTRACE(kDtCounted2);

    // 3. gather: results of the chunks owned by others, from this rank's out slot
    if (threadIdx.x < MCCS_DIRECT_MAX_RANKS) need[threadIdx.x] = sh.e_out[threadIdx.x] + sh.owned[threadIdx.x];
    __syncthreads();
    bool out_seen = false;
    direct_pieces(w, sh.idx2rank, piece, G, bx, others, [&](int64_t off, int64_t ne, int, int, uint32_t) {
      if (!sh.ok) return;
      if (!out_seen) {
        if (!direct_wait(sh, mine, MCCS_DIRECT_OUT_CNT(0), peers, need, abortFlag, a, ecfg)) return;
        out_seen = true;
        MCCS_DTRACE(kDtWait3);
      }
      const void* src[MCCS_DIRECT_MAX_RANKS] = {out_slot(mine) + off * esz};
      void* dst[MCCS_DIRECT_MAX_RANKS] = {(T*)me.recv + off};
      direct_reduce<DT, OpSum>(src, 1, dst, 1, ne);
      MCCS_DTRACE(kDtPiece3);
    });
  }
  MCCS_DTRACE(kDtEnd);
}

// ---- LL one-shot (ring_cfg.h): the smallest buckets, thread-linear over the
// bucket's 8-byte words.  Word w belongs to global thread w mod (G x threads)
// in both phases, so an in-place call overwrites a word only after the same
// thread has read and sent it.  Each word's chunk (and so its ring order) is
// found from the walk: chunk offsets are multiples of the realChunkSize
// granule ((nthr_ref - 64) x 8 bytes), so no word straddles two chunks.
template <typename T>
__device__ __forceinline__ uint64_t ll_load_word(const char* base, uint32_t wd, uint32_t size, bool aligned) {
  constexpr uint32_t EPW = 8 / sizeof(T);
  const uint32_t e = wd * EPW;
  if (aligned && e + EPW <= size) return __builtin_nontemporal_load((const uint64_t*)base + wd);
  uint64_t v = 0;
#pragma unroll
  for (uint32_t j = 0; j < EPW; ++j)
    if (e + j < size) {
      const T x = ((const T*)base)[e + j];
      uint64_t b = 0;
      __builtin_memcpy(&b, &x, sizeof(T));
      v |= b << (8 * sizeof(T) * j);
    }
  return v;
}

template <typename T>
__device__ __forceinline__ void ll_store_word(char* base, uint32_t wd, uint32_t size, bool aligned, uint64_t v) {
  constexpr uint32_t EPW = 8 / sizeof(T);
  const uint32_t e = wd * EPW;
  if (aligned && e + EPW <= size) {
    __builtin_nontemporal_store(v, (uint64_t*)base + wd);
    return;
  }
#pragma unroll
  for (uint32_t j = 0; j < EPW; ++j)
    if (e + j < size) {
      const uint64_t b = v >> (8 * sizeof(T) * j);
      T x;
      __builtin_memcpy(&x, &b, sizeof(T));
      ((T*)base)[e + j] = x;
    }
}

__device__ __forceinline__ u32x4 ll_pack(uint64_t v) {
  u32x4 p;
  p.x = (uint32_t)v;
  p.y = (uint32_t)(v >> 32);
  p.z = 0;
  p.w = 0;
  return p;
}

template <int DT, int OP>
__device__ __forceinline__ void direct_ll_body(const mccsDirectArgs& a) {
  using T = typename Elem<DT>::T;
  constexpr uint32_t EPW = 8 / sizeof(T);
  __shared__ uint64_t s_seq;
  __shared__ int s_ok;
  __shared__ uint8_t s_idx2rank[MCCS_MAX_NCHANNELS][MCCS_DIRECT_MAX_RANKS];
  const mccsDirectRank& me = a.r[blockIdx.y];
  const uint32_t n = a.nranks, rank = me.rank;
  char* const mine = a.region[rank];
  volatile uint32_t* abortFlag = me.abort_flag;
  mccsRingKernelCfg ecfg{};
  ecfg.err_line = me.err_line;
  const DirectWalk w = direct_walk<DT>(a);
  const uint32_t nwords = (uint32_t)(((uint64_t)w.size * sizeof(T) + 7) / 8);
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const char* in = (const char*)me.send;
  char* out = (char*)me.recv;
  const bool in_al = ((uintptr_t)in & 7) == 0, out_al = ((uintptr_t)out & 7) == 0;
  // the first word's input load is in flight while thread 0 reads the launch
  // count: the prologue costs one round trip
  uint64_t own0 = 0;
  if (gtid < nwords) own0 = ll_load_word<T>(in, gtid, w.size, in_al);
  if (threadIdx.x == 0) {
    s_seq = __hip_atomic_load((uint64_t*)(mine + MCCS_DIRECT_STATE) + MCCS_DIRECT_ST_LAUNCHES, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT) + 1;
    s_ok = 1;  // abortFlag (host memory) is checked in the wait, not here: see the two-shot prologue
  }
  if (threadIdx.x < 64) ((uint32_t*)s_idx2rank)[threadIdx.x] = ((const uint32_t*)a.idx2rank)[threadIdx.x];
  __syncthreads();
  // every workgroup has read the launch count once it arrives; the last one
  // to arrive advances it (after phase 1)
  uint32_t arrived = 0;
  if (threadIdx.x == 0)
    arrived = __hip_atomic_fetch_add((uint32_t*)(mine + MCCS_DIRECT_DONE), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t seq = s_seq;
  // 32-bit line flag, never 0 (the region's zeroed lines never read as
  // valid, whatever the launch count): 1 + seq mod (2^32 - 1)
  const uint32_t seq32 = 1u + (uint32_t)(seq % 0xffffffffull);
  const uint64_t flag = (uint64_t)seq32 << 32;
  const int64_t lslot = (int64_t)a.ll_slot_bytes;
  const int64_t llbase = MCCS_DIRECT_CTRL_BYTES + (int64_t)MCCS_DIRECT_SLOTS * (int64_t)a.slot_bytes +
                         2 * (int64_t)MCCS_DIRECT_MAX_RANKS * (int64_t)a.oslot_bytes +
                         (int64_t)(seq & 1) * MCCS_DIRECT_MAX_RANKS * lslot;
  bool ok = s_ok != 0;
  const bool ag = a.mode == MCCS_DIRECT_LL_AG;  // AllGather: T = int8, w.size = bytes per rank
  char* const own_seg = out + (int64_t)rank * w.size;
  const bool own_al = ((uintptr_t)own_seg & 7) == 0;
  // 1. every word to every peer's LL slot, as a flag-carrying line
  // (AllGather: and to this rank's own place in the output, unless in place)
  if (ok)
    for (uint32_t wd = gtid; wd < nwords; wd += stride) {
      const uint64_t v = wd == gtid ? own0 : ll_load_word<T>(in, wd, w.size, in_al);
      if (ag && own_seg != in) ll_store_word<T>(own_seg, wd, w.size, own_al, v);
      const uint64_t lo = flag | (v & 0xffffffffull), hi = flag | (v >> 32);
#pragma unroll
      for (uint32_t t = 0; t < MCCS_DIRECT_MAX_RANKS; ++t)
        if (t < n && t != rank) {
          uint64_t* p = (uint64_t*)(a.region[t] + llbase + (int64_t)rank * lslot + (int64_t)wd * 16);
          __hip_atomic_store(p, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(p + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
  if (threadIdx.x == 0 && arrived + 1 == gridDim.x) {
    __hip_atomic_store((uint32_t*)(mine + MCCS_DIRECT_DONE), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((uint64_t*)(mine + MCCS_DIRECT_STATE) + MCCS_DIRECT_ST_LAUNCHES, seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // 2. poll every peer's line of each word, reduce in the ring's order
  const uint32_t peers = ((1u << n) - 1u) & ~(1u << rank);
  const uint32_t parts = w.nch * n;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t wd = gtid; ok && wd < nwords; wd += stride) {
    uint32_t bid = 0, k = 0;
    if (!ag) {
      const uint32_t e = wd * EPW;
      const uint32_t g = e / w.loopSize * w.loopSize;
      uint32_t rcs = (w.size - g + parts - 1) / parts;  // realChunkSize, all_reduce.h:30-36
      rcs = w.chunkSize < rcs ? w.chunkSize : rcs;
      rcs = (rcs + w.gran - 1) / w.gran * w.gran;
      const uint32_t c = (e - g) / rcs;
      bid = c / n;
      k = c - bid * n;
    }
    const uint64_t own = ag ? 0 : wd == gtid ? own0 : ll_load_word<T>(in, wd, w.size, in_al);
    const char* lb = mine + llbase + (int64_t)wd * 16;
    uint64_t h0[MCCS_DIRECT_MAX_RANKS], h1[MCCS_DIRECT_MAX_RANKS];
    uint32_t pending = peers, spins = 0;
    for (;;) {
#pragma unroll
      for (uint32_t t = 0; t < MCCS_DIRECT_MAX_RANKS; ++t)
        if ((pending >> t) & 1u) {
          const uint64_t* p = (const uint64_t*)(lb + (int64_t)t * lslot);
          h0[t] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          h1[t] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#pragma unroll
      for (uint32_t t = 0; t < MCCS_DIRECT_MAX_RANKS; ++t)
        if (((pending >> t) & 1u) && (uint32_t)(h0[t] >> 32) == seq32 && (uint32_t)(h1[t] >> 32) == seq32)
          pending &= ~(1u << t);
      if (!pending) break;
      if (++spins % 64 == 0) {
        const bool ab = abort_raised(abortFlag);
        const bool to = !ab && a.timeout_ticks && __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks;
        if (ab || to) {
          raise_error(abortFlag, ecfg, ab ? MCCS_ERR_ABORTED : MCCS_ERR_TIMEOUT);
          ok = false;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(MCCS_POLL_SLEEP);
    }
    if (!ok) break;
    if (ag) {  // every peer's word to its place (all_gather.h: rank t's segment at t x size)
#pragma unroll
      for (uint32_t t = 0; t < MCCS_DIRECT_MAX_RANKS; ++t)
        if (t < n && t != rank) {
          char* seg = out + (int64_t)t * w.size;
          ll_store_word<T>(seg, wd, w.size, ((uintptr_t)seg & 7) == 0,
                           (h0[t] & 0xffffffffull) | (h1[t] << 32));
        }
      continue;
    }
    // acc = x[idx k+1]; acc = fn(x[idx k+j], acc)
    u32x4 acc{};
#pragma unroll
    for (uint32_t j = 0; j < MCCS_DIRECT_MAX_RANKS; ++j)
      if (j < n) {
        uint32_t idx = k + 1 + j;
        idx = idx >= n ? idx - n : idx;
        const uint32_t q = s_idx2rank[bid][idx];
        uint64_t v = own;
#pragma unroll
        for (uint32_t t = 0; t < MCCS_DIRECT_MAX_RANKS; ++t)
          if (t == q && t != rank) v = (h0[t] & 0xffffffffull) | (h1[t] << 32);
        acc = j == 0 ? ll_pack(v) : pack_op<DT, OP>(ll_pack(v), acc);
      }
    ll_store_word<T>(out, wd, w.size, out_al, (uint64_t)acc.x | ((uint64_t)acc.y << 32));
  }
}

template <int DT, int OP>
__global__ void __launch_bounds__(MCCS_DIRECT_THREADS) direct_kernel(mccsDirectArgs a) {
  // Launch guard (launch_guard.h), taken before the prologue reads the
  // control block's launch count and running totals.  The rank slots' fields
  // are read where the kernel arguments live (taking the parameter's address
  // would copy all 4 KiB of it to scratch); the guard's state waits out the
  // body in LDS.
  __shared__ GuardSlot s_guard;
  if (threadIdx.x == 0) {
    mccsLaunchGuard* g = nullptr;
    int ok = 1;
    if (!a.no_guard) {
      const uintptr_t ka = (uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
      const mccsDirectRank* ranks = (const mccsDirectRank*)(ka + offsetof(mccsDirectArgs, r));
      GuardWait w{};
      w.abortFlagRef = (uint32_t* const*)&ranks[blockIdx.y].abort_flag;
      w.timeout = a.timeout_ticks;
      w.err_line = ranks[blockIdx.y].err_line;
      g = comm_guard(ranks[blockIdx.y].comm);
      ok = guard_acquire([&](int k) { return comm_guard(ranks[k].comm); }, (int)gridDim.y, (int)blockIdx.y,
                         a.guard_order, launch_token(), blockIdx.x == 0 && blockIdx.y == 0, w);
    }
    s_guard.g = ok ? g : nullptr;
    s_guard.ok = ok;
  }
  __syncthreads();
  if (!s_guard.ok) return;
  if (a.mode == MCCS_DIRECT_LL_ONE_SHOT || a.mode == MCCS_DIRECT_LL_AG) direct_ll_body<DT, OP>(a);
  else direct_body<DT, OP>(a);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && s_guard.g) guard_release(s_guard.g, gridDim.x);
}

}  // namespace mccs

// launch_guard.h — one launch of a communicator at a time, enforced on the GPU.
//
// The reference runs every kernel of a communicator on its one private comm
// stream (src/mccs/src/proxy/init.rs:166-175, plan.rs:659-667), so two of them
// never overlap.  This library launches on the caller's streams; the host
// orders a comm's eager launches across streams (plan.cpp), but a HIP graph
// replay makes no library call, so a replay could run beside an eager launch,
// or beside another graph's replay, of the same communicator -- sharing its
// FIFO flag lines, saved steps and direct control block (wrong sums: 5 of 6
// and 6 of 6 such races at n = 2 / 4 with the guard off,
// profiles/r06_launch_guard.json).  So each library launch takes the
// communicator's guard word (ring_cfg.h mccsLaunchGuard) before it touches
// any of that state and hands it back after its last workgroup is done; a
// launch that finds it held waits, bounded by the watchdog (it never streams
// beside the holder).
//
// The word: token << 17 | confirmed << 16 | finished workgroups (0 = free).
// One rank slot per launch (the deployment shape): every workgroup's claiming
// thread CASes 0 -> its launch's token; finding its own token there is as
// good (a sibling workgroup took it, and may already have counted itself out).
// Fused launches of several rank slots (ranks sharing a GPU) need all their
// slots' words at once: workgroup (0, 0) takes them in address order (a
// parallel try first; on any miss it gives back what that try took -- no
// other workgroup of its launch moves before the confirm bit -- and then
// takes them one by one in that order, so two fused launches never hold each
// other's), then sets every word's confirm bit; the other workgroups wait for
// their slot's word to carry their token and the bit.  Release: each
// workgroup adds 1 to its slot's word once its stores completed; the add that
// completes the slot's count stores 0.
// Hand-off visibility: the state a launch leaves for the next (saved steps,
// direct launch counts) is written and read with system- / agent-scope atomics
// (uncached lines, or L2-served sc1 accesses), so the release needs only the
// store completion (s_waitcnt vmcnt(0)) before the add, and the acquire only
// the claim's return before those loads (MI355X_MICROARCH.md: 8-byte agent
// atomics on both sides).
#pragma once
#include <hip/hip_runtime.h>

#include "ring_cfg.h"

namespace mccs {

// A token no other launch in flight on the device carries: the address of the
// launch's AQL dispatch packet (two dispatches running at once sit in
// different queues, or in different slots of one queue: a slot is rewritten
// only a full ring of packets later, which an in-order queue cannot start
// before this dispatch ends), 64-byte aligned, so bits 6..47 (42 bits), and 5
// bits of the launch's kernel-argument block above them.  Never 0.
__device__ __forceinline__ uint64_t launch_token() {
  const uint64_t pkt = (uint64_t)(uintptr_t)__builtin_amdgcn_dispatch_ptr();
  const uint64_t ka = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  const uint64_t tok = ((pkt >> 6) & ((1ull << 42) - 1)) | (((ka >> 4) & 31ull) << 42);
  return tok ? tok : 1;
}

__device__ __forceinline__ uint64_t guard_ld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void guard_st(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// CAS 0 -> v; returns the value found (0: taken)
__device__ __forceinline__ uint64_t guard_cas0(uint64_t* p, uint64_t v) {
  uint64_t expect = 0;
  __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return expect;
}
__device__ __forceinline__ uint64_t guard_tok(uint64_t word) { return word >> MCCS_GUARD_TOK_SHIFT; }

// A bounded wait: abortFlag (host memory: read every 64th step) and the
// launch's watchdog end it with the comm's error bits raised, as a FIFO wait's
// would (ring_kernel.h raise_error).
struct GuardWait {
  uint32_t* const* abortFlagRef;  // where the comm's abortFlag pointer lives (read only once waiting)
  uint64_t timeout;               // s_memrealtime ticks; 0 = never
  uint32_t err_line;
  uint32_t spins;
  uint64_t t0;
};

__device__ __forceinline__ bool guard_step(GuardWait& w) {
  __builtin_amdgcn_s_sleep(2);
  if (++w.spins % 64) return true;
  uint32_t* const af = *w.abortFlagRef;
  uint32_t bits = 0;
  if (af && __hip_atomic_load(af, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
    bits = MCCS_ERR_ABORTED;
  else if (w.timeout && __builtin_amdgcn_s_memrealtime() - w.t0 > w.timeout)
    bits = MCCS_ERR_TIMEOUT;
  if (!bits) return true;
  if (af) {
    if (w.err_line) __hip_atomic_fetch_or(af + 1, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (bits & MCCS_ERR_TIMEOUT) __hip_atomic_store(af, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return false;
}

// Takes one guard for `tok`, waiting while another launch holds it; `found`
// is what the caller's first CAS (0 -> token) returned.
__device__ __forceinline__ bool guard_take(mccsLaunchGuard* g, uint64_t tok, GuardWait& w, uint64_t found) {
  bool counted = false;
  for (uint64_t o = found;; o = guard_cas0(&g->word, tok << MCCS_GUARD_TOK_SHIFT)) {
    if (o == 0 || guard_tok(o) == tok) return true;
    if (!counted) {
      __hip_atomic_fetch_add(&g->waits, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      counted = true;
    }
    for (;;) {
      if (!guard_step(w)) return false;
      const uint64_t v = guard_ld(&g->word);
      if (v != 0 && guard_tok(v) == tok) return true;
      if (v == 0) break;
    }
  }
}

// The claim of one workgroup (its claiming thread only).  `guard_of(k)` is
// rank slot k's guard, `ns` the launch's slots, `slot` this workgroup's;
// `order` lists the slots by guard address (4 bits each, the host sorts them:
// the one global order every leader takes guards in).  Returns false if the
// wait was given up (error raised; nothing may stream).
template <class GuardOf>
__device__ __forceinline__ bool guard_acquire(GuardOf guard_of, int ns, int slot, uint64_t order, uint64_t tok,
                                              bool leader, GuardWait w) {
  const uint64_t mine = tok << MCCS_GUARD_TOK_SHIFT;
  w.spins = 0;
  w.t0 = __builtin_amdgcn_s_memrealtime();
  if (ns == 1) {
    mccsLaunchGuard* const g = guard_of(0);
    return guard_take(g, tok, w, guard_cas0(&g->word, mine));
  }
  if (leader) {
    uint64_t found[MCCS_MULTI_MAX_RANKS];
    bool all = true;
#pragma unroll
    for (int i = 0; i < MCCS_MULTI_MAX_RANKS; ++i)
      if (i < ns) found[i] = guard_cas0(&guard_of((int)((order >> (4 * i)) & 15))->word, mine);
#pragma unroll
    for (int i = 0; i < MCCS_MULTI_MAX_RANKS; ++i)
      if (i < ns) all = all && found[i] == 0;
    if (!all) {
#pragma unroll
      for (int i = 0; i < MCCS_MULTI_MAX_RANKS; ++i)
        if (i < ns && found[i] == 0) guard_st(&guard_of((int)((order >> (4 * i)) & 15))->word, 0);
      for (int i = 0; i < ns; ++i) {
        mccsLaunchGuard* const g = guard_of((int)((order >> (4 * i)) & 15));
        if (!guard_take(g, tok, w, guard_cas0(&g->word, mine))) return false;
      }
    }
    // no workgroup of this launch has counted itself out yet (they wait for
    // this bit), so every word still reads exactly `mine`
    for (int k = 0; k < ns; ++k) guard_st(&guard_of(k)->word, mine | MCCS_GUARD_CONFIRMED);
    return true;
  }
  mccsLaunchGuard* const g = guard_of(slot);
  for (;;) {
    const uint64_t v = guard_ld(&g->word);
    if (guard_tok(v) == tok && (v & MCCS_GUARD_CONFIRMED)) return true;
    if (!guard_step(w)) return false;
  }
}

// The release of one workgroup (its claiming thread, after every wave waited
// for its own memory operations (s_waitcnt vmcnt(0)) and a workgroup barrier):
// `nwg` workgroups of this slot take part.
__device__ __forceinline__ void guard_release(mccsLaunchGuard* g, uint32_t nwg) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t prev = __hip_atomic_fetch_add(&g->word, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((prev & MCCS_GUARD_FIN_MASK) + 1 == nwg) guard_st(&g->word, 0);
}

// A workgroup's guard state across the kernel body (LDS): the guard it holds
// (null: none to release) and whether the body may run.
struct GuardSlot {
  mccsLaunchGuard* g;
  int ok;
};

__device__ __forceinline__ mccsLaunchGuard* comm_guard(const void* dev_comm) {
  return (mccsLaunchGuard*)((char*)dev_comm + MCCS_GUARD_OFF);
}

}  // namespace mccs

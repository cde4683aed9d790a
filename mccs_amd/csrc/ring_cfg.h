// ring_cfg.h — conventions shared by the ring kernels and the C++ host.
//
// FIFO flag lines.  A connector's `tail` / `head` pointers (mccsDevConnInfo,
// devcomm.h:36-46) point at an array of 128-byte lines, one per lane (a lane
// is one workgroup of a channel; the reference has exactly one, lane 0):
//   word 0  the step counter the peer polls / we poll
//   word 1  this side's saved step for the lane (local lines only)
// With one lane this is binary-compatible with the reference SHM metadata
// (SendBufMeta.head / RecvBufMeta.tail at offset 0 followed by 120 pad bytes,
// src/mccs/src/transport/meta.rs:7-67), so word 1 is free padding there.
#pragma once
#include <stdint.h>

#include "mccs_devcomm.h"

#define MCCS_FLAG_LINE_BYTES 128
#define MCCS_FLAG_LINE_WORDS (MCCS_FLAG_LINE_BYTES / 8)
#define MCCS_MAX_LANES 64
// Largest ring workgroup.  576 = 9 waves covers the reference's 17-warp (544
// thread) blocks (get_task_schema, plan.rs:602-635) and keeps ~168 VGPRs per
// lane (3 waves per SIMD): the fully inlined ring loop with 8 packs in flight
// per source fits without spilling, which a 1024-thread bound (128 VGPRs) did not.
#define MCCS_RING_MAX_THREADS 576

// Fence policy for FIFO hand-offs.  Communicator launches carry it in their
// launch arguments (mccsMultiLaunchArgs.cfg); the reference-named kernels,
// launched by an external planner that cannot say what memory its FIFOs are,
// always run with the reference defaults (system-scope fences, 2-step slices).
#define MCCS_FENCE_SYSTEM 0   // FIFO memory may be cached: system-scope release/acquire
#define MCCS_FENCE_UNCACHED 1 // FIFO memory is uncached (hipDeviceMallocUncached): drains only
// Uncached FIFO memory, but a system-scope release fence before every post
// (the analogue of __threadfence_system before postPeer, prims_simple.h:
// 120-125,211); polls stay relaxed.  The step between relaxed hand-offs and
// the cached-memory mode for links where a drained store might not yet be
// visible to the peer when the flag lands.
#define MCCS_FENCE_UNCACHED_RELEASE 2

// Error bits a ring kernel reports for ONE communicator: word 1 of the
// communicator's own abort line (abortFlag[1]; the library allocates that line,
// 64 bytes, zeroed at init), read back by mccsCommSync.  A process-wide word
// would let one communicator's abort fail another's sync.
#define MCCS_ERR_TIMEOUT 1u
#define MCCS_ERR_ABORTED 2u

struct mccsRingKernelCfg {
  uint32_t fence_mode;    // MCCS_FENCE_*
  uint32_t slice_steps;   // FIFO steps per slice: 2 (reference SliceSteps) or 4 (one slice per chunk)
  uint64_t timeout_ticks; // s_memrealtime ticks (100 MHz); 0 = never
  uint32_t profile;       // 1: accumulate per-slice wait / work ticks (mccs_ring_profile)
  uint32_t err_line;      // 1: error bits go to abortFlag[1] (library launches: the abort line is
                          // ours); 0: reference-named kernels, whose abortFlag is the caller's
                          // 4-byte allocation: only abortFlag itself is raised (the reference's
                          // one error channel, devcomm.h abortFlag)
  uint32_t fifo_slots;    // physical FIFO slots (power of two >= MCCS_BUFFER_SLOTS): slot = step % fifo_slots,
                          // a sender may run fifo_slots steps ahead; the reference has 8
  uint32_t no_guard;      // 1: skip the launch guard (test hook MCCS_LAUNCH_GUARD=0 only)
};

// ---- Launch guard (launch_guard.h): one launch of a communicator at a time.
// A communicator's kernels share its FIFO flag lines, the lanes' saved steps
// (word 1 above) and the direct control block, so two of its launches running
// at once return wrong sums.  The host orders eager launches across streams
// (plan.cpp), but a graph replay makes no library call; so every library
// launch first takes its communicator's guard line on the device and gives it
// back when its last workgroup is done.  The line lives in the communicator's
// device allocation, after mccsDevCommAndChannels and the per-channel views.
// One word holds the whole state, so each step is one atomic: the holder's
// token in bits 17..63 (0 = free), bit 16 "every slot held" (fused launches),
// bits 0..15 the holder's workgroups of this slot that have finished.
#define MCCS_GUARD_FIN_MASK 0xffffull
#define MCCS_GUARD_CONFIRMED (1ull << 16)
#define MCCS_GUARD_TOK_SHIFT 17
struct mccsLaunchGuard {
  uint64_t word;   // token << MCCS_GUARD_TOK_SHIFT | confirmed | finished workgroups; 0 = free
  uint64_t waits;  // workgroups that found the guard held by another launch (diagnostic, only grows)
  uint64_t pad[14];
};
#define MCCS_GUARD_OFF                                                                                      \
  ((sizeof(struct mccsDevCommAndChannels) + MCCS_MAX_NCHANNELS * sizeof(struct mccsRingConnView) + 127) / \
   128 * 128)

// Per-device ring profile counters (s_memrealtime ticks, 100 MHz), summed
// over every slice of every workgroup while mccsRingKernelCfg.profile is set.
#define MCCS_PROF_SLICES 0  // slices executed
#define MCCS_PROF_WAIT 1    // slice start -> peer flags satisfied (thread 0)
#define MCCS_PROF_WORK 2    // flags satisfied -> stores drained, both barriers included
#define MCCS_PROF_DRAIN 3   // part of WORK: thread 0's wave done issuing -> every wave drained (barrier)
#define MCCS_PROF_N 4

// Communicator launch: one or several communicators of one device in ONE
// launch (several when ranks share a GPU: tests' virtual node).
// blockIdx.y = rank slot.
#define MCCS_MULTI_MAX_RANKS 16
// A launch whose ranks' channels each run one work of one element may carry
// those works in its arguments (kernarg memory is device memory on MI355X)
// instead of the host-mapped work FIFO, whose read over PCIe is the long pole
// of the kernel prologue; inFifo = 0, so nothing is acknowledged.  Rank slot
// k's works are inline_work[k * channels used ...], each only its header and
// its one element (mccsInlineWork, 56 B instead of mccsDevWork's 512): HIP
// copies every argument byte at every launch, and 4 KiB of them cost 1-3 us
// of host time per launch (profiles/r05_host_overhead.json).  8 works: the
// n = 8 rings (7 channels), or two fused rank slots of 4 channels.
#define MCCS_INLINE_WORKS 8
struct mccsInlineWork {
  struct mccsDevWorkHeader header;
  struct mccsDevWorkElem elem;
};
// The connector addresses one channel's lanes need (the prev recv and next
// send mccsDevConnInfo fields), kept by this library beside its device
// communicator (comm.cpp comm_build_device): a launch loads them together with
// the communicator instead of one dependent round trip later through
// mccsDevChannel.peers.  Reference-built communicators have none (view = 0).
struct mccsRingConnView {
  char* rbuf;        // receive FIFO data
  char* sbuf;        // send FIFO data
  uint64_t* r_tail;  // recv: polled (ours)
  uint64_t* r_head;  // recv: posted (prev's)
  uint64_t* s_head;  // send: polled (ours)
  uint64_t* s_tail;  // send: posted (next's)
};
struct mccsMultiLaunchArgs {
  struct mccsDevComm* comm[MCCS_MULTI_MAX_RANKS];
  struct mccsDevWork* work[MCCS_MULTI_MAX_RANKS];
  const struct mccsRingConnView* view[MCCS_MULTI_MAX_RANKS];  // per channel id; 0: use comm's peers
  uint64_t channelMask;
  struct mccsRingKernelCfg cfg;  // this launch's hand-off policy
  uint32_t inline_works;         // > 0: the works are inline_work[0 .. inline_works)
  uint32_t pad3;
  uint64_t guard_order;          // rank slots by guard address, 4 bits each (launch_guard.h)
  struct mccsInlineWork inline_work[MCCS_INLINE_WORKS];
};
#ifdef __cplusplus
static_assert(sizeof(mccsInlineWork) == 56 && offsetof(mccsInlineWork, elem) == offsetof(mccsDevWork, elems),
              "an inline work is the head of a mccsDevWork: header + one element");
static_assert(sizeof(mccsMultiLaunchArgs) <= 1024, "ring launch arguments must stay within 1 KiB");
#endif

// ---- Direct AllReduce on a fully connected node (direct_kernel.h)
// Every rank reaches every peer's arena over its own xGMI link, so instead of
// 2(n-1) ring hops a bucket takes two (two-shot: each rank writes every chunk
// it does not own into the owner's "in" slot, each owner reduces its chunks
// in exactly the ring's order and writes the result into every peer's "out"
// slot, every rank copies the results it does not own to its output) or one
// (one-shot, small buckets: every rank writes its whole input into every
// peer's one-shot slot and every rank reduces every chunk itself, in the
// ring's order).  Chunk ownership and summation order are the ring's
// (all_reduce.h), so results are bit-identical to the ring and the oracle.
//
// A rank's direct region (in its FIFO arena, after the ring's data):
//   [control, MCCS_DIRECT_CTRL_BYTES]
//   [two-shot in : MCCS_DIRECT_MAX_RANKS senders x slot_bytes]  (by element offset)
//   [two-shot out: slot_bytes]
//   [one-shot in : 2 parities x MCCS_DIRECT_MAX_RANKS senders x oslot_bytes]
//   [LL one-shot : 2 parities x MCCS_DIRECT_MAX_RANKS senders x ll_slot_bytes]
// LL one-shot (the smallest buckets): every 8 data bytes travel as one
// 16-byte line {data lo, flag, data hi, flag} written with two 8-byte
// system-scope stores, flag = 1 + seq mod (2^32 - 1) (never 0, so a zeroed
// line is never valid); a receiver polls the lines
// themselves, so the hand-off needs no drain, no count atomic and no
// separate flag round trip.  Its region is written only with such lines
// (zero at init), so a line left from an earlier launch carries a smaller
// seq; its slots alternate by parity like the one-shot's (same argument).
// Hand-offs are element counts: a sender adds the elements it wrote into a
// rank's slot to that rank's IN_CNT line (one remote atomic per workgroup and
// target, after its stores drained), an owner adds the elements it broadcast
// to every peer's OUT_CNT line.  Counts only grow; the receiver keeps running
// totals of what it has been sent so far (E_IN, E_OUT) and waits for
// total + this launch's share.  Launch seq s (1, 2, ...) and the totals are
// advanced in the control block by the last workgroup of a launch to arrive
// (after every workgroup read them), so graph replays keep counting.
// Reuse across back-to-back launches:
//   two-shot slots: a rank's in slots are refilled (phase 1 of launch s+1,
//     which waits for nothing) only by a peer that finished launch s, which
//     needed this rank's broadcast of s (or this rank owned nothing and read
//     no in slot); its out slot is refilled only by an owner that counted this
//     rank's scatter of s+1, made after this rank finished launch s;
//   one-shot slots alternate by parity s & 1: a peer writes parity p in
//     launch s+2 only after finishing s+1, which needed this rank's writes of
//     s+1, made after this rank finished reading parity p in launch s.
// Both hold across any mix of variants (and AllGather): a peer cannot finish
// a launch without a hand-off this rank makes in that same launch (with
// count >= 1 some rank owns elements, and whoever it is waits, directly or
// through its broadcast, for this rank's phase-1 count).
#define MCCS_DIRECT_MAX_RANKS 8
#define MCCS_DIRECT_CTRL_BYTES 65536
// u64, added to by sender s; a rank's own line IN_CNT(rank) counts its own
// workgroups' reads of an in-place one-shot input (nobody else writes it)
#define MCCS_DIRECT_IN_CNT(s) ((s) * MCCS_FLAG_LINE_BYTES)
#define MCCS_DIRECT_OUT_CNT(o) (1024 + (o) * MCCS_FLAG_LINE_BYTES)     // u64, added to by owner o
// u64 state words (one line, read by one wave load): launches completed,
// E_IN (elements each sender has sent so far), E_OUT[o] (elements owner o
// has broadcast so far)
#define MCCS_DIRECT_STATE 2048
#define MCCS_DIRECT_ST_LAUNCHES 0
#define MCCS_DIRECT_ST_E_IN 1
#define MCCS_DIRECT_ST_E_OUT(o) (2 + (o))
#define MCCS_DIRECT_ST_E_SELF (2 + MCCS_DIRECT_MAX_RANKS)  // elements this rank counted to itself (in-place one-shot)
#define MCCS_DIRECT_ST_WORDS (3 + MCCS_DIRECT_MAX_RANKS)
#define MCCS_DIRECT_DONE 4096                                          // u32: workgroups arrived in the launch
#define MCCS_DIRECT_SLOTS (MCCS_DIRECT_MAX_RANKS + 1)                  // two-shot slots
#define MCCS_DIRECT_THREADS 512
#define MCCS_DIRECT_TWO_SHOT 0
#define MCCS_DIRECT_ONE_SHOT 1
#define MCCS_DIRECT_AG_ONE_SHOT 2  // AllGather: count = bytes per rank (dtype int8)
#define MCCS_DIRECT_LL_ONE_SHOT 3  // one-shot through flag-carrying 16-byte lines (uncached arenas)
#define MCCS_DIRECT_LL_AG 4        // AllGather through the same lines (count = bytes per rank)

struct mccsDirectRank {  // one rank slot of a direct launch (blockIdx.y)
  const void* send;
  void* recv;
  struct mccsDevComm* comm;  // the rank's device communicator
  uint32_t* abort_flag;      // comm->abortFlag (one load less in the prologue)
  uint32_t rank;
  uint32_t err_line;
};
struct mccsDirectArgs {
  struct mccsDirectRank r[MCCS_MULTI_MAX_RANKS];
  // every rank's direct region as the launching process maps it: one table
  // for all rank slots (fused slots are ranks of one communicator in one
  // process, plan.cpp direct_group), so HIP copies 64 B per launch, not 1 KiB
  char* region[MCCS_DIRECT_MAX_RANKS];
  uint64_t count;          // elements
  uint64_t slot_bytes;     // bytes of one two-shot slot (>= count * element size for two-shot)
  uint64_t oslot_bytes;    // bytes of one one-shot slot (>= count * element size for one-shot)
  uint64_t ll_slot_bytes;  // bytes of one LL slot (>= 2 x count * element size, rounded to 8 bytes, for LL)
  uint64_t timeout_ticks;  // s_memrealtime ticks; 0 = never
  uint32_t nranks, nch, nthr_ref, buff_size;  // the ring walk this launch reproduces
  uint32_t fence_mode;                        // MCCS_FENCE_*
  uint32_t mode;                              // MCCS_DIRECT_TWO_SHOT / ONE_SHOT / AG_ONE_SHOT
  uint32_t piece;                             // elements per piece of the scatter / gather phases
  uint32_t piece2;                            // elements per piece of the reduction phase
  uint32_t no_guard;                          // 1: skip the launch guard (test hook only)
  uint32_t pad2;
  uint64_t guard_order;                       // rank slots by guard address, 4 bits each (launch_guard.h)
  uint64_t owned[MCCS_DIRECT_MAX_RANKS];      // elements of the walk's chunks each rank owns
  uint8_t idx2rank[MCCS_MAX_NCHANNELS][MCCS_DIRECT_MAX_RANKS];  // rank at ring index k of channel bid
};
#ifdef __cplusplus
static_assert(sizeof(mccsDirectArgs) <= 4096, "direct launch arguments must stay within 4 KiB");
#endif

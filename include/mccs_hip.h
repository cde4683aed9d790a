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

/* hipStream_t is an opaque pointer in the HIP C API; the identical typedef in
 * hip_runtime_api.h is a compatible redeclaration (C11 / C++). */
typedef struct ihipStream_t *hipStream_t;

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
#define MCCS_REDUCE_VARIANT_REG_BLOCKED 3 /* REG with a contiguous run of tiles per block */
#define MCCS_REDUCE_VARIANT_REG_ROWS 4    /* REG with wave-contiguous 1 KiB rows */

mccsResult_t mccs_hip_reduce(void *dst, const void *const *srcs, int nsrcs, size_t count, int dtype,
                             int op, hipStream_t stream);
mccsResult_t mccs_hip_reduce_copy(void *const *dsts, int ndsts, const void *const *srcs, int nsrcs,
                                  size_t count, int dtype, int op, hipStream_t stream);
/* Select the main loop (0 = default), unroll = KiB per source per wave tile
 * for LDS / 16-byte packs per lane for REG (1/2/4/8, 0 = default), cache
 * policy (0 plain, 1 non-temporal, -1 default; REG: 2 nt loads + plain
 * stores, 3 plain loads + nt stores; LDS: 2 plain LDS-DMA + nt stores,
 * 3 nt + sc1 stores, 4 write-through sc1 stores (default), 5 sc0 sc1 nt),
 * persistent blocks per CU,
 * LDS ring stages (2..4) and waves per block (4/8); 0 = default for each.
 * Process-wide; for benchmarking and tests. */
mccsResult_t mccs_hip_reduce_tune(int variant, int unroll, int policy, int blocks_per_cu, int stages,
                                  int waves);
void mccs_hip_reduce_get_tune(int *variant, int *unroll, int *policy, int *blocks_per_cu, int *stages,
                              int *waves);
/* Caps the LDS main loop's grid at `blocks` workgroups (0 = blocks_per_cu x
 * CUs, the default).  Process-wide; for benchmarking. */
mccsResult_t mccs_hip_reduce_tune_grid(int blocks);

/* ======================================================================
 * Ring collectives: device kernels (reference src/collectives) and the
 * host runtime that plans and launches them (reference src/mccs/src/proxy,
 * comm, transport; src/libmccs).
 * ====================================================================== */

/* Host stub of the reference-named kernel mccsKernel_<Func>_RING_SIMPLE_<Op>_<T>
 * (collectives.h:43-49) for hipLaunchKernel: the value plan.rs:142-166 stores
 * in KernelPlan.kernel_fn.  func: mccsFuncAllReduce | mccsFuncAllGather. */
const void *mccs_hip_coll_kernel(int func, int dtype, int op);
/* plan.rs:638-669 launch_plan: hipLaunchKernel(fn, grid, block, {comm,
 * channelMask, workHead}, 0, stream).  grid = #channels * lanes; block =
 * 96..576 threads (one wave of it is the control wave).
 * One launch per rank, one rank per GPU (the reference deployment): ranks
 * that share a GPU spin on each other's FIFO flags, so their kernels must be
 * co-resident, which separate launches do not guarantee (two co-located ranks
 * launched one after the other deadlock until the watchdog fires).  While an
 * earlier launch of ANOTHER communicator on the current device, issued through
 * this function by this process, is still running, the call is refused with
 * mccsInvalidUsage and nothing is launched.  Co-located ranks go through the
 * communicator API (mccsCommInitAll + mccsGroupStart/End), which fuses them
 * into one launch.  The reference-named kernels run the reference FIFO depth
 * (MCCS_BUFFER_SLOTS = 8 slots per connection): a communicator of this library
 * built with another fifo_slots is refused with mccsInvalidUsage (its peers
 * would index a different slot ring). */
mccsResult_t mccs_hip_launch_coll(int func, int dtype, int op, struct mccsDevComm *comm, uint64_t channelMask,
                                  struct mccsDevWork *workHead, unsigned grid, unsigned block,
                                  hipStream_t stream);
/* Watchdog of the reference-named kernels on the current device: ms without
 * FIFO progress before a kernel raises abortFlag and returns; 0 = the default
 * (10 min), < 0 = none.  The reference kernels have none and the reference host
 * never reads abortFlag, so the default outlasts any late peer a deployment
 * sees (a watchdog that fired on one would silently end every later collective
 * of the communicator); tests lower it so a hang ends quickly.  Call it once
 * per device before the launches it should govern. */
mccsResult_t mccs_hip_set_ref_watchdog(int timeout_ms);

typedef struct mccsComm *mccsComm_t;

#define MCCS_LOCALITY_SENDER 0   /* FIFO data in the sender's HBM; receiver reads over xGMI */
#define MCCS_LOCALITY_RECEIVER 1 /* FIFO data in the receiver's HBM; sender writes over xGMI */
#define MCCS_FIFO_UNCACHED 0     /* hipDeviceMallocUncached arena: no L2 maintenance needed */
#define MCCS_FIFO_DEVICE 1       /* hipMalloc arena + system-scope release/acquire */
#define MCCS_FIFO_UNCACHED_RELEASE 2 /* uncached arena + a system-scope release fence before every
                                        post (the reference's __threadfence_system before postPeer,
                                        prims_simple.h:120-125,211); polls stay relaxed */

/* Communicator profile: comm_default_config (mccs.toml:18-20, config.rs:15-97)
 * plus the MI355X execution knobs.  Zero fields take defaults.
 * ABI note: `fifo_slots`, `direct_bytes` and `oneshot_bytes` were appended in
 * library version 0.3 and `ll_bytes` in 0.3.1, which grew the struct;
 * mccsCommConfigDefault() writes sizeof(mccsCommConfig) bytes, so a caller
 * compiled against an older header must be rebuilt.  From 0.4 the struct ends
 * in reserved words that later fields will take, so its size stays fixed;
 * callers binding the struct by hand (ctypes, bindgen) check
 * mccsCommConfigSize() or call mccsCommConfigDefaultSized(). */
typedef struct {
  int channel_count;    /* rings; 0 = auto: 2 x edge-disjoint Hamiltonian cycles of the node */
  int buffer_size;      /* FIFO bytes per connection (buffer_sizes[0]); 0 = 4 MiB */
  int lanes;            /* workgroups per channel; 0 = auto (64 / channels, <= 64, fitted to residency) */
  int block_threads;    /* threads per workgroup (96..576, multiple of 32); 0 = MCCS_RING_MAX_THREADS (576) */
  int locality;         /* MCCS_LOCALITY_*; default RECEIVER (remote writes; SENDER = reference shm layout) */
  int fifo_memory;      /* MCCS_FIFO_*; default UNCACHED (MCCS_FIFO_MEMORY=uncached|release|device) */
  int timeout_ms;       /* FIFO-wait watchdog: ms without progress before the kernel gives up (mccsTimeout);
                           0 = 600000 (10 min, torch's default collective timeout: a peer may arrive
                           minutes late, e.g. while rank 0 writes a checkpoint), < 0 = never;
                           MCCS_TIMEOUT_MS overrides the default */
  int work_fifo_depth;  /* mccsDevWork slots (power of two); 0 = 4096 */
  int bridge_streams;   /* -1 (default): launch on the caller's stream; 1: user stream -> comm stream -> user stream events (libmccs two-stream bridge) */
  const int *rings;     /* channel_count x nranks send orders (comm_patterns_override); NULL = auto */
  int fifo_slots;       /* FIFO slots per connection of buffer_size / 8 bytes each: 8 (the reference's
                           MCCS_BUFFER_SLOTS), 16 or 32; 0 = default (16).  More slots = more slices in
                           flight per lane; the chunk schedule (and so every result) still follows
                           buffer_size, as in the reference */
  int direct_bytes;     /* AllReduce buckets of at most this many bytes per rank run the direct
                           (two-shot) kernel on a fully connected node of <= 8 ranks: every chunk to
                           its ring owner, reduced in the ring's order, results broadcast, so the
                           output equals the ring's bit for bit; larger buckets take the ring.
                           0 = default (MCCS_DIRECT_BYTES; else 8 MiB at >= 4 ranks, 4 MiB at 3,
                           off at 2),
                           < 0 = never.  Every rank must agree
                           (it sizes the arena: Connect refuses a mismatch) */
  int oneshot_bytes;    /* buckets of at most this many bytes per rank take the one-shot variant
                           instead: every rank sends its whole input to every peer and reduces
                           every chunk itself (same order, same bits; one exchange instead of
                           two).  0 = default (MCCS_ONESHOT_BYTES; else 2 MiB at 2 ranks, 1 MiB at
                           3-4, 256 KiB above), < 0 = never; ranks must agree */
  int ll_bytes;         /* AllReduce / AllGather buckets of at most this many bytes per rank take the LL one-shot
                           (flag-carrying 16-byte lines: no drain, no count atomic) when the arena is
                           uncached; same order, same bits.  0 = default (MCCS_LL_BYTES; else 128 KiB),
                           < 0 = never, at most 1 MiB; ranks must agree (appended in 0.3.1) */
  int reserved[16];     /* zero; room for later fields, so the struct keeps this size from 0.4 on
                           (init and setup refuse a config whose reserved words are not zero) */
} mccsCommConfig;

void mccsCommConfigDefault(mccsCommConfig *cfg);
/* sizeof(mccsCommConfig) as this library was built (see the ABI note above). */
size_t mccsCommConfigSize(void);
/* mccsCommConfigDefault for a caller that states its struct size: writes
 * nothing and returns mccsInvalidArgument unless `size` is this library's
 * sizeof(mccsCommConfig), so a caller built against another header can never
 * have bytes written past its struct. */
mccsResult_t mccsCommConfigDefaultSized(mccsCommConfig *cfg, size_t size);

/* One process drives `nranks` ranks (the reference service model: one mccs
 * process owns every GPU of the host).  devices[r] is rank r's GPU; devices
 * may repeat (several ranks on one GPU: their collectives must be issued
 * inside one mccsGroupStart/End so they run as one launch). */
mccsResult_t mccsCommInitAll(mccsComm_t *comms, int nranks, const int *devices, const mccsCommConfig *cfg);

/* One rank per process: SetupRank allocates this rank's FIFO arena and writes
 * a connect handle (IPC memory handle + layout, mccsConnectHandleSize()
 * bytes); the caller all-gathers the handles out of band (the reference's
 * bootstrap/exchange engines) and passes all nranks of them, concatenated in
 * rank order, to Connect. */
size_t mccsConnectHandleSize(void);
mccsResult_t mccsCommSetupRank(mccsComm_t *comm, int rank, int nranks, int device, const mccsCommConfig *cfg,
                               void *handle_out);
mccsResult_t mccsCommConnect(mccsComm_t comm, const void *all_handles);

/* libmccs::all_reduce (src/libmccs/src/collectives.rs:75-138): count in
 * elements of dtype, stream-ordered on `stream`, returns after launch.
 * A communicator's collectives run in the order they are issued, whatever
 * stream each is issued on (a launch on another stream than the comm's
 * previous one waits for it), as on the reference's one private comm stream.
 * Exception: a collective captured into a HIP graph runs when the graph is
 * replayed, and a replay makes no library call, so it is not ordered against
 * the comm's other launches by issue.  Instead every launch of a communicator,
 * replayed or not, takes the communicator's launch guard on the GPU before it
 * touches the comm's FIFO state, so two of its kernels never run at once: a
 * replay and a launch on another stream with no dependency between them run
 * one after the other, in either order.  Across processes each rank decides
 * that order on its own, so ranks whose replays race other launches of the
 * comm must order those streams themselves (a captured and an eager collective
 * of the same shape could otherwise pair up differently on different ranks).
 * A launch waiting for the guard keeps its workgroup slots: launches of one
 * comm pending together on different hardware queues whose grids exceed the
 * device's co-resident slots can stall until the watchdog (an error, never a
 * wrong sum).
 * Calls on ONE communicator must come from one thread at a time (group state
 * is per thread); different communicators may be driven from different
 * threads at once. */
mccsResult_t mccsAllReduce(const void *sendbuff, void *recvbuff, size_t count, int dtype, int op, mccsComm_t comm,
                           hipStream_t stream);
/* libmccs::all_gather: sendbytes per rank; recvbuff holds nranks*sendbytes. */
mccsResult_t mccsAllGather(const void *sendbuff, void *recvbuff, size_t sendbytes, mccsComm_t comm,
                           hipStream_t stream);
/* Group calls (ProxyCommand::GroupCall): collectives issued between Start and
 * End are planned together and launched at End (one launch per device). */
mccsResult_t mccsGroupStart(void);
mccsResult_t mccsGroupEnd(void);

/* Waits for the comm's stream and reports a device-side failure (watchdog
 * timeout / abort) as mccsTimeout / mccsRemoteError. */
mccsResult_t mccsCommSync(mccsComm_t comm);
/* Raises the comm's abortFlag: in-flight kernels exit at their next poll. */
mccsResult_t mccsCommAbort(mccsComm_t comm);
/* Frees the comm after its last launch completed; no barrier with the peers
 * is needed.  A peer's kernel may still post into this rank's FIFO arena after
 * this rank's own kernel finished, so the arena goes back to a per-process pool
 * but is handed to a new communicator only once every peer has destroyed its
 * side too (each peer's destroy writes a release word into the arena, after
 * its own kernels ended) or has exited: a peer process that never destroys
 * (it crashed, or its mccsCommConnect failed) stops being awaited once it has
 * exited and been reaped, where this process can see that (same host and pid
 * namespace); otherwise the arena stays pooled and unused. */
mccsResult_t mccsCommDestroy(mccsComm_t comm);
/* rank, nranks, device, channels, lanes, block threads, fifo memory kind
 * (MCCS_FIFO_*: the hand-off mode the comm's launches run). */
mccsResult_t mccsCommInfo(mccsComm_t comm, int *info7);
/* ring send order of channel ch (nranks ints). */
mccsResult_t mccsCommRing(mccsComm_t comm, int ch, int *order);
/* Algorithm of the comm's latest launch: MCCS_ALGO_RING, MCCS_ALGO_DIRECT
 * (two-shot), MCCS_ALGO_ONESHOT or MCCS_ALGO_LL (LL one-shot) (-1 before the first). */
#define MCCS_ALGO_RING 0
#define MCCS_ALGO_DIRECT 1
#define MCCS_ALGO_ONESHOT 2
#define MCCS_ALGO_LL 3
int mccsCommLastAlgo(mccsComm_t comm);
/* 1 when the comm may run the direct kernel: a direct region was configured
 * and every device of the communicator can perform atomics on every other's
 * memory (hipDevP2PAttrNativeAtomicSupported; the hand-off counts are remote
 * atomics).  Otherwise every AllReduce takes the ring, except buckets up to
 * ll_bytes, whose LL one-shot makes no remote atomics. */
int mccsCommDirectEnabled(mccsComm_t comm);
/* Node gate (connect-time self-test, run when a communicator spans two or
 * more GPUs; MCCS_GATE=0 skips it, MCCS_GATE=1 forces it): one exact-sum
 * AllReduce through the ring in its configured hand-off and through each
 * enabled direct variant, with every rank agreeing on the verdicts.  A wrong
 * ring sum steps every rank down uncached -> uncached + release -> cached
 * (system-scope fences); a wrong direct sum disables that variant.
 * info4[0] 1 if the gate ran, [1] the hand-off the comm now runs (MCCS_FIFO_*),
 * [2] MCCS_GATE_* bits that failed, [3] MCCS_GATE_* direct variants disabled. */
#define MCCS_GATE_RING_UNCACHED 0x1 /* ring, relaxed hand-off on uncached FIFOs */
#define MCCS_GATE_RING_RELEASE 0x2  /* ring, release fence before each post */
#define MCCS_GATE_RING_SYSTEM 0x4   /* ring, system-scope release/acquire (reference) */
#define MCCS_GATE_LL 0x8            /* LL one-shot */
#define MCCS_GATE_ONESHOT 0x10      /* one-shot */
#define MCCS_GATE_TWOSHOT 0x20      /* two-shot */
#define MCCS_GATE_NO_ATOMICS 0x40   /* some rank cannot perform peer atomics (direct kernel off) */
mccsResult_t mccsCommGateInfo(mccsComm_t comm, int *info4);
/* The comm's launch guard (inspection, tests): out4[0] the token of the launch
 * holding it (0 = free), [1] 1 once a fused launch holds every rank slot's
 * guard, [2] workgroups of the holder that have finished, [3] workgroups that
 * ever found it held by another launch of the comm and waited.  Copies from
 * device memory (synchronous). */
mccsResult_t mccsCommGuardInfo(mccsComm_t comm, uint64_t *out4);
/* 1 when this process's HIP runtime tells streams apart by hipStreamGetId,
 * 0 when by address (a runtime older than ROCm 7.1 loaded first, e.g. torch's).
 * The cross-stream issue order above keys on it. */
int mccs_stream_id_native(void);
/* Device pointer of the comm's mccsDevCommAndChannels (for inspection). */
mccsResult_t mccsCommDevComm(mccsComm_t comm, void **dev_comm);
const char *mccsGetErrorString(mccsResult_t r);
/* Diagnosis of the calling thread's latest failed library call: the step it
 * failed in, the failing runtime call and its hipError_t name and text, e.g.
 * "mccsCommSetupRank(rank 2/4, device 0) > comm_alloc_local > work FIFO:
 * HostMallocMapped -> hipErrorOutOfMemory (out of memory) at comm.cpp:318".
 * "" when the latest communicator / collective call succeeded (each one clears
 * it on entry).  The pointer stays valid until this thread's next library
 * call.  The reference returns one code per failure and logs the CUDA error
 * (cuda_warning!, src/mccs/src/utils/mod.rs:7-26); this adds where it failed. */
const char *mccsGetLastErrorString(void);
/* The hipError_t of that failure (0 when the failure was not a HIP call, e.g.
 * a refused argument or mismatched peers). */
int mccsGetLastHipError(void);
/* Ring timing counters of `device` (armed by MCCS_RING_PROFILE=1 at
 * communicator init): out4[0] slices, [1] ticks waiting for peer flags,
 * [2] ticks streaming + draining (s_memrealtime, 100 MHz), [3] reserved.
 * reset != 0 zeroes them after reading. */
mccsResult_t mccs_ring_profile(int device, unsigned long long *out4, int reset);

/* ----------------------------------------------------------------------
 * Application <-> backend bridge (the reference's mCCS service model: the
 * collectives run in a backend process; the application shares buffers and
 * stream order with it through IPC handles).  Handles are the 64-byte
 * hipIpcMemHandle_t / hipIpcEventHandle_t as opaque bytes.
 * ---------------------------------------------------------------------- */
#define MCCS_IPC_HANDLE_BYTES 64
/* libmccs cuda_malloc (src/libmccs/src/memory.rs:12-37): the backend
 * allocates and exports; the application opens the handle. */
mccsResult_t mccsMemAllocShared(int device, size_t bytes, void **dptr, void *handle_out);
mccsResult_t mccsMemFreeShared(int device, void *dptr);
mccsResult_t mccsMemOpenShared(int device, const void *handle, void **dptr);
mccsResult_t mccsMemCloseShared(int device, void *dptr);
/* libmccs register_stream (communicator.rs:47-66): the application creates an
 * interprocess event per stream; the backend opens it. */
mccsResult_t mccsEventCreateShared(int device, void **event, void *handle_out);
mccsResult_t mccsEventOpenShared(int device, const void *handle, void **event);
mccsResult_t mccsEventDestroyShared(void *event);
/* The comm's completion event (recorded after every launch) exported for the
 * application (InitCommunicator's event handle, communicator.rs:35-38). */
mccsResult_t mccsCommEventHandle(mccsComm_t comm, void *handle_out);
/* The comm's own stream, and wait_user_event (proxy/engine.rs:1185-1189):
 * the comm stream waits on an (opened) application event. */
mccsResult_t mccsCommStream(mccsComm_t comm, hipStream_t *stream);
mccsResult_t mccsCommWaitEvent(mccsComm_t comm, void *event);
/* Application side of the bridge (collectives.rs:86,134): record the user
 * event on its stream before a request; wait on the backend event after. */
mccsResult_t mccsEventRecordShared(void *event, hipStream_t stream);
mccsResult_t mccsStreamWaitShared(hipStream_t stream, void *event);

/* Host-only helpers (no GPU needed). */
/* BASELINE configs[0] plumbing: the same ring schedule and FIFO protocol run
 * by nranks x nchannels host threads over host memory (no GPU).  rings as in
 * mccsCommConfig (NULL = identity order on every channel). */
mccsResult_t mccs_host_ring_allreduce(int nranks, const void *const *sendbufs, void *const *recvbufs, size_t count,
                                      int dtype, int op, int nchannels, int nthreads_ref, int buff_size,
                                      const int *rings);
/* Default ring orders for an n-rank node (edge-disjoint Hamiltonian cycles,
 * both directions); writes up to max_channels x nranks ints, returns count. */
int mccs_default_rings(int nranks, int nch_req, int *out, int max_channels);
/* The library's default direct thresholds for an n-rank communicator (what
 * mccsCommConfig.oneshot_bytes / direct_bytes = 0 resolve to without the
 * MCCS_* overrides; -1 = off). */
void mccs_direct_defaults(int nranks, int *oneshot_bytes, int *direct_bytes);
/* mccsCommConfig.ll_bytes = 0 resolves to this (without the environment override). */
int mccs_ll_default(int nranks);
/* get_task_schema (plan.rs:602-635): channels and threads for total_bytes. */
void mccs_task_schema(size_t total_bytes, int nch_cfg, int *nch, int *nthreads);

/* Library identification. */
const char *mccs_hip_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MCCS_AMD_HIP_H_ */

// comm.h — host runtime of the MI355X mCCS ring path (internal).
//
// Mirrors the reference service objects on the hot path:
//   Communicator ........... src/mccs/src/comm/mod.rs:48-122 (+ proxy/init.rs)
//   CommDevResources ....... src/mccs/src/comm/device.rs:54-188
//   ring patterns .......... src/mccs/src/proxy/engine.rs:269-320
//   KernelPlan / schedule .. src/mccs/src/proxy/plan.rs:40-700
//   SHM connector .......... src/mccs/src/transport/shm/transporter.rs (replaced
//                            by an xGMI arena: FIFO data + flag lines in HBM)
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "mccs_devcomm.h"
#include "mccs_hip.h"
#include "ring_cfg.h"
#include "rt.h"

namespace mccs {

#define MCCS_LOG(...)                        \
  do {                                       \
    std::fprintf(stderr, "[mccs] " __VA_ARGS__); \
    std::fprintf(stderr, "\n");              \
  } while (0)

// ---- failure diagnosis (diag.cpp; mccsGetLastErrorString) -----------------
// A failing library call records, on the calling thread, the step it failed
// in (the stack of StepScope names open at the failure), the failing runtime
// call and its hipError_t.  The reference logs a CUDA failure and returns one
// code (cuda_warning!, utils/mod.rs:7-26); this keeps the same one code and
// adds where and why.
struct StepScope {
  explicit StepScope(std::string name);
  ~StepScope();
  StepScope(const StepScope&) = delete;
  StepScope& operator=(const StepScope&) = delete;
};
void err_clear();                                                    // at each API entry
void err_hip(const char* call, hipError_t e, const char* file, int line);  // a HIP / rt() call failed
void err_note(const char* file, int line, const char* fmt, ...) __attribute__((format(printf, 3, 4)));

// cuda_warning! equivalent (utils/mod.rs:7-26): record + log, then fail the call.
#define MCCS_HIP(call)                                  \
  do {                                                  \
    hipError_t _e = (call);                             \
    if (_e != hipSuccess) {                             \
      ::mccs::err_hip(#call, _e, __FILE__, __LINE__);   \
      return mccsUnhandledCudaError;                    \
    }                                                   \
  } while (0)

// A refused call (bad argument, mismatched peers): record why, then fail.
#define MCCS_FAIL(code, ...)                              \
  do {                                                    \
    ::mccs::err_note(__FILE__, __LINE__, __VA_ARGS__);    \
    return (code);                                        \
  } while (0)

#define MCCS_CHECK(call)                  \
  do {                                    \
    mccsResult_t _r = (call);             \
    if (_r != mccsSuccess) return _r;     \
  } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (rt().GetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)rt().SetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && rt().GetDevice(&cur) == hipSuccess && cur != prev) (void)rt().SetDevice(prev);
  }
};

// Per-rank FIFO arena layout (identical on every rank; offsets in bytes).
// [flags: nch x {send head lines, recv tail lines}] [data: nch x fifo_bytes]
// [direct region (64 KiB aligned), when direct_slot or oneshot_slot > 0:
//  control + the slots of the direct AllReduce (two-shot, one-shot, LL), ring_cfg.h]
// fifo_bytes = fifo_slots x buffer_size / 8 (slots of the reference step size)
struct ArenaLayout {
  int nch = 0;
  size_t buffer_size = 0;
  size_t fifo_bytes = 0;
  size_t direct_slot = 0;   // bytes of one two-shot in/out slot
  size_t oneshot_slot = 0;  // bytes of one one-shot slot
  size_t ll_slot = 0;       // bytes of one LL one-shot slot (2 x the LL bucket bytes)
  static constexpr size_t kLinesBytes = (size_t)MCCS_MAX_LANES * MCCS_FLAG_LINE_BYTES;  // 8 KiB
  // after the flag lines: one release word per rank (kMaxRanks), written by
  // that peer when it destroys its communicator (comm_free)
  static constexpr size_t kReleaseBytes = 64 * sizeof(uint64_t);
  size_t head_off(int c) const { return (size_t)c * 2 * kLinesBytes; }
  size_t tail_off(int c) const { return (size_t)c * 2 * kLinesBytes + kLinesBytes; }
  size_t release_off() const { return (size_t)nch * 2 * kLinesBytes; }
  size_t flags_bytes() const { return (release_off() + kReleaseBytes + 65535) & ~(size_t)65535; }
  size_t data_off(int c) const { return flags_bytes() + (size_t)c * fifo_bytes; }
  size_t ring_total() const { return flags_bytes() + (size_t)nch * fifo_bytes; }
  size_t direct_off() const { return (ring_total() + 65535) & ~(size_t)65535; }
  size_t total() const {
    return direct_slot || oneshot_slot || ll_slot
               ? direct_off() + MCCS_DIRECT_CTRL_BYTES + (size_t)MCCS_DIRECT_SLOTS * direct_slot +
                     2 * (size_t)MCCS_DIRECT_MAX_RANKS * (oneshot_slot + ll_slot)
               : ring_total();
  }
};

// Connect handle exchanged between processes (fixed size, POD).
struct ConnectHandle {
  uint32_t magic;
  int32_t rank, nranks, device;
  int32_t pid;
  int32_t fifo_memory;
  int32_t nch;
  int32_t lanes;       // this rank's lane count before the co-residency check
  int32_t lanes_auto;  // 1: lanes came from the automatic rule (cfg.lanes == 0)
  int32_t ring_cap;    // coresident_ring_blocks() of this rank's device
  uint64_t arena_bytes;
  uint64_t buffer_size;
  hipIpcMemHandle_t ipc;
  char host[64];
  // Everything both ends of a connection must agree on beyond the arena size
  // (thresholds that round to the same arena let ranks pick
  // different kernels for one call): the resolved direct thresholds, the FIFO
  // depth and the slice size.  Connect refuses any mismatch.
  int32_t direct_bytes, oneshot_bytes, ll_bytes;
  int32_t fifo_slots, slice_steps, block_threads;
  int32_t gate_env;  // MCCS_GATE as this rank read it (-1 unset): every rank must run the node gate or none
  // PCI bus id of the rank's GPU: device ordinals are local to a process
  // (HIP_VISIBLE_DEVICES), so co-location and peer lookups use this
  char pci[32];
  // this communicator's tenancy of the rank's FIFO arena: peers write it into
  // the arena's release word when they destroy their communicator
  uint64_t arena_epoch;
  // the rank's pid namespace (inode of /proc/self/ns/pid; 0 unknown): a peer's
  // pid names a process of this host only within the same namespace
  uint64_t pidns;
};
constexpr uint32_t kHandleMagic = 0x6d636373;  // "mccs"
// Default FIFO-wait watchdog (mccsCommConfig.timeout_ms = 0): 10 minutes,
// torch's default collective timeout.  A rank may reach a collective minutes
// before a peer (rank 0 writing a checkpoint while the others start the next
// step); the watchdog counts time without progress, so it must outlast that.
constexpr int kDefaultTimeoutMs = 600000;

struct WorkElemHost {
  uint8_t nWarps;
  const void* send;
  void* recv;
  size_t count;
  uint8_t bid, nChannels;
};

// One KernelWork (plan.rs): up to MCCS_MAX_WORK_ELEMENTS elements of one
// function, held inline so planning a launch allocates nothing.
struct HostWork {
  WorkElemHost e[MCCS_MAX_WORK_ELEMENTS];
  int n = 0;
  int func = 0;  // func id (for batching)
  size_t size() const { return (size_t)n; }
  const WorkElemHost& operator[](size_t i) const { return e[i]; }
};

struct ChannelSchedule {  // plan.rs ChanWorkSchedule
  size_t coll_bytes = 0;
  std::vector<HostWork> works;  // KernelWork list
  void reset() {                // after a launch: empty, capacity kept for the next
    coll_bytes = 0;
    works.clear();
  }
};

// Entries of a comm's graph work arena held by captured launches.  A
// captured launch takes a contiguous range, which returns when the graph that
// holds it is destroyed (rt().GraphOnDestroy), so graphs captured again and
// again reuse the arena.  Shared with those callbacks, which may run on a
// runtime thread after the comm is gone.
struct GraphWorkPool {
  std::mutex mu;
  std::map<uint32_t, uint32_t> free_ranges;  // start -> entries
  uint32_t held = 0;
  explicit GraphWorkPool(uint32_t entries) { free_ranges[0] = entries; }
  bool take(uint32_t n, uint32_t* start);  // first fit
  void give(uint32_t start, uint32_t n);   // coalescing
  uint32_t held_now() {
    std::lock_guard<std::mutex> lk(mu);
    return held;
  }
};

struct Comm {
  int rank = 0, nranks = 1, device = 0;
  mccsCommConfig cfg{};
  int nch = 0, lanes = 1, block_threads = 512;
  std::vector<std::vector<int>> rings;  // per channel send order
  ArenaLayout layout;
  // arena: own + mapped peers (index by rank); own_arena is peer_arena[rank]
  char* own_arena = nullptr;
  size_t own_arena_bytes = 0;  // the allocation (its size class), >= layout.total()
  bool own_arena_uncached = true;
  // Release protocol of the pooled arenas: this comm's tenancy of its own
  // arena (unique per process and comm), whether peers may hold or have held
  // it (exported / built into their device structures), and each peer's
  // tenancy, written back into that peer's arena at comm_free.
  uint64_t arena_epoch = 0;
  bool arena_shared = false;
  std::vector<uint64_t> peer_epoch;
  // each peer's pid where this process can tell whether it is alive (same
  // host and pid namespace; else 0): a dead peer's release is not awaited
  std::vector<int32_t> peer_pid;
  std::vector<char*> peer_arena;
  std::vector<bool> peer_opened_ipc;
  bool all_uncached = true;
  bool fifo_release = false;  // some rank asked for MCCS_FIFO_UNCACHED_RELEASE: release fence before posts
  // device resources (comm/device.rs)
  mccsDevCommAndChannels* d_comm = nullptr;
  std::vector<mccsDevChannelPeer*> d_peers;
  std::vector<int*> d_user_ranks;
  mccsRingConnView* d_view = nullptr;  // per channel, in d_comm's allocation after the channels
  mccsLaunchGuard* d_guard = nullptr;  // launch guard (launch_guard.h), in d_comm's allocation at MCCS_GUARD_OFF
  // The abort line (word 0 abortFlag, word 1 error bits) in host-mapped memory:
  // the host reads and writes it with plain CPU accesses (comm.cpp
  // place_abort_line), kernels through d_abort.
  uint32_t* d_abort = nullptr;
  uint32_t* h_abort = nullptr;
  // host-mapped work FIFO (comm/mod.rs MCCS_WORK_FIFO_DEPTH) + done counters
  mccsDevWork* h_work = nullptr;
  mccsDevWork* d_work = nullptr;
  uint32_t* h_done = nullptr;
  uint32_t* d_done = nullptr;
  uint32_t work_depth = 4096;
  // Work lists of launches captured into HIP graphs: a graph replays the
  // same kernel arguments forever, so its works cannot live in the rolling
  // FIFO (slots get reused).  Captured launches take entries from this
  // host-mapped arena (allocated at init: allocation is not allowed while a
  // stream captures) until their graph is destroyed.
  static constexpr uint32_t kGraphWorkEntries = 2048;
  mccsDevWork* h_graph_work = nullptr;
  mccsDevWork* d_graph_work = nullptr;
  std::shared_ptr<GraphWorkPool> graph_pool;
  uint32_t work_next = 0;      // work_queue_next_available
  uint32_t work_acked_min = 0; // work_queue_acked_min
  std::vector<uint32_t> chan_next;  // per channel work_queue_next_available
  // The comm stream (libmccs two-stream bridge) and the interprocess flavour
  // of the comm event are created on first need: a stream a process never
  // uses costs nothing, but every queue a process activates competes for the
  // GPU's hardware queues (ranks sharing one GPU measured 0.40 -> 0.62 ms
  // per 64 MiB AllReduce after one extra active queue per process).
  hipStream_t stream = nullptr;
  hipEvent_t event = nullptr;       // comm -> user
  bool event_ipc = false;           // event created with hipEventInterprocess
  // Whether the comm's latest launch recorded `event`.  A launch records it
  // only when something consumes it (the two-stream bridge, an exported
  // backend event, a work-FIFO launch whose acknowledgements the host may
  // wait on): each record is a marker packet behind the ring kernel, measured
  // at ~5 us of device time per call (2 processes, 32 KiB fp16: 16.5 vs
  // 11.6 us per AllReduce).  Without it mccsCommSync waits for the device.
  bool event_recorded = false;
  // When the latest launch did not record `event` but was fused with a comm
  // whose event it did record (rank slots k >= 1 of a fused launch): that
  // event, so mccsCommSync waits on this launch and not on the whole device
  // (a device-wide wait would also wait on other communicators' kernels that
  // spin on their peers: ADVICE r03).  Cleared when the owner is freed.
  // The owner's event is read at wait time (under the live-comm lock), so an
  // owner that replaces its event (comm_make_event_ipc) leaves no dangling copy.
  Comm* sync_owner = nullptr;
  // The stream the comm's latest launch went to (plan_launch_group orders a
  // launch on another stream after it).
  unsigned long long last_stream_id = 0;  // DeviceRuntime::StreamId of the latest launch's stream
  bool launched = false;
  // Threads synchronizing on this comm's event outside the live-comm lock
  // (comm_wait_last_launch): the event is not destroyed or replaced while > 0.
  std::atomic<int> waiters{0};
  hipEvent_t user_event = nullptr;  // user -> comm
  bool connected = false;
  bool failed = false;
  mccsRingKernelCfg kcfg{};  // hand-off policy of this comm's launches (launch arguments)
  // plan state
  std::vector<ChannelSchedule> sched;
  int plan_func = -1, plan_dtype = -1, plan_op = -1, plan_threads = 0;
  bool plan_pending = false;
  // direct AllReduce (direct_kernel.h): the pending call when the plan is one
  // AllReduce of at most cfg.direct_bytes / cfg.oneshot_bytes (plan.cpp)
  bool plan_direct = false;
  struct {
    const void* send;
    void* recv;
    size_t count;
  } direct{};
  int share = 1;         // ranks of this communicator on this rank's GPU (co-residency of spinning launches)
  // operator / test overrides read once at creation (make_comm), not per
  // launch: MCCS_INLINE_WORKS=0 (works always through the work FIFO) and
  // MCCS_DIRECT_BLOCKS (most workgroups per rank of a direct launch)
  bool inline_works = true;
  int direct_blocks = 128;
  // Every device of the communicator can perform atomics on every other's
  // memory (the direct kernel's hand-off counts are remote atomics); all ranks
  // derive it from the same device set, so they agree.
  bool direct_ok = false;
  int last_algo = -1;    // MCCS_ALGO_* of the latest launch
  int slice_steps = ALLREDUCE_CHUNKSTEPS;  // FIFO steps per ring slice (MCCS_SLICE_STEPS=2: the reference's 2)
  // node gate (gate.cpp): a hand-off mode the gate stepped down to (-1: none;
  // MCCS_FENCE_UNCACHED_RELEASE or MCCS_FENCE_SYSTEM), whether it ran, the
  // MCCS_GATE_* bits that failed and the direct variants it disabled
  int gate_fence = -1;
  bool gate_ran = false;
  unsigned gate_failed = 0, gate_disabled = 0;
};

// comm.cpp
bool devices_p2p_atomics(const std::vector<int>& devices);
mccsResult_t comm_alloc_local(Comm* c);
mccsResult_t comm_switch_to_device_arena(Comm* c);
mccsResult_t comm_build_device(Comm* c);
void default_rings(int nranks, int nch_req, std::vector<std::vector<int>>* rings);
mccsResult_t comm_free(Comm* c);
hipError_t comm_wait_last_launch(Comm* c);  // host wait for the comm's latest launch
// hipSuccess once the comm's latest launch finished (its event, or its fused
// launch owner's); hipErrorNotReady while it runs or when nothing recorded it.
hipError_t comm_query_last_launch(Comm* c);
// Makes stream `s` wait for the comm's latest launch (none recorded: no-op).
hipError_t comm_order_after_last_launch(Comm* c, hipStream_t s);
mccsResult_t comm_set_kernel_cfg(Comm* c);
mccsResult_t comm_stream(Comm* c, hipStream_t* out);  // creates the comm stream on first use
mccsResult_t comm_make_event_ipc(Comm* c);             // switches the comm event to an interprocess one
int comm_fifo_slots_of(const void* d_comm);            // fifo_slots of a live library comm's device struct, else 0
void comm_pool_drop_generation(unsigned generation);   // forgets arenas pooled under a removed fake runtime
mccsResult_t place_abort_line(Comm* c);     // the host-mapped abort line
int comm_pool_count(unsigned generation);    // arenas pooled under that runtime (tests)
int comm_pool_waiting(unsigned generation);  // pooled arenas still awaiting a peer's release (tests)
// gate.cpp
bool gate_wanted(bool distinct_gpus);
int gate_env();  // MCCS_GATE: -1 unset, else its value
mccsResult_t comm_gate(std::vector<Comm*>& cs, const std::vector<bool>& atomics_ok);
// plan.cpp
void plan_discard(Comm* c);  // drops the pending plan
mccsResult_t plan_enqueue(Comm* c, int func, int dtype, int op, const void* send, void* recv, size_t count);
mccsResult_t plan_launch_group(std::vector<Comm*>& comms, std::vector<hipStream_t>& user_streams);
// ring.hip
const void* ring_kernel_ptr(int func, int dtype, int op);
const void* ring_multi_kernel_ptr(int func, int dtype, int op);
int coresident_ring_blocks(int block, int device);
// direct.hip
const void* direct_kernel_ptr(int dtype, int op);
hipError_t ring_read_profile(unsigned long long* out, bool reset);
hipError_t ring_flush_caches(hipStream_t st);

}  // namespace mccs

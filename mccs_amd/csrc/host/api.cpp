// api.cpp — extern "C" communicator / collective API of libmccs_hip.so.
//
// The reference splits this across libmccs (app shim, src/libmccs/src/*.rs),
// the daemon relay and the proxy engine; here the app calls the planner
// directly (no daemon process on the hot path: the reference's WR/WC shared
// memory queues only relay the same arguments, collectives.rs:88-131).
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "comm.h"
#include "dtypes.h"

namespace mccs {
void task_schema(size_t total_bytes, int nch_cfg, int* nch_out, int* nthreads_out);

struct GroupState {
  int depth = 0;
  mccsResult_t error = mccsSuccess;  // first failure inside the group
  std::vector<Comm*> comms;
  std::vector<hipStream_t> streams;
};
static thread_local GroupState g_group;

// Drops every plan queued in the current group (error path).
static void group_discard() {
  for (Comm* c : g_group.comms) plan_discard(c);
  g_group.comms.clear();
  g_group.streams.clear();
}

// Direct AllReduce thresholds when the config leaves them 0 (MCCS_DIRECT_BYTES /
// MCCS_ONESHOT_BYTES override): buckets up to this many bytes per rank take
// the one-shot / two-shot kernel (bit-identical to the ring either way).
// Virtual node, graph replay, fp16 (profiles/r03_direct_vnode*.json): one-shot
// beat the ring to 2 MiB at n = 2, and beat two-shot to ~1 MiB at n = 3 / 4
// and to 512 KiB at n = 8; two-shot beat the ring to 2 MiB at n = 3 and to
// 8 MiB at n = 4 / 8 and only tied it at n = 2 (the ring is two hops there).  Over xGMI
// the ring's 2(n-1) sequential hops cost more than here, so these are
// conservative; the node's sweep (bench config.direct_sweep_fp16) refines them.
static int default_oneshot_bytes(int nranks) {
  return nranks == 2 ? 2 << 20 : nranks <= 4 ? 1 << 20 : 256 << 10;
}
static int default_direct_bytes(int nranks) { return nranks >= 4 ? 8 << 20 : nranks == 3 ? 4 << 20 : -1; }
// LL one-shot (ring_cfg.h): buckets whose hand-off round trips cost more than
// their bytes; its lines carry 8 data bytes per 16, so it stays small.
// Virtual node, graph replay, fp16 (profiles/r03_direct_ll_vnode.json): LL
// beat the one-shot at every n up to 128 KiB (n = 8: 32 KiB 15.1 -> 8.6 us,
// 128 KiB 22.0 -> 14.2; n = 2: 32 KiB 8.4 -> 5.0) and lost at n = 8 from
// 512 KiB.  Over xGMI its doubled line bytes cost link time
// (2 x 128 KiB per peer link ~ 4 us at ~64 GB/s, about the round trips it
// saves), so the default stays at 128 KiB for every n.
static int default_ll_bytes(int nranks) {
  (void)nranks;
  return 128 << 10;
}

static void fill_defaults(mccsCommConfig* c, int nranks) {
  if (c->buffer_size <= 0) c->buffer_size = 1 << 22;  // mccs.toml:19
  if (c->block_threads <= 0) c->block_threads = MCCS_RING_MAX_THREADS;
  if (c->work_fifo_depth <= 0) c->work_fifo_depth = 4096;
  // launch on the caller's stream (stream order is the same as libmccs's
  // user-event -> comm-stream -> backend-event bridge, without the ~10 us per
  // cross-stream wait measured on MI355X); 1 keeps the two-stream bridge
  if (c->bridge_streams == 0) c->bridge_streams = -1;
  // 16 slots: four 4-step slices in flight per lane instead of two (n = 8
  // virtual node +5 % at 128 MiB, +10 % at 16 MiB; n = 2 / 4 unchanged), more
  // bytes in flight per lane to cover an xGMI hop; 2 x the FIFO memory
  // (8 MiB per connection)
  if (c->fifo_slots == 0) c->fifo_slots = 2 * MCCS_BUFFER_SLOTS;
  if (c->direct_bytes == 0) c->direct_bytes = default_direct_bytes(nranks);
  if (c->oneshot_bytes == 0) c->oneshot_bytes = default_oneshot_bytes(nranks);
  if (c->ll_bytes == 0) c->ll_bytes = default_ll_bytes(nranks);
}

static mccsResult_t validate_cfg(const mccsCommConfig& c, int nranks) {
  StepScope st("config");
  // a chunk (buffer_size/2 bytes) must be a multiple of the largest thread
  // granule (512 x 8 B, all_reduce.h:34-35) so a rounded chunk fits 4 steps
  if (c.buffer_size < 8192 || c.buffer_size % 8192 != 0)
    MCCS_FAIL(mccsInvalidArgument, "buffer_size %d is not a multiple of 8192", c.buffer_size);
  // multiples of 32 keep the reference's nWarps*32 blocks (e.g. 544) valid;
  // at least one data wave next to the control wave (ring_kernel.h), like
  // the reference's smallest block (96 threads, plan.rs:602-635)
  if (c.block_threads < 96 || c.block_threads > MCCS_RING_MAX_THREADS || c.block_threads % 32)
    MCCS_FAIL(mccsInvalidArgument, "block_threads %d outside 96..%d or not a multiple of 32", c.block_threads,
              MCCS_RING_MAX_THREADS);
  if (c.lanes < 0 || c.lanes > MCCS_MAX_LANES) MCCS_FAIL(mccsInvalidArgument, "lanes %d outside 0..%d", c.lanes, MCCS_MAX_LANES);
  if (c.channel_count < 0 || c.channel_count > MCCS_MAX_NCHANNELS)
    MCCS_FAIL(mccsInvalidArgument, "channel_count %d outside 0..%d", c.channel_count, MCCS_MAX_NCHANNELS);
  if (c.work_fifo_depth & (c.work_fifo_depth - 1))
    MCCS_FAIL(mccsInvalidArgument, "work_fifo_depth %d is not a power of two", c.work_fifo_depth);
  if (c.locality != MCCS_LOCALITY_SENDER && c.locality != MCCS_LOCALITY_RECEIVER)
    MCCS_FAIL(mccsInvalidArgument, "locality %d unknown", c.locality);
  if (c.fifo_memory != MCCS_FIFO_UNCACHED && c.fifo_memory != MCCS_FIFO_DEVICE &&
      c.fifo_memory != MCCS_FIFO_UNCACHED_RELEASE)
    MCCS_FAIL(mccsInvalidArgument, "fifo_memory %d unknown", c.fifo_memory);
  if (nranks < 1 || nranks > 64) MCCS_FAIL(mccsInvalidArgument, "nranks %d outside 1..64", nranks);
  if (c.fifo_slots != 8 && c.fifo_slots != 16 && c.fifo_slots != 32)
    MCCS_FAIL(mccsInvalidArgument, "fifo_slots %d is not 8, 16 or 32", c.fifo_slots);
  // 9 slots of direct_bytes, 16 of oneshot_bytes and 16 of twice ll_bytes live in every rank's arena
  if (c.direct_bytes > (1 << 30)) MCCS_FAIL(mccsInvalidArgument, "direct_bytes %d above 1 GiB", c.direct_bytes);
  if (c.oneshot_bytes > (64 << 20)) MCCS_FAIL(mccsInvalidArgument, "oneshot_bytes %d above 64 MiB", c.oneshot_bytes);
  if (c.ll_bytes > (1 << 20)) MCCS_FAIL(mccsInvalidArgument, "ll_bytes %d above 1 MiB", c.ll_bytes);
  return mccsSuccess;
}

static mccsResult_t make_comm(int rank, int nranks, int device, const mccsCommConfig* user_cfg, Comm** out) {
  StepScope st("make_comm");
  mccsCommConfig cfg;
  mccsCommConfigDefault(&cfg);
  if (user_cfg) cfg = *user_cfg;
  for (int w : cfg.reserved)
    if (w != 0) MCCS_FAIL(mccsInvalidArgument, "a reserved config word is not zero");  // a field this library does not know
  fill_defaults(&cfg, nranks);
  MCCS_CHECK(validate_cfg(cfg, nranks));
  if (rank < 0 || rank >= nranks) MCCS_FAIL(mccsInvalidArgument, "rank %d outside 0..%d", rank, nranks - 1);
  int ndev = 0;
  MCCS_HIP(rt().GetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) MCCS_FAIL(mccsInvalidArgument, "device %d not visible (%d devices)", device, ndev);
  Comm* c = new Comm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  c->cfg = cfg;
  if (cfg.rings) {
    const int nch = cfg.channel_count > 0 ? cfg.channel_count : 1;
    for (int ch = 0; ch < nch; ++ch) {
      std::vector<int> r(cfg.rings + (size_t)ch * nranks, cfg.rings + (size_t)(ch + 1) * nranks);
      std::vector<int> s = r;
      std::sort(s.begin(), s.end());
      for (int i = 0; i < nranks; ++i)
        if (s[i] != i) {
          delete c;
          // not a permutation (engine.rs:274-279 asserts)
          MCCS_FAIL(mccsInvalidArgument, "rings[%d] is not a permutation of 0..%d", ch, nranks - 1);
        }
      c->rings.push_back(r);
    }
  } else {
    default_rings(nranks, cfg.channel_count, &c->rings);
  }
  c->cfg.rings = nullptr;  // not owned
  c->nch = (int)c->rings.size();
  if (const char* v = std::getenv("MCCS_SLICE_STEPS")) c->slice_steps = std::atoi(v) == 2 ? 2 : ALLREDUCE_CHUNKSTEPS;
  if (const char* v = std::getenv("MCCS_INLINE_WORKS")) c->inline_works = std::atoi(v) != 0;
  // (at most 4096: a launch guard counts a slot's workgroups in 16 bits)
  if (const char* v = std::getenv("MCCS_DIRECT_BLOCKS")) c->direct_blocks = std::atoi(v) > 0 ? std::min(std::atoi(v), 4096) : 128;
  c->block_threads = cfg.block_threads;
  // auto lanes: ~64 streaming workgroups per rank (128 at n = 2).  A lane's
  // throughput is bound by its per-slice latency chain (flag poll, loads,
  // store drain), not by bandwidth: the 2-rank virtual node at 128 MiB runs
  // 335 / 488 / 499 GB/s at 2 channels x 16 / 32 / 64 lanes and 754 at
  // 4 x 32 (comm.cpp default_rings); an 8-GPU rank must feed 7 links x
  // ~77 GB/s per direction (7 channels x 9 lanes).
  const int wgs = nranks == 2 ? 128 : 64;
  c->lanes = cfg.lanes > 0 ? cfg.lanes : (nranks == 1 ? 1 : std::max(1, std::min(MCCS_MAX_LANES, wgs / c->nch)));
  // every lane owns a >= 256-byte region of each 2-step slot pair (ring.hip)
  while (c->lanes > 1 && (size_t)cfg.buffer_size / MCCS_BUFFER_SLOTS * 2 / c->lanes < 256) {
    if (cfg.lanes > 0) {
      delete c;
      MCCS_FAIL(mccsInvalidArgument, "lanes %d leave under 256 bytes of a slot pair per lane", cfg.lanes);
    }
    c->lanes /= 2;
  }
  *out = c;
  return mccsSuccess;
}

static mccsResult_t enable_peer(int a, int b) {
  if (a == b) return mccsSuccess;
  StepScope st("peer access " + std::to_string(a) + " -> " + std::to_string(b));
  int can = 0;
  MCCS_HIP(rt().CanAccessPeer(&can, a, b));
  if (!can) MCCS_FAIL(mccsSystemError, "device %d cannot access device %d", a, b);
  DeviceGuard g(a);
  MCCS_HIP(rt().EnablePeerAccess(b));
  return mccsSuccess;
}

static mccsResult_t launch_single(Comm* c, int func, int dtype, int op, const void* send, void* recv, size_t count,
                                  hipStream_t stream) {
  // inside a group the diagnosis of a rejected call must survive to GroupEnd
  // (the group was cleared at GroupStart)
  if (g_group.depth == 0) err_clear();
  auto reject = [](mccsResult_t e, const char* why) {
    const bool first = g_group.depth == 0 || g_group.error == mccsSuccess;  // a group keeps its first failure
    if (g_group.depth > 0 && first) g_group.error = e;
    if (first) err_note(__FILE__, __LINE__, "%s", why);
    return e;
  };
  if (!c || !c->connected) return reject(mccsInvalidUsage, "the communicator is not connected");
  if (c->failed) return reject(mccsRemoteError, "the communicator failed earlier (watchdog or abort): destroy it");
  if (count == 0) return mccsSuccess;
  if (!send || !recv) return reject(mccsInvalidArgument, "null send or recv buffer");
  if (func == mccsFuncAllReduce && (dtype < 0 || dtype >= mccsNumTypes || op < 0 || op > mccsDevMin))
    return reject(mccsInvalidArgument, "unknown dtype or reduction op");
  if (std::find(g_group.comms.begin(), g_group.comms.end(), c) == g_group.comms.end()) {
    g_group.comms.push_back(c);
    g_group.streams.push_back(stream);
  }
  mccsResult_t er;
  {
    StepScope st(func == mccsFuncAllGather ? "mccsAllGather" : "mccsAllReduce");
    er = plan_enqueue(c, func, dtype, op, send, recv, count);
  }
  if (er != mccsSuccess) {
    if (g_group.depth == 0) group_discard();
    else if (g_group.error == mccsSuccess) g_group.error = er;
    return er;
  }
  if (g_group.depth == 0) {
    StepScope st(func == mccsFuncAllGather ? "mccsAllGather launch" : "mccsAllReduce launch");
    mccsResult_t r = plan_launch_group(g_group.comms, g_group.streams);
    group_discard();
    return r;
  }
  return mccsSuccess;
}

}  // namespace mccs

using namespace mccs;

extern "C" void mccsCommConfigDefault(mccsCommConfig* cfg) {
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->buffer_size = 1 << 22;
  // 8 data waves + the control wave (ring_kernel.h workgroup roles)
  cfg->block_threads = MCCS_RING_MAX_THREADS;
  // FIFO data lives with the receiver: the sender's stores cross xGMI as
  // posted writes and every read is local HBM (the reference SHM default was
  // Sender for host-pinned memory; both remain selectable)
  cfg->locality = MCCS_LOCALITY_RECEIVER;
  cfg->fifo_memory = MCCS_FIFO_UNCACHED;
  cfg->work_fifo_depth = 4096;
  cfg->bridge_streams = -1;
  // operator overrides (no rebuild needed): MCCS_LOCALITY=sender|receiver,
  // MCCS_LANES, MCCS_BLOCK_THREADS, MCCS_CHANNELS, MCCS_BUFFER_SIZE,
  // MCCS_BRIDGE_STREAMS, MCCS_FIFO_MEMORY=uncached|release|device,
  // MCCS_FIFO_SLOTS, MCCS_DIRECT_BYTES, MCCS_ONESHOT_BYTES, MCCS_TIMEOUT_MS
  if (const char* v = std::getenv("MCCS_LOCALITY"))
    cfg->locality = (v[0] == 's' || v[0] == 'S') ? MCCS_LOCALITY_SENDER : MCCS_LOCALITY_RECEIVER;
  if (const char* v = std::getenv("MCCS_LANES")) cfg->lanes = std::atoi(v);
  if (const char* v = std::getenv("MCCS_BRIDGE_STREAMS")) cfg->bridge_streams = std::atoi(v);
  if (const char* v = std::getenv("MCCS_FIFO_MEMORY"))
    cfg->fifo_memory = (v[0] == 'd' || v[0] == 'D')   ? MCCS_FIFO_DEVICE
                       : (v[0] == 'r' || v[0] == 'R') ? MCCS_FIFO_UNCACHED_RELEASE
                                                      : MCCS_FIFO_UNCACHED;
  if (const char* v = std::getenv("MCCS_BLOCK_THREADS")) cfg->block_threads = std::atoi(v);
  if (const char* v = std::getenv("MCCS_CHANNELS")) cfg->channel_count = std::atoi(v);
  if (const char* v = std::getenv("MCCS_BUFFER_SIZE")) cfg->buffer_size = std::atoi(v);
  if (const char* v = std::getenv("MCCS_FIFO_SLOTS")) cfg->fifo_slots = std::atoi(v);
  if (const char* v = std::getenv("MCCS_DIRECT_BYTES")) cfg->direct_bytes = std::atoi(v);
  if (const char* v = std::getenv("MCCS_ONESHOT_BYTES")) cfg->oneshot_bytes = std::atoi(v);
  if (const char* v = std::getenv("MCCS_LL_BYTES")) cfg->ll_bytes = std::atoi(v);
  if (const char* v = std::getenv("MCCS_TIMEOUT_MS")) cfg->timeout_ms = std::atoi(v);
}

extern "C" mccsResult_t mccsCommInitAll(mccsComm_t* comms, int nranks, const int* devices, const mccsCommConfig* cfg) {
  err_clear();
  StepScope st0("mccsCommInitAll(" + std::to_string(nranks) + " ranks)");
  if (!comms || !devices || nranks < 1) MCCS_FAIL(mccsInvalidArgument, "null comms/devices or nranks < 1");
  std::vector<Comm*> cs(nranks, nullptr);
  mccsResult_t r = mccsSuccess;
  for (int i = 0; i < nranks && r == mccsSuccess; ++i) {
    StepScope st("rank " + std::to_string(i));
    r = make_comm(i, nranks, devices[i], cfg, &cs[i]);
  }
  // ranks sharing a GPU run as one fused launch that must be co-resident:
  // shrink automatic lanes to fit (explicit lanes are checked at launch)
  for (int i = 0; i < nranks && r == mccsSuccess; ++i) {
    Comm* c = cs[i];
    int share = 0;
    for (int j = 0; j < nranks; ++j) share += devices[j] == devices[i];
    c->share = share;
    if (share < 2 || c->cfg.lanes > 0) continue;
    const int cap = coresident_ring_blocks(c->block_threads, c->device);
    const int fit = cap / (share * c->nch);
    if (fit < 1) {
      err_note(__FILE__, __LINE__, "%d ranks x %d channels do not fit %d co-resident workgroups on device %d", share,
               c->nch, cap, c->device);
      r = mccsInvalidUsage;
    } else {
      c->lanes = std::min(c->lanes, fit);
    }
  }
  for (int i = 0; i < nranks && r == mccsSuccess; ++i) {
    StepScope st("rank " + std::to_string(i));
    r = comm_alloc_local(cs[i]);
  }
  for (int i = 0; i < nranks && r == mccsSuccess; ++i)
    for (int j = 0; j < nranks && r == mccsSuccess; ++j) r = enable_peer(devices[i], devices[j]);
  if (r == mccsSuccess)  // every rank's arena is every peer's to write (released at comm_free)
    for (int i = 0; i < nranks; ++i) {
      cs[i]->arena_shared = nranks > 1;
      for (int j = 0; j < nranks; ++j) cs[i]->peer_epoch[j] = j == i ? 0 : cs[j]->arena_epoch;
    }
  if (r == mccsSuccess) {
    bool all_uc = true, release = false;
    for (int i = 0; i < nranks; ++i) {
      all_uc = all_uc && cs[i]->own_arena_uncached;
      release = release || cs[i]->cfg.fifo_memory == MCCS_FIFO_UNCACHED_RELEASE;
    }
    const bool atomics = devices_p2p_atomics(std::vector<int>(devices, devices + nranks));
    for (int i = 0; i < nranks; ++i) {
      for (int j = 0; j < nranks; ++j) cs[i]->peer_arena[j] = cs[j]->own_arena;
      cs[i]->all_uncached = all_uc;
      cs[i]->fifo_release = release;
      cs[i]->direct_ok = atomics;
    }
    for (int i = 0; i < nranks && r == mccsSuccess; ++i) {
      StepScope st("rank " + std::to_string(i));
      r = comm_build_device(cs[i]);
    }
    // node gate: one process sees every rank, so the host combines their verdicts
    bool distinct = false;
    for (int i = 1; i < nranks; ++i) distinct = distinct || devices[i] != devices[0];
    if (r == mccsSuccess && nranks > 1 && gate_wanted(distinct)) {
      StepScope st("node gate");
      std::vector<bool> atomics_ok(nranks, atomics);
      r = comm_gate(cs, atomics_ok);
    }
  }
  if (r != mccsSuccess) {
    for (auto c : cs)
      if (c) {
        comm_free(c);
        delete c;
      }
    return r;
  }
  for (int i = 0; i < nranks; ++i) comms[i] = (mccsComm_t)cs[i];
  return mccsSuccess;
}

// This process's pid namespace (the inode of /proc/self/ns/pid), 0 if unknown.
static uint64_t pid_namespace() {
  struct stat st;
  return stat("/proc/self/ns/pid", &st) == 0 ? (uint64_t)st.st_ino : 0;
}

// Two connect handles name the same GPU: same host and PCI bus id (ordinals
// are local to a process, so they would match across different GPUs).
static bool same_gpu(const ConnectHandle& a, const ConnectHandle& b) {
  return std::strncmp(a.host, b.host, sizeof(a.host)) == 0 && std::strncmp(a.pci, b.pci, sizeof(a.pci)) == 0;
}

extern "C" size_t mccsConnectHandleSize(void) { return sizeof(ConnectHandle); }

// Exports the comm's FIFO arena for its peers.  An uncached arena whose
// export is refused falls back to a plain device arena (system fences).
static mccsResult_t export_arena(Comm* c, hipIpcMemHandle_t* h) {
  StepScope st("IPC export of the FIFO arena");
  DeviceGuard g(c->device);
  hipError_t e = rt().IpcGetMemHandle(h, c->own_arena);
  if (e == hipSuccess || !c->own_arena_uncached) {
    MCCS_HIP(e);
    return mccsSuccess;
  }
  MCCS_LOG("hipIpcGetMemHandle(uncached arena): %s; retrying with hipMalloc", hipGetErrorString(e));
  MCCS_CHECK(comm_switch_to_device_arena(c));
  MCCS_HIP(rt().IpcGetMemHandle(h, c->own_arena));
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommSetupRank(mccsComm_t* out, int rank, int nranks, int device, const mccsCommConfig* cfg,
                                          void* handle_out) {
  err_clear();
  StepScope st0("mccsCommSetupRank(rank " + std::to_string(rank) + "/" + std::to_string(nranks) + ", device " +
                std::to_string(device) + ")");
  if (!out || !handle_out) MCCS_FAIL(mccsInvalidArgument, "null comm or handle pointer");
  Comm* c = nullptr;
  MCCS_CHECK(make_comm(rank, nranks, device, cfg, &c));
  ConnectHandle h;
  std::memset(&h, 0, sizeof(h));
  mccsResult_t r = comm_alloc_local(c);
  if (r == mccsSuccess) r = export_arena(c, &h.ipc);
  if (r != mccsSuccess) {
    comm_free(c);
    delete c;
    return r;
  }
  c->arena_shared = nranks > 1;  // exported: any peer may map it from now on
  h.arena_epoch = c->arena_epoch;
  h.magic = kHandleMagic;
  h.rank = rank;
  h.nranks = nranks;
  h.device = device;
  h.pid = (int32_t)getpid();
  h.pidns = pid_namespace();
  h.fifo_memory = !c->own_arena_uncached                              ? MCCS_FIFO_DEVICE
                  : c->cfg.fifo_memory == MCCS_FIFO_UNCACHED_RELEASE ? MCCS_FIFO_UNCACHED_RELEASE
                                                                     : MCCS_FIFO_UNCACHED;
  h.nch = c->nch;
  h.lanes = c->lanes;
  h.lanes_auto = c->cfg.lanes > 0 ? 0 : 1;
  h.ring_cap = coresident_ring_blocks(c->block_threads, device);
  h.arena_bytes = c->layout.total();
  h.buffer_size = c->layout.buffer_size;
  h.direct_bytes = c->cfg.direct_bytes;
  h.oneshot_bytes = c->cfg.oneshot_bytes;
  h.ll_bytes = c->cfg.ll_bytes;
  h.fifo_slots = c->cfg.fifo_slots;
  h.slice_steps = c->slice_steps;
  h.block_threads = c->block_threads;
  h.gate_env = gate_env();
  if (rt().DeviceGetPCIBusId(h.pci, sizeof(h.pci) - 1, device) != hipSuccess)
    std::snprintf(h.pci, sizeof(h.pci), "ordinal:%d", device);
  gethostname(h.host, sizeof(h.host) - 1);
  std::memcpy(handle_out, &h, sizeof(h));
  *out = (mccsComm_t)c;
  return mccsSuccess;
}

// Why rank r's handle cannot join this communicator ("" if it can).
static std::string handle_mismatch(const Comm* c, const ConnectHandle& h, const ConnectHandle& mine, int r) {
  char b[200];
  auto diff = [&](const char* what, long long theirs, long long ours) {
    std::snprintf(b, sizeof(b), "rank %d's %s %lld differs from this rank's %lld", r, what, theirs, ours);
    return std::string(b);
  };
  if (h.magic != kHandleMagic) return "rank " + std::to_string(r) + "'s handle is not a connect handle";
  if (h.rank != r) return diff("handle rank", h.rank, r);
  if (h.nranks != c->nranks) return diff("nranks", h.nranks, c->nranks);
  if (h.nch != c->nch) return diff("channel count", h.nch, c->nch);
  if (h.arena_bytes != c->layout.total()) return diff("arena bytes", (long long)h.arena_bytes, (long long)c->layout.total());
  if (h.buffer_size != c->layout.buffer_size) return diff("buffer_size", (long long)h.buffer_size, (long long)c->layout.buffer_size);
  // ... or on which kernel / slice shape a call takes (both ends of every
  // connection must run the same one: ADVICE r03)
  if (h.direct_bytes != c->cfg.direct_bytes) return diff("direct_bytes", h.direct_bytes, c->cfg.direct_bytes);
  if (h.oneshot_bytes != c->cfg.oneshot_bytes) return diff("oneshot_bytes", h.oneshot_bytes, c->cfg.oneshot_bytes);
  if (h.ll_bytes != c->cfg.ll_bytes) return diff("ll_bytes", h.ll_bytes, c->cfg.ll_bytes);
  if (h.fifo_slots != c->cfg.fifo_slots) return diff("fifo_slots", h.fifo_slots, c->cfg.fifo_slots);
  if (h.slice_steps != c->slice_steps) return diff("slice steps", h.slice_steps, c->slice_steps);
  if (h.block_threads != c->block_threads) return diff("block_threads", h.block_threads, c->block_threads);
  // the node gate's collectives need every rank (a rank that skipped it
  // would leave the others in its vote until the watchdog)
  if (h.gate_env != mine.gate_env) return diff("MCCS_GATE", h.gate_env, mine.gate_env);
  return "";
}

extern "C" mccsResult_t mccsCommConnect(mccsComm_t comm, const void* all_handles) {
  err_clear();
  Comm* c = (Comm*)comm;
  if (!c || !all_handles || c->connected) {
    StepScope st0("mccsCommConnect");
    MCCS_FAIL(mccsInvalidUsage, "null comm or handles, or the comm is already connected");
  }
  StepScope st0("mccsCommConnect(rank " + std::to_string(c->rank) + "/" + std::to_string(c->nranks) + ")");
  const ConnectHandle* hs = (const ConnectHandle*)all_handles;
  bool all_uc = true, release = false;
  {
    StepScope st("handle check");
    // A refused handle set is refused by every rank: each compares every
    // handle with its own and with rank 0's, and any disagreement between two
    // ranks shows up at every rank.  So no rank goes on to map this rank's
    // arena, and it need not wait for peers' release words when it is
    // destroyed (a service retrying failed connects lost one FIFO
    // arena per attempt on every rank).  Failures after this point keep the
    // wait: a peer past its own check may have mapped the arena, and its ring
    // sender writes up to fifo_slots steps into it before any credit.
    auto refuse = [&](const char* why) {
      c->arena_shared = false;
      err_note(__FILE__, __LINE__, "%s", why);
      return mccsInvalidArgument;
    };
    for (int r = 0; r < c->nranks; ++r) {
      const ConnectHandle& h = hs[r];
      const std::string why = handle_mismatch(c, h, hs[c->rank], r);
      // ranks disagree on the communicator profile
      if (!why.empty()) return refuse(why.c_str());
      all_uc = all_uc && h.fifo_memory != MCCS_FIFO_DEVICE;
      release = release || h.fifo_memory == MCCS_FIFO_UNCACHED_RELEASE;
      if (h.lanes != hs[0].lanes || h.lanes_auto != hs[0].lanes_auto) {
        char b[160];
        std::snprintf(b, sizeof(b), "rank %d's lanes %d (auto %d) differ from rank 0's %d (auto %d)", r, h.lanes,
                      h.lanes_auto, hs[0].lanes, hs[0].lanes_auto);
        return refuse(b);
      }
    }
    // From here a peer may map this rank's arena, so its destroy awaits every
    // peer's release word -- or, for a peer whose exit this process can see
    // (same host and pid namespace), that peer's exit: a peer that crashed, or
    // whose Connect failed before it mapped the arena, never writes the word
    // (ADVICE r05), and once it has exited none of its kernels can write here.
    const ConnectHandle& me = hs[c->rank];
    c->peer_pid.assign(c->nranks, 0);
    for (int r = 0; r < c->nranks; ++r)
      if (r != c->rank && hs[r].pidns && hs[r].pidns == me.pidns && hs[r].pid > 0 &&
          std::strncmp(hs[r].host, me.host, sizeof(me.host)) == 0)
        c->peer_pid[r] = hs[r].pid;
  }
  // Ranks of this communicator that share a GPU as separate processes run
  // separate launches that spin on each other's flags, so all of them must be
  // resident together.  Unlike one fused launch (mccsCommInitAll), the GPU
  // does not co-schedule separate processes' grids as a unit (4 processes x
  // 60 workgroups = 240 of 256 slots timed out on MI355X), so automatic lanes
  // shrink to half the slots; explicit lanes that cannot fit at all are
  // refused instead of deadlocking.  Every rank derives the same lane count
  // from the same handles (a connection's two ends must agree on lanes).
  {
    StepScope st("co-residency");
    int max_share = 1, cap = 1 << 30;
    for (int r = 0; r < c->nranks; ++r) {
      int share = 0;
      for (int q = 0; q < c->nranks; ++q) share += same_gpu(hs[q], hs[r]);
      max_share = std::max(max_share, share);
      if (hs[r].ring_cap > 0) cap = std::min(cap, (int)hs[r].ring_cap);
    }
    c->share = max_share;
    if (max_share > 1 && cap < (1 << 30)) {
      if (hs[0].lanes_auto) {
        const int fit = cap / 2 / (max_share * c->nch);
        if (fit < 1)
          MCCS_FAIL(mccsInvalidUsage, "%d ranks x %d channels per GPU do not fit half of %d workgroup slots", max_share,
                    c->nch, cap);
        c->lanes = std::min(c->lanes, fit);
      } else if ((long)max_share * c->nch * c->lanes > cap) {
        MCCS_FAIL(mccsInvalidUsage, "%d ranks x %d channels x %d lanes per GPU exceed %d workgroup slots", max_share,
                  c->nch, c->lanes, cap);
      }
    }
  }
  DeviceGuard g(c->device);
  for (int r = 0; r < c->nranks; ++r) {
    if (r == c->rank) continue;
    StepScope st("IPC open of rank " + std::to_string(r) + "'s arena");
    const ConnectHandle& h = hs[r];
    if (h.pid == (int32_t)getpid())  // same process: use mccsCommInitAll
      MCCS_FAIL(mccsInvalidUsage, "rank %d is in this process (pid %d): use mccsCommInitAll", r, (int)h.pid);
    int peer_dev = -1;  // the peer's GPU as this process numbers it
    if (rt().DeviceGetByPCIBusId(&peer_dev, h.pci) != hipSuccess) peer_dev = -1;
    if (peer_dev >= 0 && enable_peer(c->device, peer_dev) != mccsSuccess)
      err_clear();  // best effort; IPC maps regardless
    void* p = nullptr;
    MCCS_HIP(rt().IpcOpenMemHandle(&p, h.ipc));
    c->peer_arena[r] = (char*)p;
    c->peer_opened_ipc[r] = true;
    c->peer_epoch[r] = h.arena_epoch;
  }
  c->all_uncached = all_uc;
  c->fifo_release = release;
  // Peer atomics as THIS process sees them: every peer's GPU looked up by PCI
  // bus id (ordinals are per process).  A peer GPU this process cannot see,
  // or cannot do atomics on, turns the count-based direct variants off here;
  // the node gate's vote then turns them off on every rank alike.
  bool atomics = true, distinct = false;
  for (int r = 0; r < c->nranks; ++r) {
    if (same_gpu(hs[r], hs[c->rank])) continue;
    distinct = true;
    int dev = -1, ok = 0;
    if (rt().DeviceGetByPCIBusId(&dev, hs[r].pci) != hipSuccess || dev < 0) atomics = false;
    else if (rt().P2PAtomics(&ok, c->device, dev) != hipSuccess || !ok) atomics = false;
  }
  c->direct_ok = atomics;
  {
    StepScope st("device structures");
    MCCS_CHECK(comm_build_device(c));
  }
  if (gate_wanted(distinct)) {
    StepScope st("node gate");
    std::vector<Comm*> cs{c};
    mccsResult_t r = comm_gate(cs, std::vector<bool>{atomics});
    if (r != mccsSuccess) {
      c->connected = false;  // the caller destroys it; no collective may run on it
      return r;
    }
  } else if (distinct) {
    // no gate, no vote: keep the count-based direct variants only where every
    // rank can be trusted to decide alike (they cannot tell without a vote)
    c->direct_ok = false;
  }
  return mccsSuccess;
}

extern "C" mccsResult_t mccsAllReduce(const void* sendbuff, void* recvbuff, size_t count, int dtype, int op,
                                      mccsComm_t comm, hipStream_t stream) {
  return launch_single((Comm*)comm, mccsFuncAllReduce, dtype, op, sendbuff, recvbuff, count, stream);
}

extern "C" mccsResult_t mccsAllGather(const void* sendbuff, void* recvbuff, size_t sendbytes, mccsComm_t comm,
                                      hipStream_t stream) {
  return launch_single((Comm*)comm, mccsFuncAllGather, mccsInt8, mccsDevSum, sendbuff, recvbuff, sendbytes, stream);
}

extern "C" mccsResult_t mccsGroupStart(void) {
  if (g_group.depth++ == 0) err_clear();
  return mccsSuccess;
}

extern "C" mccsResult_t mccsGroupEnd(void) {
  if (g_group.depth <= 0) {
    err_clear();
    MCCS_FAIL(mccsInvalidUsage, "mccsGroupEnd without mccsGroupStart");
  }
  if (--g_group.depth > 0) return mccsSuccess;
  if (g_group.error != mccsSuccess) {  // a collective of the group was rejected: launch none
    const mccsResult_t e = g_group.error;
    g_group.error = mccsSuccess;
    group_discard();
    return e;
  }
  StepScope st("mccsGroupEnd launch");
  mccsResult_t r = plan_launch_group(g_group.comms, g_group.streams);
  group_discard();  // plans not launched after an error are dropped, not left queued
  return r;
}

extern "C" mccsResult_t mccsCommSync(mccsComm_t comm) {
  err_clear();
  StepScope st0("mccsCommSync");
  Comm* c = (Comm*)comm;
  if (!c) return mccsInvalidArgument;
  DeviceGuard g(c->device);
  // the latest launch recorded the comm event only if something consumes it
  // (plan.cpp); else the event of the comm it was fused with; else wait for
  // every stream of the device, a superset
  MCCS_HIP(comm_wait_last_launch(c));
  if (c->stream) MCCS_HIP(rt().StreamSynchronize(c->stream));
  // the communicator's abort line: word 0 abortFlag, word 1 the error bits its
  // kernels reported (ring_cfg.h), so another communicator's failure never
  // shows up here
  const uint32_t abort_val = __atomic_load_n(c->h_abort, __ATOMIC_ACQUIRE);
  const uint32_t err = __atomic_load_n(c->h_abort + 1, __ATOMIC_ACQUIRE);
  if (err || abort_val) c->failed = true;
  if (err & MCCS_ERR_TIMEOUT)
    MCCS_FAIL(mccsTimeout, "rank %d: a FIFO wait passed the %d ms watchdog (error bits 0x%x)", c->rank,
              c->cfg.timeout_ms == 0 ? kDefaultTimeoutMs : c->cfg.timeout_ms, err);
  if (err || abort_val) MCCS_FAIL(mccsRemoteError, "rank %d: abortFlag %u, error bits 0x%x", c->rank, abort_val, err);
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommAbort(mccsComm_t comm) {
  Comm* c = (Comm*)comm;
  if (!c) return mccsInvalidArgument;
  c->failed = true;
  // a CPU store into the host-mapped line: no stream, so nothing can queue it
  // behind the kernel it must stop (comm.cpp place_abort_line)
  if (c->h_abort) __atomic_store_n(c->h_abort, 1u, __ATOMIC_SEQ_CST);
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommDestroy(mccsComm_t comm) {
  Comm* c = (Comm*)comm;
  if (!c) return mccsInvalidArgument;
  comm_free(c);
  delete c;
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommInfo(mccsComm_t comm, int* info) {
  Comm* c = (Comm*)comm;
  if (!c || !info) return mccsInvalidArgument;
  info[0] = c->rank;
  info[1] = c->nranks;
  info[2] = c->device;
  info[3] = c->nch;
  info[4] = c->lanes;
  info[5] = c->block_threads;
  // the hand-off the launches run (after any node-gate step-down)
  info[6] = c->kcfg.fence_mode == MCCS_FENCE_SYSTEM             ? MCCS_FIFO_DEVICE
            : c->kcfg.fence_mode == MCCS_FENCE_UNCACHED_RELEASE ? MCCS_FIFO_UNCACHED_RELEASE
                                                                : MCCS_FIFO_UNCACHED;
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommRing(mccsComm_t comm, int ch, int* order) {
  Comm* c = (Comm*)comm;
  if (!c || !order || ch < 0 || ch >= c->nch) return mccsInvalidArgument;
  for (int i = 0; i < c->nranks; ++i) order[i] = c->rings[ch][i];
  return mccsSuccess;
}

extern "C" int mccsCommLastAlgo(mccsComm_t comm) {
  const Comm* c = (const Comm*)comm;
  return c ? c->last_algo : -1;
}

extern "C" int mccsCommDirectEnabled(mccsComm_t comm) {
  const Comm* c = (const Comm*)comm;
  return c && c->direct_ok && (c->layout.direct_slot > 0 || c->layout.oneshot_slot > 0 || c->layout.ll_slot > 0);
}

extern "C" mccsResult_t mccsCommGuardInfo(mccsComm_t comm, uint64_t* out4) {
  Comm* c = (Comm*)comm;
  if (!c || !out4 || !c->d_guard) return mccsInvalidArgument;
  DeviceGuard g(c->device);
  mccsLaunchGuard line;
  MCCS_HIP(rt().Memcpy(&line, c->d_guard, sizeof(line), hipMemcpyDeviceToHost));
  out4[0] = line.word >> MCCS_GUARD_TOK_SHIFT;
  out4[1] = (line.word & MCCS_GUARD_CONFIRMED) ? 1 : 0;
  out4[2] = line.word & MCCS_GUARD_FIN_MASK;
  out4[3] = line.waits;
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommDevComm(mccsComm_t comm, void** dev_comm) {
  Comm* c = (Comm*)comm;
  if (!c || !dev_comm) return mccsInvalidArgument;
  *dev_comm = c->d_comm;
  return mccsSuccess;
}

extern "C" const char* mccsGetErrorString(mccsResult_t r) {
  switch (r) {
    case mccsSuccess: return "no error";
    case mccsUnhandledCudaError: return "unhandled HIP error";
    case mccsSystemError: return "system error";
    case mccsInternalError: return "internal error";
    case mccsInvalidArgument: return "invalid argument";
    case mccsInvalidUsage: return "invalid usage";
    case mccsRemoteError: return "remote process exited or the kernel aborted";
    case mccsInProgress: return "in progress";
    case mccsTimeout: return "FIFO watchdog timeout";
    default: return "unknown result";
  }
}

// Pure host helpers, usable without a GPU (tests, tools).
extern "C" int mccs_default_rings(int nranks, int nch_req, int* out, int max_channels) {
  std::vector<std::vector<int>> rings;
  default_rings(nranks, nch_req, &rings);
  int n = std::min((int)rings.size(), max_channels);
  for (int c = 0; c < n; ++c)
    for (int i = 0; i < nranks; ++i) out[c * nranks + i] = rings[c][i];
  return n;
}

extern "C" int mccs_ll_default(int nranks) { return default_ll_bytes(nranks); }

extern "C" void mccs_direct_defaults(int nranks, int* oneshot_bytes, int* direct_bytes) {
  if (oneshot_bytes) *oneshot_bytes = default_oneshot_bytes(nranks);
  if (direct_bytes) *direct_bytes = default_direct_bytes(nranks);
}

extern "C" void mccs_task_schema(size_t total_bytes, int nch_cfg, int* nch, int* nthreads) {
  task_schema(total_bytes, nch_cfg, nch, nthreads);
}

// Ring profile counters of `device` (MCCS_RING_PROFILE=1 at communicator
// init arms them): out[0] slices, out[1] wait ticks, out[2] work ticks
// (s_memrealtime, 100 MHz), out[3] reserved.
extern "C" mccsResult_t mccs_ring_profile(int device, unsigned long long* out4, int reset) {
  if (!out4) return mccsInvalidArgument;
  DeviceGuard g(device);
  MCCS_HIP(ring_read_profile(out4, reset != 0));
  return mccsSuccess;
}

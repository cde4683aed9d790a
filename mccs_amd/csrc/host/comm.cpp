// comm.cpp — communicator resources, ring patterns and xGMI FIFO connectors.
//
// Reference counterparts:
//   ring user_ranks / index ..... src/mccs/src/proxy/engine.rs:269-320
//   CommDevResources::new ....... src/mccs/src/comm/device.rs:81-183
//   conn_info_to_dev ............ src/mccs/src/comm/device.rs:35-52
//   SHM connector setup ......... src/mccs/src/transport/shm/transporter.rs:49-183
// The SHM connector's host-pinned FIFO (cudaHostRegister'd, PCIe) is replaced
// by one per-rank HBM arena holding, per channel, the FIFO data of one
// connection and the head/tail flag lines; peers reach it over xGMI through
// peer access (same process) or IPC (one rank per process).
#include <hip/hip_runtime.h>
#include <sched.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <mutex>

#include "comm.h"

namespace mccs {

// ---------------------------------------------------------------------------
// Ring patterns.  Default topology for one fully connected MI355X node:
//   n = 8: 7 arc-disjoint directed Hamiltonian cycles (every GPU sends and
//          receives on all 7 of its xGMI links, one ring per link and
//          direction);
//   n = 4: all 6 directed Hamiltonian cycles (each link carries two);
//   other n: edge-disjoint Hamiltonian cycles of K_n (greedy DFS,
//          deterministic so every rank derives the same rings), each used in
//          both directions: n-2 or n-1 of a GPU's n-1 links;
//   n = 2: the one ring, 4 channels of it (below).
static bool ham_dfs(int n, std::vector<std::vector<char>>& used, std::vector<int>& path,
                    std::vector<char>& seen) {
  if ((int)path.size() == n) return !used[path.back()][path[0]];
  const int u = path.back();
  for (int k = 1; k < n; ++k) {
    const int v = (u + k) % n;  // rotate neighbour order: spreads early cycles
    if (seen[v] || used[u][v]) continue;
    seen[v] = 1;
    path.push_back(v);
    if (ham_dfs(n, used, path, seen)) return true;
    path.pop_back();
    seen[v] = 0;
  }
  return false;
}

void default_rings(int n, int nch_req, std::vector<std::vector<int>>* rings) {
  rings->clear();
  std::vector<std::vector<int>> base;
  if (n <= 2) {
    std::vector<int> r(n);
    for (int i = 0; i < n; ++i) r[i] = i;
    base.push_back(r);
  } else if (n == 8) {
    // The complete symmetric digraph on 8 vertices splits into 7 arc-disjoint
    // directed Hamiltonian cycles (Tillson 1980: K_n* does for every n except
    // 4 and 6; these 7 were found by search and are checked arc-disjoint in
    // tests/test_ring_host.py).  Every GPU then sends on all 7 of its xGMI
    // links and receives on all 7, where both directions of 3 undirected
    // cycles (the n != 8 construction below) leave one link per GPU idle.
    base = {{0, 5, 6, 3, 7, 2, 1, 4}, {0, 4, 2, 3, 5, 7, 1, 6}, {0, 3, 2, 7, 5, 4, 6, 1}, {0, 7, 6, 2, 4, 1, 5, 3},
            {0, 6, 7, 4, 3, 1, 2, 5}, {0, 2, 6, 5, 1, 3, 4, 7}, {0, 1, 7, 3, 6, 4, 5, 2}};
  } else if (n == 4) {
    // K4 has no two edge-disjoint Hamiltonian cycles; its three cycles cover
    // every edge exactly twice, so all six directed rings load links evenly.
    base = {{0, 1, 2, 3}, {0, 3, 2, 1}, {0, 2, 1, 3}, {0, 3, 1, 2}, {0, 1, 3, 2}, {0, 2, 3, 1}};
  } else {
    std::vector<std::vector<char>> used(n, std::vector<char>(n, 0));
    for (int k = 0; k < n; ++k) {
      std::vector<int> path{0};
      std::vector<char> seen(n, 0);
      seen[0] = 1;
      if (!ham_dfs(n, used, path, seen)) break;
      for (int i = 0; i < n; ++i) {
        const int a = path[i], b = path[(i + 1) % n];
        used[a][b] = used[b][a] = 1;
      }
      base.push_back(path);
      std::vector<int> rev{0};
      for (int i = n - 1; i >= 1; --i) rev.push_back(path[i]);
      base.push_back(rev);
    }
    if (base.empty()) {
      std::vector<int> r(n);
      for (int i = 0; i < n; ++i) r[i] = i;
      base.push_back(r);
    }
  }
  // n = 2: one ring, 4 channels of it.  A channel keeps one 4-step slice per
  // lane in flight, so the bytes a rank has in flight grow with channels x
  // slice, not with lanes (2-rank virtual node, 128 MiB, graph replay: 2 x 32
  // lanes 507 GB/s, 4 x 16 541, 4 x 32 754, 8 x 16 751).  Two-term sums
  // commute, so the channel count leaves every n = 2 result unchanged.
  int nch = nch_req > 0 ? nch_req : (n == 2 ? 4 : n == 1 ? 2 : (int)base.size());
  nch = std::min(nch, (int)MCCS_MAX_NCHANNELS);
  for (int c = 0; c < nch; ++c) rings->push_back(base[c % base.size()]);
}

// ---------------------------------------------------------------------------
bool devices_p2p_atomics(const std::vector<int>& devices) {
  for (int a : devices)
    for (int b : devices) {
      int ok = 0;
      if (rt().P2PAtomics(&ok, a, b) != hipSuccess || !ok) return false;
    }
  return true;
}

mccsResult_t comm_set_kernel_cfg(Comm* c) {
  mccsRingKernelCfg k{};
  k.fence_mode = !c->all_uncached ? MCCS_FENCE_SYSTEM : c->fifo_release ? MCCS_FENCE_UNCACHED_RELEASE : MCCS_FENCE_UNCACHED;
  // the node gate only ever steps the hand-off down (gate.cpp)
  if (c->gate_fence == MCCS_FENCE_SYSTEM) k.fence_mode = MCCS_FENCE_SYSTEM;
  else if (c->gate_fence == MCCS_FENCE_UNCACHED_RELEASE && k.fence_mode == MCCS_FENCE_UNCACHED)
    k.fence_mode = MCCS_FENCE_UNCACHED_RELEASE;
  k.err_line = 1;  // d_abort is a 64-byte line of ours: errors go to its word 1
  k.fifo_slots = (uint32_t)c->cfg.fifo_slots;
  const int tmo = c->cfg.timeout_ms == 0 ? kDefaultTimeoutMs : c->cfg.timeout_ms;
  k.timeout_ticks = tmo < 0 ? 0 : (uint64_t)tmo * 100000ull;  // s_memrealtime: 100 MHz
  // one 4-step slice per chunk (2 slices in flight per lane): one flag
  // round trip and one drain per chunk instead of two; +6-27 % on the virtual
  // node.  MCCS_SLICE_STEPS=2 restores the reference's SliceSteps (read at
  // communicator creation, carried in the connect handle: both ends agree).
  k.slice_steps = (uint32_t)c->slice_steps;
  if (const char* v = std::getenv("MCCS_RING_PROFILE")) k.profile = std::atoi(v) != 0;
  // MCCS_LAUNCH_GUARD=0 (test hook, honoured only with MCCS_TEST_HOOKS=1, read
  // when the comm connects): its launches skip the launch guard
  // (launch_guard.h), so a test can show the overlap the guard prevents
  const char* hooks = std::getenv("MCCS_TEST_HOOKS");
  const char* guard = std::getenv("MCCS_LAUNCH_GUARD");
  k.no_guard = hooks && std::atoi(hooks) == 1 && guard && std::atoi(guard) == 0;
  c->kcfg = k;  // travels in every launch's arguments (no device global)
  return mccsSuccess;
}

// Process-wide FIFO arena pool.  Arenas are not returned to the runtime while
// the device has memory: on this ROCm stack a virtual range freed as one memory
// type (coarse device memory) and re-allocated as another (uncached) kept
// behaving like the old type inside kernels (stale translations), corrupting
// FIFO hand-offs.  Pooling by (device, type) means the library never flips the
// type of a range it owns.  Requests round up to a size class and take the
// smallest pooled arena of at least that size (at most twice it), so
// communicators of nearby shapes share arenas and a process that creates many
// shapes does not keep one arena per shape (a 2,000-case fuzz on one GPU ran
// out of HBM at case 876 with exact-size pooling).
//
// An arena is handed out again only once every peer of its last communicator
// has released it: a peer's kernel may still post head lines into it after
// this rank's own kernel finished, and such a late post would land in the next
// tenant's flags.  Each peer writes the tenancy's epoch into the arena's
// release word for its rank when it destroys its communicator (comm_free,
// after its last kernel ended); until every awaited word holds the epoch the
// arena stays pooled but unused.
struct PooledArena {
  unsigned generation;  // rt_generation() of the runtime that allocated it
  int device;
  bool uncached;
  size_t bytes;
  char* ptr;
  uint64_t epoch;        // the last tenancy
  size_t release_off;    // its release words (ArenaLayout::release_off of that tenancy)
  uint64_t waiting;      // bit r: rank r's release not seen yet
  std::vector<int32_t> pid;  // rank r's process where its exit can be seen (0: wait for the word)
};
static std::mutex g_pool_mu;
static std::vector<PooledArena> g_pool;

// need rounded up to a quarter of its power of two (64 KiB granule at least):
// at most 25 % over, a few dozen classes between 1 MiB and 4 GiB
static size_t arena_class(size_t need) {
  size_t q = (size_t)1 << 16;
  while (q * 2 <= need) q <<= 1;
  const size_t g = std::max<size_t>((size_t)1 << 16, q / 4);
  return (need + g - 1) / g * g;
}

// Reads the release words of the pooled arenas `pick` selects that still
// await a peer, and clears the bits of the peers whose word now holds the
// tenancy's epoch.  The copies run outside g_pool_mu: a device copy can queue
// behind a running kernel, and other threads' setups must not wait on that.
// An entry taken or re-pooled meanwhile is matched by (ptr, epoch), which no
// later tenancy repeats.
template <class Pick>
static void pool_refresh(Pick pick) {
  struct Check {
    char* ptr;
    size_t off;
    uint64_t epoch, waiting;
    std::vector<int32_t> pid;
  };
  std::vector<Check> todo;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (const auto& a : g_pool)
      if (a.waiting && a.generation == rt_generation() && pick(a))
        todo.push_back({a.ptr, a.release_off, a.epoch, a.waiting, a.pid});
  }
  if (todo.empty()) return;
  for (auto& t : todo) {
    uint64_t w[ArenaLayout::kReleaseBytes / sizeof(uint64_t)];
    uint64_t released = 0;
    const bool read = rt().Memcpy(w, t.ptr + t.off, sizeof(w), hipMemcpyDeviceToHost) == hipSuccess;
    for (int r = 0; r < 64; ++r) {
      if (!(t.waiting >> r & 1)) continue;
      // its word holds the tenancy, or the peer process exited without
      // writing it (crashed, or its Connect failed before mapping this
      // arena): either way none of its kernels can still write here
      if ((read && w[r] == t.epoch) || (r < (int)t.pid.size() && t.pid[r] > 0 && rt().ProcessGone(t.pid[r])))
        released |= 1ull << r;
    }
    t.waiting = released;
  }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (auto& a : g_pool)
    for (const auto& t : todo)
      if (a.ptr == t.ptr && a.epoch == t.epoch) a.waiting &= ~t.waiting;
}

static char* pool_take(int device, bool uncached, size_t need, size_t* got) {
  auto fits = [&](const PooledArena& a) {
    return a.generation == rt_generation() && a.device == device && a.uncached == uncached && a.bytes >= need &&
           a.bytes <= 2 * need;
  };
  pool_refresh(fits);
  std::lock_guard<std::mutex> lk(g_pool_mu);
  size_t best = g_pool.size();
  for (size_t i = 0; i < g_pool.size(); ++i)
    if (fits(g_pool[i]) && !g_pool[i].waiting && (best == g_pool.size() || g_pool[i].bytes < g_pool[best].bytes))
      best = i;
  if (best == g_pool.size()) return nullptr;
  char* p = g_pool[best].ptr;
  *got = g_pool[best].bytes;
  g_pool.erase(g_pool.begin() + best);
  return p;
}

static void pool_give(int device, bool uncached, size_t bytes, char* p, uint64_t epoch = 0, size_t release_off = 0,
                      uint64_t waiting = 0, std::vector<int32_t> pid = {}) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool.push_back(PooledArena{rt_generation(), device, uncached, bytes, p, epoch, release_off, waiting, std::move(pid)});
}

// Out of device memory: return this device's released pooled uncached arenas
// to the runtime (no communicator uses them and no peer will write them).
// Only uncached ones: whatever re-allocates such a range at worst sees
// uncached behaviour, which is still correct; a freed coarse range
// re-allocated as an uncached arena is the case the pool exists to avoid.
// Returns the bytes released.
static size_t pool_release_uncached(int device) {
  std::vector<char*> drop;
  size_t bytes = 0;
  pool_refresh([&](const PooledArena& a) { return a.device == device && a.uncached; });
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size();)
      if (g_pool[i].generation == rt_generation() && g_pool[i].device == device && g_pool[i].uncached &&
          !g_pool[i].waiting) {
        drop.push_back(g_pool[i].ptr);
        bytes += g_pool[i].bytes;
        g_pool.erase(g_pool.begin() + i);
      } else {
        ++i;
      }
  }
  for (char* p : drop) (void)rt().Free(p);
  if (!drop.empty()) MCCS_LOG("device %d out of memory: released %zu pooled FIFO arenas (%zu bytes)", device,
                              drop.size(), bytes);
  return bytes;
}

// A FIFO arena of at least `need` bytes and the given type on the current
// device: a pooled one if one fits, else a new allocation of need's size
// class, retried once after releasing the pooled uncached arenas when the
// device is out of memory.
static hipError_t arena_alloc(int device, bool uncached, size_t need, char** p, size_t* got) {
  if ((*p = pool_take(device, uncached, need, got))) return hipSuccess;
  const size_t bytes = arena_class(need);
  auto alloc = [&] { return uncached ? rt().MallocUncached((void**)p, bytes) : rt().Malloc((void**)p, bytes); };
  hipError_t e = alloc();
  if (e == hipErrorOutOfMemory && pool_release_uncached(device) > 0) e = alloc();
  if (e != hipSuccess) {
    *p = nullptr;
    return e;
  }
  *got = bytes;
  return hipSuccess;
}

// A tenancy id unique in this process and across processes: pid, then a count.
static uint64_t next_arena_epoch() {
  static std::atomic<uint32_t> n{0};
  return ((uint64_t)(uint32_t)getpid() << 32) | (uint64_t)(n.fetch_add(1) + 1);
}

// A fake runtime's "device" memory dies with it (rt.cpp): its pooled arenas
// must never be handed out again.  Real HIP arenas (generation 0) stay.
void comm_pool_drop_generation(unsigned generation) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (size_t i = 0; i < g_pool.size();)
    if (g_pool[i].generation == generation) g_pool.erase(g_pool.begin() + i);
    else ++i;
}

int comm_pool_count(unsigned generation) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  int n = 0;
  for (const auto& a : g_pool) n += a.generation == generation;
  return n;
}

int comm_pool_waiting(unsigned generation) {
  if (generation == rt_generation()) pool_refresh([](const PooledArena&) { return true; });
  std::lock_guard<std::mutex> lk(g_pool_mu);
  int n = 0;
  for (const auto& a : g_pool) n += a.generation == generation && a.waiting != 0;
  return n;
}

bool GraphWorkPool::take(uint32_t n, uint32_t* start) {
  std::lock_guard<std::mutex> lk(mu);
  for (auto it = free_ranges.begin(); it != free_ranges.end(); ++it)
    if (it->second >= n) {
      *start = it->first;
      const uint32_t rest = it->second - n, at = it->first + n;
      free_ranges.erase(it);
      if (rest) free_ranges[at] = rest;
      held += n;
      return true;
    }
  return false;
}

void GraphWorkPool::give(uint32_t start, uint32_t n) {
  std::lock_guard<std::mutex> lk(mu);
  held -= n;
  auto it = free_ranges.emplace(start, n).first;
  auto next = std::next(it);
  if (next != free_ranges.end() && it->first + it->second == next->first) {
    it->second += next->second;
    free_ranges.erase(next);
  }
  if (it != free_ranges.begin()) {
    auto prev = std::prev(it);
    if (prev->first + prev->second == it->first) {
      prev->second += it->second;
      free_ranges.erase(it);
    }
  }
}

// Live communicators' device structures -> their FIFO depth, so the external
// launch (mccs_hip_launch_coll, whose reference-named kernels assume the
// reference's 8 slots) can refuse a library communicator built with another.
static std::mutex g_live_mu;
static std::map<const void*, int> g_live_fifo_slots;
static std::set<Comm*> g_live_comms;  // connected comms of this process (Comm::sync_owner lookups)

int comm_fifo_slots_of(const void* d_comm) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  auto it = g_live_fifo_slots.find(d_comm);
  return it == g_live_fifo_slots.end() ? 0 : it->second;
}

// The abort line must reach a kernel that polls it right after the host writes
// it (mccsCommAbort, the node gate's reset), with no GPU queue in between: a
// copy on any stream can wait behind the very kernel it must stop, since HIP
// maps a process's streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4
// here) and a stream created for the abort can share the spinning kernel's
// queue -- on MI355X an abort written that way was seen only when the kernel's
// 30 s watchdog ended it.  (A line in coarse device memory could also be held
// stale by L2, which a host DMA write does not update.)  So the line is
// host-mapped memory the CPU writes and reads directly; kernels read it over
// PCIe only when they check (every 64 polls of a wait, and between works).
// (The reference leaves its abortFlag uninitialised, device.rs:157; here it
// starts at zero.)
mccsResult_t place_abort_line(Comm* c) {
  StepScope st("abort line");
  MCCS_HIP(rt().HostMallocMapped((void**)&c->h_abort, 64));
  std::memset(c->h_abort, 0, 64);
  MCCS_HIP(rt().HostGetDevicePointer((void**)&c->d_abort, c->h_abort));
  return mccsSuccess;
}

// Swap this comm's uncached arena for a plain device arena (used when IPC
// export of the uncached one is refused).  The old range goes back to the pool.
mccsResult_t comm_switch_to_device_arena(Comm* c) {
  StepScope st("device arena fallback");
  DeviceGuard g(c->device);
  const size_t bytes = c->layout.total();
  // (its export was refused, so no peer ever saw it: nothing to await)
  if (c->own_arena) pool_give(c->device, c->own_arena_uncached, c->own_arena_bytes, c->own_arena);
  c->own_arena = nullptr;
  c->own_arena_uncached = false;
  {
    const hipError_t e = arena_alloc(c->device, false, bytes, &c->own_arena, &c->own_arena_bytes);
    if (e != hipSuccess) {
      err_hip("Malloc", e, __FILE__, __LINE__);
      return mccsUnhandledCudaError;
    }
  }
  MCCS_HIP(rt().Memset(c->own_arena, 0, bytes));
  MCCS_HIP(rt().FlushCaches());
  MCCS_HIP(rt().DeviceSynchronize());
  c->peer_arena[c->rank] = c->own_arena;
  return mccsSuccess;
}

mccsResult_t comm_alloc_local(Comm* c) {
  StepScope st0("comm_alloc_local");
  DeviceGuard g(c->device);
  c->layout.nch = c->nch;
  c->layout.buffer_size = (size_t)c->cfg.buffer_size;
  c->layout.fifo_bytes = (size_t)c->cfg.buffer_size / MCCS_BUFFER_SLOTS * (size_t)c->cfg.fifo_slots;
  // direct AllReduce region: only where the kernel can run (2..8 ranks)
  const bool direct_ok = c->nranks >= 2 && c->nranks <= MCCS_DIRECT_MAX_RANKS;
  c->layout.direct_slot =
      direct_ok && c->cfg.direct_bytes > 0 ? ((size_t)c->cfg.direct_bytes + 65535) & ~(size_t)65535 : 0;
  c->layout.oneshot_slot =
      direct_ok && c->cfg.oneshot_bytes > 0 ? ((size_t)c->cfg.oneshot_bytes + 65535) & ~(size_t)65535 : 0;
  // exactly 2 x ll_bytes (8-byte multiple): ranks that disagree on ll_bytes
  // get different arena sizes, which Connect refuses
  c->layout.ll_slot = direct_ok && c->cfg.ll_bytes > 0 ? 2 * (((size_t)c->cfg.ll_bytes + 7) & ~(size_t)7) : 0;
  const size_t bytes = c->layout.total();
  c->own_arena = nullptr;
  c->own_arena_uncached = false;
  // the peer tables first: comm_free may run after any step below fails
  c->peer_arena.assign(c->nranks, nullptr);
  c->peer_opened_ipc.assign(c->nranks, false);
  c->d_peers.assign(c->nch, nullptr);
  c->d_user_ranks.assign(c->nch, nullptr);
  {
    StepScope st("FIFO arena");
    if (c->cfg.fifo_memory != MCCS_FIFO_DEVICE) {  // UNCACHED or UNCACHED_RELEASE
      const hipError_t e = arena_alloc(c->device, true, bytes, &c->own_arena, &c->own_arena_bytes);
      if (e == hipSuccess)
        c->own_arena_uncached = true;
      else
        MCCS_LOG("uncached FIFO arena unavailable (%s); using hipMalloc + system fences", hipGetErrorString(e));
    }
    if (!c->own_arena) {
      const hipError_t e = arena_alloc(c->device, false, bytes, &c->own_arena, &c->own_arena_bytes);
      if (e != hipSuccess) {
        err_hip("Malloc", e, __FILE__, __LINE__);
        return mccsUnhandledCudaError;
      }
    }
    // trust but verify: the runtime must report the uncached allocation flag
    if (c->own_arena_uncached && !rt().IsUncached(c->own_arena)) {
      MCCS_LOG("arena %p is not reported uncached: using system fences", (void*)c->own_arena);
      c->own_arena_uncached = false;
    }
    if (std::getenv("MCCS_DEBUG"))
      MCCS_LOG("rank %d arena %p bytes %zu uncached=%d", c->rank, (void*)c->own_arena, bytes,
               (int)c->own_arena_uncached);
    c->peer_arena[c->rank] = c->own_arena;
    c->arena_epoch = next_arena_epoch();
    c->arena_shared = false;
    c->peer_epoch.assign(c->nranks, 0);
  }
  {
    StepScope st("FIFO arena zero-fill");
    MCCS_HIP(rt().Memset(c->own_arena, 0, bytes));
    MCCS_HIP(rt().FlushCaches());
    MCCS_HIP(rt().DeviceSynchronize());
  }
  MCCS_CHECK(place_abort_line(c));
  {
    StepScope st("device comm");
    // device communicator, per-channel views, launch guard (ring_cfg.h)
    MCCS_HIP(rt().Malloc((void**)&c->d_comm, MCCS_GUARD_OFF + sizeof(mccsLaunchGuard)));
    c->d_view = (mccsRingConnView*)((char*)c->d_comm + sizeof(mccsDevCommAndChannels));
    c->d_guard = (mccsLaunchGuard*)((char*)c->d_comm + MCCS_GUARD_OFF);
    MCCS_HIP(rt().Memset(c->d_guard, 0, sizeof(mccsLaunchGuard)));
    for (int ch = 0; ch < c->nch; ++ch) {
      MCCS_HIP(rt().Malloc((void**)&c->d_peers[ch], sizeof(mccsDevChannelPeer) * c->nranks));
      MCCS_HIP(rt().Malloc((void**)&c->d_user_ranks[ch], sizeof(int) * c->nranks));
    }
  }
  {
    StepScope st("work FIFO");
    c->work_depth = (uint32_t)c->cfg.work_fifo_depth;
    MCCS_HIP(rt().HostMallocMapped((void**)&c->h_work, sizeof(mccsDevWork) * c->work_depth));
    MCCS_HIP(rt().HostGetDevicePointer((void**)&c->d_work, c->h_work));
    std::memset(c->h_work, 0, sizeof(mccsDevWork) * c->work_depth);
  }
  {
    StepScope st("graph work arena");
    MCCS_HIP(rt().HostMallocMapped((void**)&c->h_graph_work, sizeof(mccsDevWork) * Comm::kGraphWorkEntries));
    MCCS_HIP(rt().HostGetDevicePointer((void**)&c->d_graph_work, c->h_graph_work));
    std::memset(c->h_graph_work, 0, sizeof(mccsDevWork) * Comm::kGraphWorkEntries);
    c->graph_pool = std::make_shared<GraphWorkPool>(Comm::kGraphWorkEntries);
  }
  {
    StepScope st("work done counters");
    MCCS_HIP(rt().HostMallocMapped((void**)&c->h_done, sizeof(uint32_t) * MCCS_MAX_NCHANNELS));
    MCCS_HIP(rt().HostGetDevicePointer((void**)&c->d_done, c->h_done));
    std::memset(c->h_done, 0, sizeof(uint32_t) * MCCS_MAX_NCHANNELS);
  }
  c->chan_next.assign(c->nch, 0);
  c->work_next = 0;
  c->work_acked_min = 0;
  {
    // comm stream: created on first use (comm_stream); the event becomes
    // interprocess only when a backend exports it (comm_make_event_ipc)
    StepScope st("events");
    MCCS_HIP(rt().EventCreate(&c->event, hipEventDisableTiming));
    MCCS_HIP(rt().EventCreate(&c->user_event, hipEventDisableTiming));
  }
  c->sched.assign(c->nch, ChannelSchedule{});
  return mccsSuccess;
}

// Builds mccsDevCommAndChannels once every peer arena is reachable
// (CommDevResources::new, device.rs:81-183; ring fields engine.rs:274-286).
mccsResult_t comm_build_device(Comm* c) {
  DeviceGuard g(c->device);
  const int n = c->nranks;
  mccsDevCommAndChannels hc;
  std::memset(&hc, 0, sizeof(hc));
  hc.comm.rank = c->rank;
  hc.comm.nRanks = n;
  hc.comm.buffSizes[MCCS_PROTO_SIMPLE] = c->cfg.buffer_size;
  hc.comm.abortFlag = c->d_abort;
  mccsRingConnView views[MCCS_MAX_NCHANNELS];
  std::memset(views, 0, sizeof(views));
  for (int ch = 0; ch < c->nch; ++ch) {
    const std::vector<int>& ring = c->rings[ch];
    const int ix_rank = (int)(std::find(ring.begin(), ring.end(), c->rank) - ring.begin());
    const int ix_zero = (int)(std::find(ring.begin(), ring.end(), 0) - ring.begin());
    std::vector<int> user_ranks(n);
    for (int i = 0; i < n; ++i) user_ranks[i] = ring[(i + ix_rank) % n];
    const int prev = user_ranks[n - 1], next = n > 1 ? user_ranks[1] : user_ranks[0];
    std::vector<mccsDevChannelPeer> peers(n);
    std::memset(peers.data(), 0, sizeof(mccsDevChannelPeer) * n);
    if (n > 1) {
      const bool sender_local = c->cfg.locality == MCCS_LOCALITY_SENDER;
      char* me = c->peer_arena[c->rank];
      char* nx = c->peer_arena[next];
      char* pv = c->peer_arena[prev];
      if (!me || !nx || !pv) MCCS_FAIL(mccsInternalError, "channel %d: a neighbour's FIFO arena is not mapped", ch);
      const ArenaLayout& L = c->layout;
      // send connector (to next): poll our head lines, post next's tail lines
      mccsDevConnInfo& s = peers[next].send[0];
      s.buffs[MCCS_PROTO_SIMPLE] = sender_local ? me + L.data_off(ch) : nx + L.data_off(ch);
      s.head = (uint64_t*)(me + L.head_off(ch));
      s.tail = (uint64_t*)(nx + L.tail_off(ch));
      // recv connector (from prev): poll our tail lines, post prev's head lines
      mccsDevConnInfo& r = peers[prev].recv[0];
      r.buffs[MCCS_PROTO_SIMPLE] = sender_local ? pv + L.data_off(ch) : me + L.data_off(ch);
      r.tail = (uint64_t*)(me + L.tail_off(ch));
      r.head = (uint64_t*)(pv + L.head_off(ch));
      views[ch] = {r.buffs[MCCS_PROTO_SIMPLE], s.buffs[MCCS_PROTO_SIMPLE], r.tail, r.head, s.head, s.tail};
    }
    MCCS_HIP(rt().Memcpy(c->d_peers[ch], peers.data(), sizeof(mccsDevChannelPeer) * n, hipMemcpyHostToDevice));
    MCCS_HIP(rt().Memcpy(c->d_user_ranks[ch], user_ranks.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    mccsDevChannel& dc = hc.channels[ch];
    dc.peers = c->d_peers[ch];
    dc.ring.prev = prev;
    dc.ring.next = next;
    dc.ring.userRanks = c->d_user_ranks[ch];
    dc.ring.index = (ix_rank + n - ix_zero) % n;
    dc.workFifoDone = c->d_done + ch;
  }
  MCCS_HIP(rt().Memcpy(c->d_comm, &hc, sizeof(hc), hipMemcpyHostToDevice));
  MCCS_HIP(rt().Memcpy(c->d_view, views, sizeof(views), hipMemcpyHostToDevice));
  MCCS_CHECK(comm_set_kernel_cfg(c));
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live_fifo_slots[c->d_comm] = c->cfg.fifo_slots;
    g_live_comms.insert(c);
  }
  c->connected = true;
  return mccsSuccess;
}

mccsResult_t comm_stream(Comm* c, hipStream_t* out) {
  if (!c->stream) {
    DeviceGuard g(c->device);
    MCCS_HIP(rt().StreamCreate(&c->stream));
  }
  *out = c->stream;
  return mccsSuccess;
}

// InitCommunicator's event handle (libmccs communicator.rs:35-38): a backend
// process exports the comm event to the application, so it must be an
// interprocess event.  Pending work is drained first, so the new event is
// recorded after every later launch and no earlier one is lost.  Fused comms
// whose launches this comm's event tracked read it through sync_owner at wait
// time, so they see the new one; the old one is destroyed once no thread
// synchronizes on it.
// Waits until no thread synchronizes on the comm's event outside the
// live-comm lock (comm_wait_last_launch).  Such a wait can last as long as a
// kernel spinning on late peers (up to the watchdog, 10 min by default), so
// after a few yields this sleeps, backing off to 1 ms (a busy
// spin here burnt a core for that long).
static void wait_no_waiters(Comm* c) {
  long ns = 0;
  for (int i = 0; c->waiters.load() > 0; ++i) {
    if (i < 64) {
      sched_yield();
      continue;
    }
    ns = ns ? std::min(ns * 2, 1000000L) : 1000L;
    const timespec ts{0, ns};
    nanosleep(&ts, nullptr);
  }
}

mccsResult_t comm_make_event_ipc(Comm* c) {
  if (c->event_ipc) return mccsSuccess;
  StepScope st("interprocess comm event");
  DeviceGuard g(c->device);
  if (c->event_recorded) MCCS_HIP(rt().EventSynchronize(c->event));
  else MCCS_HIP(rt().DeviceSynchronize());  // the latest launches recorded no event
  hipEvent_t e = nullptr;
  MCCS_HIP(rt().EventCreate(&e, hipEventDisableTiming | hipEventInterprocess));
  hipEvent_t old;
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    old = c->event;
    c->event = e;
  }
  wait_no_waiters(c);
  (void)rt().EventDestroy(old);
  c->event_ipc = true;
  return mccsSuccess;
}

hipError_t comm_wait_last_launch(Comm* c) {
  if (c->event_recorded) return rt().EventSynchronize(c->event);
  Comm* owner = nullptr;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    if (c->sync_owner && g_live_comms.count(c->sync_owner)) {
      owner = c->sync_owner;
      ev = owner->event;
      owner->waiters.fetch_add(1);
    }
  }
  if (owner) {
    // Outside the lock: a kernel spinning on its peers can keep
    // this wait going until the watchdog, and the lock guards every launch's
    // FIFO-depth lookup and every comm's build and free.
    const hipError_t e = rt().EventSynchronize(ev);
    owner->waiters.fetch_sub(1);
    return e;
  }
  return rt().DeviceSynchronize();  // nothing recorded the launch: every stream of the device
}

hipError_t comm_query_last_launch(Comm* c) {
  if (c->event_recorded) return rt().EventQuery(c->event);
  std::lock_guard<std::mutex> lk(g_live_mu);  // the owner's event: read while it cannot be replaced or freed
  if (c->sync_owner && g_live_comms.count(c->sync_owner)) return rt().EventQuery(c->sync_owner->event);
  return hipErrorNotReady;  // nothing recorded the launch: it cannot be told finished
}

hipError_t comm_order_after_last_launch(Comm* c, hipStream_t s) {
  if (c->event_recorded) return rt().StreamWaitEvent(s, c->event);
  std::lock_guard<std::mutex> lk(g_live_mu);  // the owner's event: read while it cannot be replaced or freed
  if (c->sync_owner && g_live_comms.count(c->sync_owner)) return rt().StreamWaitEvent(s, c->sync_owner->event);
  return hipSuccess;
}

mccsResult_t comm_free(Comm* c) {
  DeviceGuard g(c->device);
  // the last launch (any stream) must be done before its arenas are reused
  (void)comm_wait_last_launch(c);
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live_fifo_slots.erase(c->d_comm);
    g_live_comms.erase(c);
    for (Comm* x : g_live_comms)
      if (x->sync_owner == c) x->sync_owner = nullptr;
  }
  wait_no_waiters(c);  // a fused comm's wait on our event
  if (c->stream) (void)rt().StreamSynchronize(c->stream);
  // Our kernels are done: release every peer's arena (its release word for
  // our rank gets its tenancy's epoch), then unmap it.  Best effort: a peer
  // arena whose release is lost stays pooled, unused, in the peer's process.
  for (int r = 0; r < (int)c->peer_arena.size(); ++r) {
    if (r == c->rank || !c->peer_arena[r] || r >= (int)c->peer_epoch.size() || !c->peer_epoch[r]) continue;
    const uint64_t ep = c->peer_epoch[r];
    if (rt().Memcpy(c->peer_arena[r] + c->layout.release_off() + sizeof(uint64_t) * c->rank, &ep, sizeof(ep),
                    hipMemcpyHostToDevice) != hipSuccess)
      MCCS_LOG("rank %d: could not release rank %d's FIFO arena", c->rank, r);
  }
  for (int r = 0; r < (int)c->peer_arena.size(); ++r)
    if (c->peer_opened_ipc[r] && c->peer_arena[r]) (void)rt().IpcCloseMemHandle(c->peer_arena[r]);
  if (c->own_arena) {
    uint64_t waiting = 0;
    if (c->arena_shared)
      for (int r = 0; r < c->nranks; ++r)
        if (r != c->rank) waiting |= 1ull << r;
    pool_give(c->device, c->own_arena_uncached, c->own_arena_bytes, c->own_arena, c->arena_epoch,
              c->layout.release_off(), waiting, c->peer_pid);
  }
  for (auto p : c->d_peers)
    if (p) (void)rt().Free(p);
  for (auto p : c->d_user_ranks)
    if (p) (void)rt().Free(p);
  if (c->d_comm) (void)rt().Free(c->d_comm);
  if (c->h_abort) (void)rt().HostFree(c->h_abort);
  if (c->h_work) (void)rt().HostFree(c->h_work);
  if (c->h_graph_work) (void)rt().HostFree(c->h_graph_work);
  if (c->h_done) (void)rt().HostFree(c->h_done);
  if (c->event) (void)rt().EventDestroy(c->event);
  if (c->user_event) (void)rt().EventDestroy(c->user_event);
  if (c->stream) (void)rt().StreamDestroy(c->stream);
  return mccsSuccess;
}

}  // namespace mccs

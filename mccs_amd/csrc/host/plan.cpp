// plan.cpp — kernel plans: task schema, per-channel work elements, the
// host-mapped work FIFO and the launch (reference src/mccs/src/proxy/plan.rs).
//
//   get_task_schema ........ plan.rs:602-635   -> task_schema()
//   compute_coll_work ...... plan.rs:172-289   -> plan_enqueue()
//   select_best_channels ... plan.rs:292-302   -> select_channels()
//   enqueue_work_elem_coll . plan.rs:68-90     -> enqueue_elem()
//   wait_work_queue ........ plan.rs:380-422   -> wait_work_queue()
//   upload_work ............ plan.rs:424-541   -> upload_work()
//   work_elem_conversion ... plan.rs:550-600   -> to_dev_work()
//   launch_plan ............ plan.rs:638-669   -> plan_launch_group()
// MI355X differences: the grid is (#channels x lanes) workgroups of
// cfg.block_threads (the reference launches one block of nWarps*32 per
// channel); nWarps in each work element keeps the reference value because the
// kernel's chunk arithmetic (all_reduce.h:30-36) depends on it.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "comm.h"
#include "dtypes.h"

namespace mccs {

static constexpr int kMaxElemsPerWork = MCCS_MAX_WORK_ELEMENTS;
static constexpr size_t kSimpleMaxThreads = 512;
static constexpr size_t kSimpleThreadThreshold = 64;

void task_schema(size_t total_bytes, int nch_cfg, int* nch_out, int* nthreads_out) {
  size_t nch = (size_t)nch_cfg, nthr = kSimpleMaxThreads;
  while (total_bytes < nch * nthr * kSimpleThreadThreshold) {
    if (nch >= 2) nch -= 1;
    else if (nthr % 128 == 0) nthr /= 2;
    else break;
  }
  nthr += WARP_SIZE;
  if (nthr / WARP_SIZE < 3) nthr = WARP_SIZE * 3;
  *nch_out = (int)nch;
  *nthreads_out = (int)nthr;
}

static inline bool rolling_less_u32(uint32_t a, uint32_t b) { return (uint32_t)(a - b) > 0x7fffffffu; }
static inline uint32_t rolling_min_u32(uint32_t a, uint32_t b) { return (uint32_t)(b - a) <= 0x7fffffffu ? a : b; }

// The k least-loaded channels, ties by id (ChannelLoad ordering,
// plan.rs:673-692), into ids[0..return); no allocation.
static int select_channels(const Comm* c, int k, int* ids) {
  int n = 0;
  for (int i = 0; i < c->nch; ++i) {  // stable insertion sort by load
    int j = n++;
    for (; j > 0 && c->sched[ids[j - 1]].coll_bytes > c->sched[i].coll_bytes; --j) ids[j] = ids[j - 1];
    ids[j] = i;
  }
  return std::min(k, c->nch);
}

static void enqueue_elem(ChannelSchedule& s, const WorkElemHost& e, int func_index, size_t esize) {
  s.coll_bytes += e.count * esize;
  if (!s.works.empty()) {
    HostWork& tail = s.works.back();
    if (tail.func == func_index && tail.e[0].nWarps == e.nWarps && tail.n < kMaxElemsPerWork) {
      tail.e[tail.n++] = e;
      return;
    }
  }
  s.works.emplace_back();
  HostWork& w = s.works.back();
  w.e[0] = e;
  w.n = 1;
  w.func = func_index;
}

static mccsResult_t ring_enqueue(Comm* c, int func, int dtype, int op, const void* send, void* recv, size_t count) {
  const size_t esize = (size_t)elem_bytes(dtype);
  const size_t total = func == mccsFuncAllGather ? count * c->nranks : count * esize;  // task.rs:95-102
  int nch = 0, nthr = 0;
  task_schema(total, c->nch, &nch, &nthr);
  int chans[MCCS_MAX_NCHANNELS];
  const int nsel = select_channels(c, nch, chans);
  for (int bid = 0; bid < nsel; ++bid) {
    WorkElemHost e{};
    e.nWarps = (uint8_t)(nthr / WARP_SIZE);
    e.send = send;
    e.recv = recv;
    e.count = count;
    e.bid = (uint8_t)bid;
    e.nChannels = (uint8_t)nsel;
    enqueue_elem(c->sched[chans[bid]], e, /*funcIndex, unused (plan.rs:585)*/ 0,
                 func == mccsFuncAllGather ? 1 : esize);
  }
  c->plan_pending = true;
  c->plan_func = func;
  c->plan_dtype = dtype;
  c->plan_op = op;
  return mccsSuccess;
}

void plan_discard(Comm* c) {
  for (auto& s : c->sched) s.reset();
  c->plan_pending = false;
  c->plan_direct = false;
}

// A pending direct AllReduce goes back to the ring after all: the group holds
// another collective of this comm, or the device's fused launch cannot run it.
static mccsResult_t demote_direct(Comm* c) {
  if (!c->plan_direct) return mccsSuccess;
  c->plan_direct = false;
  c->plan_pending = false;
  return ring_enqueue(c, c->plan_func, c->plan_dtype, c->plan_op, c->direct.send, c->direct.recv, c->direct.count);
}

// The LL one-shot needs an uncached arena: its lines are polled with
// system-scope loads, which a cached (device) arena's L2 could serve stale.
static bool ll_fits(const Comm* c, size_t bytes) {
  return c->layout.ll_slot > 0 && c->own_arena_uncached && c->kcfg.fence_mode != MCCS_FENCE_SYSTEM &&
         bytes <= (size_t)c->cfg.ll_bytes && 2 * ((bytes + 7) & ~(size_t)7) <= c->layout.ll_slot;
}

mccsResult_t plan_enqueue(Comm* c, int func, int dtype, int op, const void* send, void* recv, size_t count) {
  if (c->plan_pending && (c->plan_func != func || c->plan_dtype != dtype || c->plan_op != op))
    // pre_launch_schedule batches same func/dtype/op only (plan.rs:122-141)
    MCCS_FAIL(mccsInvalidUsage, "a group mixes collectives of different function / dtype / op on one communicator");
  MCCS_CHECK(demote_direct(c));
  // One AllReduce that fits the direct region (every rank decides alike: same
  // call, same config) is held for the direct kernel; the launch may still
  // send it to the ring (plan_launch_group).
  // (AllGather: count is bytes per rank; its one-shot moves the ring's link
  // bytes in one exchange instead of n-1 hops)
  const size_t bytes = func == mccsFuncAllGather ? count : count * (size_t)elem_bytes(dtype);
  const bool oneshot = c->layout.oneshot_slot > 0 && bytes <= (size_t)c->cfg.oneshot_bytes;
  const bool twoshot = func == mccsFuncAllReduce && c->layout.direct_slot > 0 && bytes <= (size_t)c->cfg.direct_bytes;
  const bool ll = ll_fits(c, bytes);
  // (the LL one-shot makes no remote atomics: it runs without peer atomics,
  // the count-based variants need them)
  if (!c->plan_pending && (func == mccsFuncAllReduce || func == mccsFuncAllGather) &&
      ((c->direct_ok && (oneshot || twoshot)) || ll)) {
    c->plan_direct = true;
    c->direct.send = send;
    c->direct.recv = recv;
    c->direct.count = count;
    c->plan_pending = true;
    c->plan_func = func;
    c->plan_dtype = dtype;
    c->plan_op = op;
    return mccsSuccess;
  }
  return ring_enqueue(c, func, dtype, op, send, recv, count);
}

static mccsDevWork to_dev_work(const HostWork& elems, bool in_fifo, bool is_last, uint32_t u) {
  mccsDevWork w;
  std::memset(&w, 0, sizeof(w));
  for (size_t i = 0; i < elems.size(); ++i) {
    mccsDevWorkElem& d = w.elems[i];
    d.isUsed = 1;
    d.nWarps = elems[i].nWarps;
    d.sendbuff = elems[i].send;
    d.recvbuff = elems[i].recv;
    d.count = elems[i].count;
    d.root = 0;
    d.bid = elems[i].bid;
    d.nChannels = elems[i].nChannels;
    d.redOpArg = 0;
  }
  w.header.funcIndex = 0;
  w.header.type = mccsDevWorkTypeColl;
  w.header.inFifo = in_fifo ? 1 : 0;
  w.header.isLast = is_last ? 1 : 0;
  if (is_last) w.header.doneAcks = u;
  else w.header.workNext = (int32_t)u;
  return w;
}

static mccsResult_t wait_work_queue(Comm* c, uint32_t target) {
  if (!rolling_less_u32(c->work_acked_min + c->work_depth, target)) return mccsSuccess;
  for (uint64_t spins = 0;; ++spins) {
    uint32_t ackd[MCCS_MAX_NCHANNELS];
    for (int i = 0; i < MCCS_MAX_NCHANNELS; ++i) ackd[i] = __atomic_load_n(&c->h_done[i], __ATOMIC_RELAXED);
    uint32_t all = c->work_next;
    for (int ch = 0; ch < c->nch; ++ch)
      if (ackd[ch] != c->chan_next[ch]) all = rolling_min_u32(all, ackd[ch]);
    for (int ch = 0; ch < c->nch; ++ch)
      if (ackd[ch] == c->chan_next[ch]) __atomic_store_n(&c->h_done[ch], all, __ATOMIC_RELAXED);
    c->work_acked_min = all;
    if (!rolling_less_u32(c->work_acked_min + c->work_depth, target)) return mccsSuccess;
    if ((spins & 0xfffff) == 0xfffff && comm_query_last_launch(c) == hipSuccess) {
      // stream idle but acks missing: the kernel aborted
      MCCS_FAIL(mccsRemoteError, "work FIFO full and its kernel no longer running (aborted or timed out)");
    }
    sched_yield();
  }
}

struct LaunchDesc {
  const void* fn = nullptr;
  const void* multi_fn = nullptr;
  uint64_t mask = 0;
  int nch_used = 0;
  mccsDevWork* work = nullptr;
  bool work_inline = false;  // works in the launch arguments: no FIFO entry, no acknowledgement
};

// MCCS_EAGER_EVENTS=1: record the comm event after every launch (round-2
// behaviour; A/B and callers that poll the event themselves).
static bool eager_events() {
  static const bool on = [] {
    const char* v = std::getenv("MCCS_EAGER_EVENTS");
    return v && std::atoi(v) != 0;
  }();
  return on;
}

// Rank slots of a launch listed by the address of their comm's launch guard,
// 4 bits each (launch_guard.h: every fused launch takes its guards in this
// one order, so two of them never hold each other's).
static uint64_t guard_order(const std::vector<Comm*>& comms, const std::vector<int>& idx) {
  int k[MCCS_MULTI_MAX_RANKS];
  const int n = (int)idx.size();
  for (int i = 0; i < n; ++i) {  // insertion sort of the slots by guard address
    int j = i;
    for (; j > 0 && comms[idx[k[j - 1]]]->d_guard > comms[idx[i]]->d_guard; --j) k[j] = k[j - 1];
    k[j] = i;
  }
  uint64_t order = 0;
  for (int i = 0; i < n; ++i) order |= (uint64_t)k[i] << (4 * i);
  return order;
}

namespace {
struct GraphWorkRelease {
  std::shared_ptr<GraphWorkPool> pool;
  uint32_t start, n;
};
void graph_work_release(void* p) {  // runs when the graph holding the range is gone
  auto* r = (GraphWorkRelease*)p;
  r->pool->give(r->start, r->n);
  delete r;
}
}  // namespace

// A launch being captured into HIP graph `graph`: its works go to a range of
// the comm's graph arena, laid out like one FIFO upload (first work of channel
// i at entry i, later ones chained by workNext relative to the head), with
// inFifo = 0 so replays never write workFifoDone (common.h:153-155).  The
// range returns to the arena when the graph and its executables are destroyed.
static mccsResult_t upload_work_graph(Comm* c, LaunchDesc* ld, hipGraph_t graph) {
  std::vector<int> chan_list;
  uint64_t mask = 0;
  uint32_t work_count = 0;
  for (int ch = 0; ch < c->nch; ++ch)
    if (!c->sched[ch].works.empty()) {
      chan_list.push_back(ch);
      mask |= 1ull << ch;
      work_count += (uint32_t)c->sched[ch].works.size();
    }
  if (chan_list.empty()) return mccsInternalError;
  uint32_t start = 0;
  if (work_count > Comm::kGraphWorkEntries)
    MCCS_FAIL(mccsInvalidUsage, "one captured launch needs %u work entries, more than the graph work arena's %u: "
              "split the group", work_count, Comm::kGraphWorkEntries);
  if (!c->graph_pool->take(work_count, &start))
    MCCS_FAIL(mccsInvalidUsage, "graph work arena exhausted (%u of %u entries held by live graphs, %u needed)",
              c->graph_pool->held_now(), Comm::kGraphWorkEntries, work_count);
  auto* rel = new GraphWorkRelease{c->graph_pool, start, work_count};
  if (rt().GraphOnDestroy(graph, &graph_work_release, rel) != hipSuccess) {
    MCCS_LOG("graph work entries %u..%u stay held for the comm's lifetime (no destroy callback)", start,
             start + work_count - 1);
    delete rel;
  }
  mccsDevWork* head = c->h_graph_work + start;
  const uint32_t nchan = (uint32_t)chan_list.size();
  uint32_t subsequent = nchan;
  for (uint32_t nth = 0; nth < nchan; ++nth) {
    auto& works = c->sched[chan_list[nth]].works;
    for (size_t wid = 0; wid < works.size(); ++wid) {
      const bool last = wid == works.size() - 1;
      const uint32_t next = wid == 0 ? subsequent : subsequent + 1;
      mccsDevWork dw = to_dev_work(works[wid], false, last, last ? 0u : next);
      const uint32_t cur = wid == 0 ? nth : subsequent++;
      head[cur] = dw;
    }
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);
  ld->mask = mask;
  ld->nch_used = (int)nchan;
  ld->work = c->d_graph_work + start;
  ld->fn = ring_kernel_ptr(c->plan_func, c->plan_dtype, c->plan_op);
  ld->multi_fn = ring_multi_kernel_ptr(c->plan_func, c->plan_dtype, c->plan_op);
  for (auto& s : c->sched) s.reset();
  c->plan_pending = false;
  return (ld->fn && ld->multi_fn) ? mccsSuccess : mccsInvalidArgument;
}

// A launch whose ranks' used channels each hold one work carries the works in
// its arguments (mccsMultiLaunchArgs.inline_work, ring_cfg.h): no FIFO slot,
// no acknowledgement, and no PCIe read in the kernel prologue.  Returns the
// channels used per rank (0: use the work FIFO).  MCCS_INLINE_WORKS=0 turns it
// off.
static int inline_channels(const Comm* c) {
  if (!c->inline_works) return 0;
  int used = 0;
  for (int ch = 0; ch < c->nch; ++ch) {
    const auto& works = c->sched[ch].works;
    if (works.size() > 1 || (works.size() == 1 && works[0].size() != 1)) return 0;  // one work of one element
    used += works.size() == 1;
  }
  return used;
}

static mccsResult_t upload_work_inline(Comm* c, LaunchDesc* ld, mccsMultiLaunchArgs* ma) {
  uint64_t mask = 0;
  uint32_t n = 0;
  for (int ch = 0; ch < c->nch; ++ch)
    if (!c->sched[ch].works.empty()) {
      mask |= 1ull << ch;
      const mccsDevWork w = to_dev_work(c->sched[ch].works[0], false, true, 0);
      ma->inline_work[ma->inline_works + n].header = w.header;
      ma->inline_work[ma->inline_works + n++].elem = w.elems[0];
    }
  ma->inline_works += n;
  ld->mask = mask;
  ld->nch_used = (int)n;
  ld->work = nullptr;
  ld->work_inline = true;
  ld->fn = ring_kernel_ptr(c->plan_func, c->plan_dtype, c->plan_op);
  ld->multi_fn = ring_multi_kernel_ptr(c->plan_func, c->plan_dtype, c->plan_op);
  for (auto& s : c->sched) s.reset();
  c->plan_pending = false;
  return (ld->fn && ld->multi_fn) ? mccsSuccess : mccsInvalidArgument;
}

static mccsResult_t upload_work(Comm* c, LaunchDesc* ld) {
  std::vector<int> chan_list;
  uint64_t mask = 0;
  uint32_t work_count = 0;
  for (int ch = 0; ch < c->nch; ++ch)
    if (!c->sched[ch].works.empty()) {
      chan_list.push_back(ch);
      mask |= 1ull << ch;
      work_count += (uint32_t)c->sched[ch].works.size();
    }
  if (chan_list.empty()) return mccsInternalError;
  // one launch's works must fit the ring at once (they are all read by the
  // one kernel): more could never be acknowledged, and the wait below would
  // spin until it mistook the idle stream for a dead kernel
  if (work_count > c->work_depth)
    MCCS_FAIL(mccsInvalidUsage, "one launch needs %u work entries, more than the work FIFO's %u: split the group "
              "or raise mccsCommConfig.work_fifo_depth", work_count, c->work_depth);
  const uint32_t qmask = c->work_depth - 1;
  const uint32_t nchan = (uint32_t)chan_list.size();
  uint32_t first = c->work_next;
  if (((first + nchan - 1) & qmask) < (first & qmask)) {  // wrap: restart at slot 0
    first = (first + qmask) & ~qmask;
    c->work_next = first;
  }
  MCCS_CHECK(wait_work_queue(c, first + work_count));
  // Acknowledgements: a chained channel's last work sits at `subsequent`, so
  // subsequent + 1 (plan.rs:461-470) is one past it.  A single-work channel's
  // entry is first + nth, where plan.rs's subsequent + 1 = first + nchan + 1
  // reaches one entry PAST this launch: once read, it would release the
  // next launch's first entry before that launch has read it.  Here a
  // single work acknowledges the launch's end; entries of this launch not
  // yet read by other channels stay covered by wait_work_queue's minimum
  // over busy channels.
  const uint32_t launch_end = first + work_count;
  uint32_t subsequent = first + nchan;
  for (uint32_t nth = 0; nth < nchan; ++nth) {
    const int ch = chan_list[nth];
    auto& works = c->sched[ch].works;
    for (size_t wid = 0; wid < works.size(); ++wid) {
      mccsDevWork dw;
      if (wid == works.size() - 1) {
        const uint32_t ack = works.size() == 1 ? launch_end : subsequent + 1;
        c->chan_next[ch] = ack;
        dw = to_dev_work(works[wid], true, true, ack);
      } else {
        const uint32_t nxt = (wid == 0 ? subsequent : subsequent + 1) & qmask;
        dw = to_dev_work(works[wid], false, false, (uint32_t)((int32_t)nxt - (int32_t)(first & qmask)));
      }
      uint32_t cur;
      if (wid == 0) {
        cur = first + nth;
      } else {
        cur = subsequent;
        subsequent += 1;
      }
      c->h_work[cur & qmask] = dw;
    }
  }
  c->work_next = subsequent;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  ld->mask = mask;
  ld->nch_used = (int)nchan;
  ld->work = c->d_work + (first & qmask);
  ld->fn = ring_kernel_ptr(c->plan_func, c->plan_dtype, c->plan_op);
  ld->multi_fn = ring_multi_kernel_ptr(c->plan_func, c->plan_dtype, c->plan_op);
  for (auto& s : c->sched) s.reset();
  c->plan_pending = false;
  return (ld->fn && ld->multi_fn) ? mccsSuccess : mccsInvalidArgument;
}

// Blocks of the fused multi-rank kernels the device holds at once, minimised
// over every (func, dtype, op) instantiation.  Ranks sharing a GPU spin on
// each other's flags, so their fused launch must be fully co-resident.
// A probe the runtime refuses returns 0 ("unknown": callers check it) and
// is not cached, so a transient failure does not stick for the process; the
// cache is per device runtime (rt_generation: the real one, or a test fake).
int coresident_ring_blocks(int block, int device) {
  static std::mutex mu;
  static std::map<std::tuple<unsigned, int, int>, int> cache;  // (runtime, device, block) -> blocks
  const auto key = std::make_tuple(rt_generation(), device, block);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  DeviceGuard g(device);
  int ncu = 0;
  if (rt().CuCount(&ncu, device) != hipSuccess) return 0;
  int best = 1 << 30;
  const void* fns[1 + mccsNumTypes * 4];
  int nf = 0;
  fns[nf++] = ring_multi_kernel_ptr(mccsFuncAllGather, mccsInt8, 0);
  for (int dt = 0; dt < mccsNumTypes; ++dt)
    for (int op = 0; op < 4; ++op) fns[nf++] = ring_multi_kernel_ptr(mccsFuncAllReduce, dt, op);
  for (int i = 0; i < nf; ++i) {
    int per_cu = 0;
    if (!fns[i] || rt().BlocksPerCu(&per_cu, fns[i], block) != hipSuccess) return 0;
    best = std::min(best, per_cu);
  }
  std::lock_guard<std::mutex> lk(mu);
  return cache[key] = best * ncu;
}

// Workgroups of the direct kernels the device holds at once (min over the
// instantiations): a direct launch spins on peers' flags, so all of its
// workgroups, and those of ranks sharing the GPU, must be resident together.
static int coresident_direct_blocks(int device, int* ncu_out = nullptr) {
  static std::mutex mu;
  static std::map<std::pair<unsigned, int>, std::pair<int, int>> cache;  // (runtime, device) -> (blocks, CUs)
  const auto key = std::make_pair(rt_generation(), device);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) {
      if (ncu_out) *ncu_out = it->second.second;
      return it->second.first;
    }
  }
  DeviceGuard g(device);
  int ncu = 0;
  if (rt().CuCount(&ncu, device) != hipSuccess) return 0;
  int best = 1 << 30;
  for (int dt = 0; dt < mccsNumTypes; ++dt)
    for (int op = 0; op < 4; ++op) {
      int per_cu = 0;
      const void* fn = direct_kernel_ptr(dt, op);
      if (!fn || rt().BlocksPerCu(&per_cu, fn, MCCS_DIRECT_THREADS) != hipSuccess) return 0;  // not cached
      best = std::min(best, per_cu);
    }
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = {best * ncu, ncu};
  if (ncu_out) *ncu_out = ncu;
  return best * ncu;
}

// Every comm of the device group holds one direct AllReduce of the same shape
// (fused ranks share the launch's walk arguments).
static bool direct_group(std::vector<Comm*>& comms, const std::vector<int>& idx) {
  const Comm* c0 = comms[idx[0]];
  for (size_t k = 0; k < idx.size(); ++k) {
    const Comm* ck = comms[idx[k]];
    if (!ck->plan_direct) return false;
    if (ck->nranks != c0->nranks || ck->direct.count != c0->direct.count || ck->plan_func != c0->plan_func ||
        ck->plan_dtype != c0->plan_dtype ||
        ck->plan_op != c0->plan_op || ck->rings != c0->rings || ck->cfg.buffer_size != c0->cfg.buffer_size ||
        ck->layout.direct_slot != c0->layout.direct_slot || ck->layout.oneshot_slot != c0->layout.oneshot_slot ||
        ck->layout.ll_slot != c0->layout.ll_slot || ck->cfg.ll_bytes != c0->cfg.ll_bytes ||
        ck->cfg.oneshot_bytes != c0->cfg.oneshot_bytes || ck->cfg.direct_bytes != c0->cfg.direct_bytes ||
        ck->nch != c0->nch || ck->peer_arena != c0->peer_arena)  // one region table for every slot
      return false;
  }
  return idx.size() <= MCCS_MULTI_MAX_RANKS;
}

// The direct launch's arguments: the ring walk this call would take (the
// channels and thread count of get_task_schema, each channel's ring read as
// rank-at-ring-index, engine.rs:274-286) and every rank slot's buffers and
// direct regions.
static mccsResult_t build_direct(std::vector<Comm*>& comms, const std::vector<int>& idx, mccsDirectArgs* da,
                                 unsigned* grid_x) {
  const Comm* c0 = comms[idx[0]];
  const bool gather = c0->plan_func == mccsFuncAllGather;
  const size_t esize = gather ? 1 : (size_t)elem_bytes(c0->plan_dtype);
  int nch = 0, nthr = 0;
  task_schema(c0->direct.count * esize, c0->nch, &nch, &nthr);
  int chans[MCCS_MAX_NCHANNELS];
  const int nsel = select_channels(c0, nch, chans);
  std::memset(da, 0, sizeof(*da));
  const int n = c0->nranks;
  da->count = c0->direct.count;
  da->slot_bytes = c0->layout.direct_slot;
  da->oslot_bytes = c0->layout.oneshot_slot;
  da->ll_slot_bytes = c0->layout.ll_slot;
  const size_t nbytes = (size_t)c0->direct.count * esize;
  bool ll = true;  // every rank slot of the launch must take it (uncached arena)
  for (size_t k = 0; k < idx.size(); ++k) ll = ll && ll_fits(comms[idx[k]], nbytes);
  if (!ll && !c0->direct_ok) return mccsInternalError;  // plan_enqueue held it for LL only
  const bool oneshot = ll || (c0->layout.oneshot_slot > 0 && nbytes <= (size_t)c0->cfg.oneshot_bytes);
  da->mode = gather ? (ll ? MCCS_DIRECT_LL_AG : MCCS_DIRECT_AG_ONE_SHOT)
             : ll   ? MCCS_DIRECT_LL_ONE_SHOT
             : oneshot ? MCCS_DIRECT_ONE_SHOT
                       : MCCS_DIRECT_TWO_SHOT;
  da->nranks = (uint32_t)n;
  da->nch = (uint32_t)nsel;
  da->nthr_ref = (uint32_t)nthr;
  da->buff_size = (uint32_t)c0->cfg.buffer_size;
  da->fence_mode = c0->kcfg.fence_mode;
  da->timeout_ticks = c0->kcfg.timeout_ticks;
  for (int bid = 0; bid < nsel; ++bid) {
    const std::vector<int>& ring = c0->rings[chans[bid]];
    const int pos0 = (int)(std::find(ring.begin(), ring.end(), 0) - ring.begin());
    for (int k = 0; k < n; ++k) da->idx2rank[bid][k] = (uint8_t)ring[(pos0 + k) % n];
  }
  // elements each rank owns: the ring walk (all_reduce.h:28-42), chunk k of
  // channel bid owned by the rank at ring index k (AllGather: unused)
  if (!gather) {
    const int64_t size = (int64_t)da->count, parts = (int64_t)da->nch * n;
    const int64_t chunk = (int64_t)((int)da->buff_size / MCCS_BUFFER_SLOTS / (int)esize) * ALLREDUCE_CHUNKSTEPS;
    const int64_t gran = std::max<int64_t>(1, (int64_t)(nthr - WARP_SIZE) * 8 / (int64_t)esize);
    for (int64_t g = 0; g < size; g += parts * chunk) {
      int64_t rcs = std::min(chunk, (size - g + parts - 1) / parts);
      rcs = (rcs + gran - 1) / gran * gran;
      for (int64_t c = 0; c < parts; ++c) {
        const int64_t off = g + c * rcs;
        if (off < size) da->owned[da->idx2rank[c / n][c % n]] += (uint64_t)std::min(rcs, size - off);
      }
    }
  }
  for (size_t k = 0; k < idx.size(); ++k) {
    const Comm* ck = comms[idx[k]];
    mccsDirectRank& r = da->r[k];
    r.send = ck->direct.send;
    r.recv = ck->direct.recv;
    for (int t = 0; t < n; ++t) {
      if (!ck->peer_arena[t]) return mccsInternalError;
      if (k == 0) da->region[t] = ck->peer_arena[t] + ck->layout.direct_off();
      else if (da->region[t] != ck->peer_arena[t] + ck->layout.direct_off()) return mccsInternalError;  // direct_group
    }
    r.comm = (mccsDevComm*)ck->d_comm;
    r.abort_flag = ck->d_abort;
    r.rank = (uint32_t)ck->rank;
    r.err_line = 1;
    // safest hand-off of the group, as for the ring (SYSTEM > UNCACHED_RELEASE > UNCACHED)
    if (ck->kcfg.fence_mode == MCCS_FENCE_SYSTEM) da->fence_mode = MCCS_FENCE_SYSTEM;
    else if (ck->kcfg.fence_mode == MCCS_FENCE_UNCACHED_RELEASE && da->fence_mode == MCCS_FENCE_UNCACHED)
      da->fence_mode = MCCS_FENCE_UNCACHED_RELEASE;
    da->timeout_ticks = (da->timeout_ticks == 0 || ck->kcfg.timeout_ticks == 0)
                            ? 0
                            : std::max(da->timeout_ticks, ck->kcfg.timeout_ticks);
  }
  // Workgroups: ~4 KiB of phase-1 bytes each at least, at most
  // MCCS_DIRECT_BLOCKS; pieces: each phase's bytes over the workgroups, in
  // 4 KiB steps (aligned: chunk offsets are granule multiples), 4..64 KiB.
  // One-shot: phase 1 sends the whole input, phase 2 reduces all of it.
  const size_t bytes = nbytes;
  // two-shot phases 1 and 3: the chunks others own; AllGather phase 2: n-1 segments
  const size_t scatter = gather ? bytes * (n - 1) : oneshot ? bytes : bytes - bytes / n;
  // Ranks sharing a GPU split its CUs: at most one direct workgroup per CU
  // per rank (the virtual node ran n = 4 / 8 fastest at 64 / 32 workgroups
  // per rank, i.e. one per CU in all; two per CU cost up to 1.5x), and never
  // more than can be resident at once (they spin on each other's counts).
  int ncu = 0;
  const int cap = coresident_direct_blocks(c0->device, &ncu);
  if (ncu <= 0) ncu = cap;
  // scatter bytes per workgroup (MCCS_DIRECT_WG_BYTES): 4 KiB beat 8 / 16 KiB
  // on the virtual node at 32-512 KiB (n = 8 32 KiB one-shot 19.1 -> 14.4 us,
  // 16 KiB: 27.0) and tied 2 KiB (pieces are >= 4 KiB)
  static const long wg_bytes = [] {
    const char* v = std::getenv("MCCS_DIRECT_WG_BYTES");
    const long x = v ? std::atol(v) : 0;
    return x >= 1024 ? x : 4096L;
  }();
  long g = std::min<long>((long)((scatter + wg_bytes - 1) / wg_bytes), c0->direct_blocks);
  // LL: one 8-byte word per thread
  if (ll) g = std::min<long>((long)((nbytes + 8 * MCCS_DIRECT_THREADS - 1) / (8 * MCCS_DIRECT_THREADS)), c0->direct_blocks);
  if (idx.size() > 1) g = std::min<long>(g, std::min(cap, ncu) / (long)idx.size());  // one fused launch
  else if (c0->share > 1) g = std::min<long>(g, std::min(cap / 2, ncu) / c0->share);  // separate processes
  g = std::max<long>(g, 1);
  if (g * (long)idx.size() > cap)
    MCCS_FAIL(mccsInvalidUsage, "direct launch of %zu ranks x %ld workgroups exceeds the %d co-resident ones of device %d",
              idx.size(), g, cap, c0->device);
  *grid_x = (unsigned)g;
  auto piece = [&](size_t phase_bytes) {
    size_t p = (phase_bytes + (size_t)g - 1) / (size_t)g;
    p = std::min<size_t>(std::max<size_t>((p + 4095) & ~(size_t)4095, 4096), 65536);
    return (uint32_t)(p / esize);
  };
  da->piece = piece(gather ? bytes : scatter);
  da->piece2 = piece(gather ? scatter : oneshot ? bytes : bytes / n + 1);
  for (size_t k = 0; k < idx.size(); ++k) {
    Comm* ck = comms[idx[k]];
    ck->plan_direct = false;
    ck->plan_pending = false;
  }
  return mccsSuccess;
}

// Launch every pending plan.  By default a comm launches on the caller's
// stream (stream order equals libmccs's bridge).  With bridge_streams = 1 it
// launches on its own stream, bridged to the caller's with events like
// libmccs (collectives.rs:86,134 + proxy/engine.rs:1185-1189).  Comms sharing
// a device are fused into one multi-rank launch so their blocks are
// co-resident (they spin on each other's flags); events join their streams
// only when the callers used different ones.  A device group whose comms each
// hold one direct-sized AllReduce runs the direct kernel, anything else the
// ring.
mccsResult_t plan_launch_group(std::vector<Comm*>& comms, std::vector<hipStream_t>& user_streams) {
  // pending comms grouped by device, in device order (buffers kept per
  // thread: an eager launch allocates nothing)
  static thread_local std::vector<int> order, idx;
  order.clear();
  for (int i = 0; i < (int)comms.size(); ++i) {
    if (!comms[i]->plan_pending) continue;
    order.push_back(i);
    for (size_t j = order.size() - 1; j > 0 && comms[order[j - 1]]->device > comms[i]->device; --j)
      std::swap(order[j], order[j - 1]);
  }
  for (size_t run = 0; run < order.size();) {
    const int dev = comms[order[run]]->device;
    idx.clear();
    while (run < order.size() && comms[order[run]]->device == dev) idx.push_back(order[run++]);
    if (idx.size() > MCCS_MULTI_MAX_RANKS)
      MCCS_FAIL(mccsInvalidUsage, "%zu ranks share one device (at most %d)", idx.size(), (int)MCCS_MULTI_MAX_RANKS);
    DeviceGuard g(dev);
    const bool direct = direct_group(comms, idx);
    if (!direct)
      for (int i : idx) MCCS_CHECK(demote_direct(comms[i]));
    if (!direct && idx.size() > 1) {  // checked before any work is uploaded, so the comms stay usable
      const Comm* c0 = comms[idx[0]];
      const int cap = coresident_ring_blocks(c0->block_threads, dev);
      const long need = (long)c0->nch * c0->lanes * (long)idx.size();
      if (need > cap) {
        // would deadlock: every block spins on a peer's flag
        MCCS_FAIL(mccsInvalidUsage, "fused launch of %zu ranks x %d blocks exceeds the %d co-resident blocks of device %d",
                  idx.size(), c0->nch * c0->lanes, cap, dev);
      }
    }
    // A capturing stream records this launch into a HIP graph: its work
    // list must outlive the FIFO's rolling slots (upload_work_graph).
    bool capturing = false;
    hipGraph_t graph = nullptr;
    MCCS_HIP(rt().StreamIsCapturing(user_streams[idx[0]], &capturing));
    if (capturing) MCCS_HIP(rt().CaptureGraph(user_streams[idx[0]], &graph));
    LaunchDesc lds[MCCS_MULTI_MAX_RANKS];
    mccsMultiLaunchArgs ma;
    mccsDirectArgs da;
    const void* fn = nullptr;
    void* args[1] = {nullptr};
    unsigned grid = 0, block = 0;
    Comm* c0 = comms[idx[0]];
    if (direct) {
      MCCS_CHECK(build_direct(comms, idx, &da, &grid));
      fn = c0->plan_func == mccsFuncAllGather ? direct_kernel_ptr(mccsInt8, mccsDevSum)
                                              : direct_kernel_ptr(c0->plan_dtype, c0->plan_op);
      if (!fn) return mccsInvalidArgument;
      block = MCCS_DIRECT_THREADS;
      da.guard_order = guard_order(comms, idx);
      for (int i : idx) da.no_guard |= comms[i]->kcfg.no_guard;  // comm_set_kernel_cfg's test hook
      args[0] = &da;
    } else {
      std::memset(&ma, 0, sizeof(ma));
      int per_rank = inline_channels(comms[idx[0]]);
      for (size_t k = 1; k < idx.size() && per_rank > 0; ++k)
        if (inline_channels(comms[idx[k]]) != per_rank) per_rank = 0;
      if (per_rank > 0 && per_rank * idx.size() <= MCCS_INLINE_WORKS) {
        for (size_t k = 0; k < idx.size(); ++k) MCCS_CHECK(upload_work_inline(comms[idx[k]], &lds[k], &ma));
      } else {
        for (size_t k = 0; k < idx.size(); ++k)
          MCCS_CHECK(capturing ? upload_work_graph(comms[idx[k]], &lds[k], graph) : upload_work(comms[idx[k]], &lds[k]));
      }
      // Communicator launches carry their hand-off policy in the arguments
      // (one launch per device; blockIdx.y = rank slot when ranks share it).
      // Fused ranks take the safest policy of the group.
      ma.channelMask = lds[0].mask;
      ma.cfg = c0->kcfg;
      for (size_t k = 0; k < idx.size(); ++k) {
        const Comm* ck = comms[idx[k]];
        if (lds[k].mask != lds[0].mask || lds[k].multi_fn != lds[0].multi_fn || ck->lanes != c0->lanes ||
            ck->block_threads != c0->block_threads || ck->kcfg.slice_steps != c0->kcfg.slice_steps ||
            ck->kcfg.fifo_slots != c0->kcfg.fifo_slots)
          MCCS_FAIL(mccsInvalidUsage, "ranks sharing a GPU issued different collectives in one group");
        ma.comm[k] = (mccsDevComm*)ck->d_comm;
        ma.work[k] = lds[k].work;
        ma.view[k] = ck->d_view;
        // safest of the group: SYSTEM > UNCACHED_RELEASE > UNCACHED
        if (ck->kcfg.fence_mode == MCCS_FENCE_SYSTEM) ma.cfg.fence_mode = MCCS_FENCE_SYSTEM;
        else if (ck->kcfg.fence_mode == MCCS_FENCE_UNCACHED_RELEASE && ma.cfg.fence_mode == MCCS_FENCE_UNCACHED)
          ma.cfg.fence_mode = MCCS_FENCE_UNCACHED_RELEASE;
        ma.cfg.timeout_ticks = (ma.cfg.timeout_ticks == 0 || ck->kcfg.timeout_ticks == 0)
                                   ? 0
                                   : std::max(ma.cfg.timeout_ticks, ck->kcfg.timeout_ticks);
        ma.cfg.profile |= ck->kcfg.profile;
      }
      ma.guard_order = guard_order(comms, idx);
      fn = lds[0].multi_fn;
      grid = (unsigned)(lds[0].nch_used * c0->lanes);
      block = (unsigned)c0->block_threads;
      args[0] = &ma;
    }
    const bool bridge = c0->cfg.bridge_streams >= 0;
    hipStream_t st = user_streams[idx[0]];
    if (bridge) MCCS_CHECK(comm_stream(c0, &st));
    bool one_user_stream = true;  // ranks sharing a GPU issued from one stream: no events needed
    for (size_t k = 1; k < idx.size(); ++k) one_user_stream = one_user_stream && user_streams[idx[k]] == user_streams[idx[0]];
    const bool events = bridge || !one_user_stream;
    if (events) {
      for (size_t k = 0; k < idx.size(); ++k) {
        Comm* c = comms[idx[k]];
        MCCS_HIP(rt().EventRecord(c->user_event, user_streams[idx[k]]));
        MCCS_HIP(rt().StreamWaitEvent(st, c->user_event));
      }
    }
    // A communicator's launches run one at a time in issue order, as on the
    // reference's private comm stream (proxy/init.rs:166-175): its kernels
    // share the FIFO flags, the lanes' saved steps and the direct counters.
    // A launch on another stream than the comm's previous one therefore waits
    // for that launch first (two launches of one comm on two streams ran
    // concurrently and returned wrong sums, 2 of 6 cases at n = 4).  Not while
    // capturing: a graph cannot depend on an event recorded outside it, and a
    // replay makes no library call -- the device's launch guard
    // (launch_guard.h) keeps replays from running beside any other launch of
    // the comm.  Streams are told apart by id, not address: a stream destroyed
    // with the comm's kernel still queued gives its address to the next one
    // created.
    unsigned long long st_id = 0;
    MCCS_HIP(rt().StreamId(st, &st_id));
    if (!capturing)
      for (size_t k = 0; k < idx.size(); ++k) {
        Comm* c = comms[idx[k]];
        if (c->launched && c->last_stream_id != st_id) MCCS_HIP(comm_order_after_last_launch(c, st));
      }
    // The launching comm's event rides on the dispatch's own completion signal
    // (hipExtLaunchKernel stopEvent): a hipEventRecord behind the kernel is a
    // marker packet that cost ~3 us of device time per launch on MI355X, the
    // stop event nothing (tools/launch_cost.hip).  Not while capturing (a
    // graph replays plain kernel nodes) and not for an interprocess event
    // (exported to a backend: recorded the usual way).
    const bool stop_on_launch = !capturing && !c0->event_ipc;
    const dim3 g3(grid, (unsigned)idx.size());
    if (stop_on_launch) MCCS_HIP(rt().LaunchKernelExt(fn, g3, dim3(block), args, st, c0->event));
    else MCCS_HIP(rt().LaunchKernel(fn, g3, dim3(block), args, st));
    // Other events are recorded only when consumed (Comm::event_recorded):
    // cross-stream ordering or an exported backend event.  Fused rank slots
    // otherwise answer for their launch through the launching comm's stop
    // event (sync_owner): mccsCommSync waits on it and wait_work_queue asks it
    // whether a work-FIFO kernel still runs.  (A record per fused slot was a
    // marker packet and ~1.5 us of host time per FIFO launch.)
    bool record = events || eager_events();
    for (size_t k = 0; k < idx.size() && !record; ++k) record = comms[idx[k]]->event_ipc;
    if (record && !stop_on_launch) MCCS_HIP(rt().EventRecord(c0->event, st));
    if (events) {
      for (size_t k = 0; k < idx.size(); ++k) {
        if (!bridge && k == 0) continue;
        MCCS_HIP(rt().StreamWaitEvent(user_streams[idx[k]], c0->event));
      }
    }
    if (record)
      for (size_t k = 1; k < idx.size(); ++k) MCCS_HIP(rt().EventRecord(comms[idx[k]]->event, st));
    for (size_t k = 0; k < idx.size(); ++k) {
      // A capture launches nothing: the comm's latest launch, its stream and
      // its event stay those of the last eager launch (letting a
      // capture overwrite them let the next eager launch on a third stream skip
      // its wait for that one).
      if (!capturing) {
        comms[idx[k]]->last_stream_id = st_id;
        comms[idx[k]]->launched = true;
        comms[idx[k]]->event_recorded = record;
        // fused rank slots without their own record wait on the launching comm's event
        comms[idx[k]]->sync_owner = (k > 0 && !record && stop_on_launch) ? c0 : nullptr;
      }
      comms[idx[k]]->last_algo = !direct                            ? MCCS_ALGO_RING
                                 : da.mode == MCCS_DIRECT_TWO_SHOT ? MCCS_ALGO_DIRECT
                                 : da.mode == MCCS_DIRECT_LL_ONE_SHOT || da.mode == MCCS_DIRECT_LL_AG ? MCCS_ALGO_LL
                                                                   : MCCS_ALGO_ONESHOT;
    }
    if (!capturing) c0->event_recorded = record || stop_on_launch;
  }
  return mccsSuccess;
}

}  // namespace mccs

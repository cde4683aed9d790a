// gate.cpp — the connect-time self-test of every default-on hand-off path
// ("node gate").
//
// The library's defaults were tuned where ranks share one GPU: the ring's
// relaxed hand-off on uncached FIFOs (ring_cfg.h MCCS_FENCE_UNCACHED) and the
// direct LL / one-shot / two-shot exchanges (direct_kernel.h).  On a node
// nobody has tested, a hand-off that is fast here could read a stale slot
// over a link.  So when a communicator spans two or more GPUs, connecting it
// runs one exact-sum AllReduce through each path before any caller's
// collective (inputs k/64, |k| <= 127: every partial sum is exact in fp32, so
// the result does not depend on the summation order, and each repetition
// uses different values so a stale slot shows):
//   ring      in the configured hand-off; on a wrong sum every rank steps
//             down uncached -> uncached + release -> cached (system-scope
//             release/acquire, the reference's own ordering), re-testing each;
//   LL, one-shot, two-shot (the enabled ones): a wrong sum disables that
//             variant for the communicator (its buckets take the ring).
// Ranks agree on every decision: in one process (mccsCommInitAll) the host
// ORs the ranks' verdicts; across processes (mccsCommConnect) each rank's
// verdicts travel through one ring AllReduce(MAX) in the cached mode with
// system-scope fences, so all ranks step down together.  The same vote ANDs
// the ranks' own view of peer atomics (each rank judged it from
// device ordinals that are local to its process).  A direct test launch that
// hits the (5 s) watchdog counts as a wrong sum for that variant; a ring
// launch that does fails the connect with mccsTimeout (a hang leaves the
// ranks' FIFO steps out of step, which no local reset repairs).  Across
// processes the ranks first meet in one ring launch under the configured
// watchdog (gate_barrier), so a peer that enters Connect late is waited for.
//
// MCCS_GATE=0 skips the gate; MCCS_GATE=1 runs it even when every rank is on
// one GPU (tests).  Test seams, honoured only with MCCS_TEST_HOOKS=1:
// MCCS_GATE_INJECT (a mask of MCCS_GATE_* bits treated as wrong sums on the
// ranks named by MCCS_GATE_INJECT_RANK, default every rank), MCCS_GATE_SKIP
// (direct paths those ranks do not launch, so their peers' launches hang
// until the watchdog) and
// MCCS_GATE_ASSUME_PASS=1 (the fake runtime runs no kernel: results are
// taken as correct).  mccsCommGateInfo reports the outcome.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "comm.h"
#include "dtypes.h"

namespace mccs {

namespace {

bool hooks_on() {
  const char* h = std::getenv("MCCS_TEST_HOOKS");
  return h && std::atoi(h) == 1;
}

unsigned hook_mask(const char* var, int rank) {
  if (!hooks_on()) return 0;
  const char* m = std::getenv(var);
  if (!m) return 0;
  const char* r = std::getenv("MCCS_GATE_INJECT_RANK");
  if (r && std::atoi(r) != rank) return 0;
  return (unsigned)std::strtoul(m, nullptr, 0);
}
// paths reported wrong on this rank (MCCS_GATE_INJECT)
unsigned injected(int rank) { return hook_mask("MCCS_GATE_INJECT", rank); }
// direct paths this rank does not launch at all (MCCS_GATE_SKIP): its peers'
// launches of them then hang until the watchdog, the failure mode of a
// variant whose hand-off never arrives
unsigned skipped(int rank) { return hook_mask("MCCS_GATE_SKIP", rank); }

bool assume_pass() {
  const char* a = std::getenv("MCCS_GATE_ASSUME_PASS");
  return hooks_on() && a && std::atoi(a) == 1;
}

float gate_val(int rank, size_t i, int rep) {
  const int k = (int)((i * 7 + (size_t)rank * 13 + (size_t)rep * 29) % 255) - 127;
  return (float)k / 64.0f;
}

// The gate bit of the ring in hand-off mode `fence`.
unsigned ring_bit(uint32_t fence) {
  return fence == MCCS_FENCE_UNCACHED           ? MCCS_GATE_RING_UNCACHED
         : fence == MCCS_FENCE_UNCACHED_RELEASE ? MCCS_GATE_RING_RELEASE
                                                : MCCS_GATE_RING_SYSTEM;
}

struct Buf {
  float* send = nullptr;
  float* recv = nullptr;
};

// Test sizes (fp32 elements per rank; ragged so tails are exercised) and the
// algorithm the planner must report for each path.
constexpr size_t kRingCount = 262144 + 3007;  // ~1 MiB: every channel, several slices
constexpr uint64_t kGateTimeoutTicks = 500000000ull;  // 5 s (s_memrealtime, 100 MHz) per gate launch
size_t path_count(const Comm* c, unsigned bit) {
  switch (bit) {
    case MCCS_GATE_LL: return std::min<size_t>((size_t)c->cfg.ll_bytes, 65536) / 4 - 1;
    case MCCS_GATE_ONESHOT: return std::min<size_t>((size_t)c->cfg.oneshot_bytes, 524288) / 4 - 3;
    case MCCS_GATE_TWOSHOT: return std::min<size_t>((size_t)c->cfg.direct_bytes, 2 << 20) / 4 - 5;
    default: return kRingCount;
  }
}
int path_algo(unsigned bit) {
  return bit == MCCS_GATE_LL        ? MCCS_ALGO_LL
         : bit == MCCS_GATE_ONESHOT ? MCCS_ALGO_ONESHOT
         : bit == MCCS_GATE_TWOSHOT ? MCCS_ALGO_DIRECT
                                    : MCCS_ALGO_RING;
}

// Routes the next AllReduce of `c` through one path: the other variants'
// thresholds read 0 (plan_enqueue takes none of them) until restore().
struct Route {
  Comm* c;
  int ll, one, dir;
  Route(Comm* cc, unsigned bit) : c(cc), ll(cc->cfg.ll_bytes), one(cc->cfg.oneshot_bytes), dir(cc->cfg.direct_bytes) {
    if (bit != MCCS_GATE_LL) c->cfg.ll_bytes = 0;
    if (bit != MCCS_GATE_ONESHOT) c->cfg.oneshot_bytes = 0;
    if (bit != MCCS_GATE_TWOSHOT) c->cfg.direct_bytes = 0;
  }
  ~Route() {
    c->cfg.ll_bytes = ll;
    c->cfg.oneshot_bytes = one;
    c->cfg.direct_bytes = dir;
  }
};

// Whether `c` can run a direct variant at all (the planner would pick it).
bool path_enabled(const Comm* c, unsigned bit) {
  switch (bit) {
    case MCCS_GATE_LL:
      return c->layout.ll_slot > 0 && c->cfg.ll_bytes >= 64 && c->own_arena_uncached &&
             c->kcfg.fence_mode != MCCS_FENCE_SYSTEM;
    case MCCS_GATE_ONESHOT: return c->direct_ok && c->layout.oneshot_slot > 0 && c->cfg.oneshot_bytes >= 64;
    case MCCS_GATE_TWOSHOT: return c->direct_ok && c->layout.direct_slot > 0 && c->cfg.direct_bytes >= 64;
  }
  return true;
}

// One exact-sum AllReduce of `count` fp32 per rank on every comm of `cs`
// (fused per device), repetition `rep`.  ok[k]: rank slot k's output matched
// and the planner took `want_algo`.
mccsResult_t gate_allreduce(std::vector<Comm*>& cs, std::vector<Buf>& bufs, size_t count, int rep, int want_algo,
                            std::vector<bool>* ok, std::vector<bool>* hung_out) {
  const int n = cs[0]->nranks;
  std::vector<float> host(count), want(count);
  for (size_t i = 0; i < count; ++i) {
    double s = 0;
    for (int r = 0; r < n; ++r) s += gate_val(r, i, rep);
    want[i] = (float)s;
  }
  for (size_t k = 0; k < cs.size(); ++k) {
    DeviceGuard g(cs[k]->device);
    for (size_t i = 0; i < count; ++i) host[i] = gate_val(cs[k]->rank, i, rep);
    MCCS_HIP(rt().Memcpy(bufs[k].send, host.data(), count * 4, hipMemcpyHostToDevice));
    MCCS_HIP(rt().Memset(bufs[k].recv, 0xff, count * 4));  // NaN: an untouched element never matches
  }
  MCCS_CHECK(mccsGroupStart());
  mccsResult_t er = mccsSuccess;
  for (size_t k = 0; k < cs.size() && er == mccsSuccess; ++k)
    er = mccsAllReduce(bufs[k].send, bufs[k].recv, count, mccsFloat32, mccsDevSum, (mccsComm_t)cs[k], nullptr);
  const mccsResult_t ge = mccsGroupEnd();
  MCCS_CHECK(er);
  MCCS_CHECK(ge);
  // A direct launch that hits the watchdog is a wrong answer for that path,
  // not a dead communicator: the direct kernel keeps no state the ring uses
  // (its region is never touched again once the vote disables it), so the
  // rank clears its abort line and votes.  A ring launch that hangs leaves
  // the ranks' FIFO steps out of step: that one fails the connect.
  std::vector<bool> hung(cs.size(), false);
  for (size_t k = 0; k < cs.size(); ++k) {
    Comm* c = cs[k];
    const mccsResult_t sr = mccsCommSync((mccsComm_t)c);
    if (sr == mccsSuccess) continue;
    if (want_algo == MCCS_ALGO_RING || (sr != mccsTimeout && sr != mccsRemoteError)) return sr;
    MCCS_LOG("node gate: a direct AllReduce (algo %d) hit the watchdog on rank %d; voting it off", want_algo, c->rank);
    DeviceGuard g(c->device);
    __atomic_store_n(c->h_abort + 1, 0u, __ATOMIC_SEQ_CST);
    __atomic_store_n(c->h_abort, 0u, __ATOMIC_SEQ_CST);
    c->failed = false;
    hung[k] = true;
  }
  const bool pass = assume_pass();
  for (size_t k = 0; k < cs.size(); ++k) {
    DeviceGuard g(cs[k]->device);
    MCCS_HIP(rt().Memcpy(host.data(), bufs[k].recv, count * 4, hipMemcpyDeviceToHost));
    const bool same = pass || std::memcmp(host.data(), want.data(), count * 4) == 0;
    (*ok)[k] = same && !hung[k] && cs[k]->last_algo == want_algo;
    if (hung[k]) (*hung_out)[k] = true;
  }
  return mccsSuccess;
}

// Failure bits of `bit`'s path for every comm of `cs` (2 repetitions; ring 3).
// `direct_dead`: a direct launch hung on one of these ranks earlier; the
// direct variants share one control block (launch sequence, running counts)
// that a hang leaves out of step, so none is launched again and all of them
// are reported wrong (the vote turns them off on every rank).
mccsResult_t gate_path(std::vector<Comm*>& cs, std::vector<Buf>& bufs, unsigned bit, std::vector<unsigned>* fail,
                       bool* direct_dead) {
  StepScope st(bit == MCCS_GATE_LL        ? "LL test"
               : bit == MCCS_GATE_ONESHOT ? "one-shot test"
               : bit == MCCS_GATE_TWOSHOT ? "two-shot test"
                                          : "ring test (hand-off " + std::to_string(cs[0]->kcfg.fence_mode) + ")");
  constexpr unsigned kDirect = MCCS_GATE_LL | MCCS_GATE_ONESHOT | MCCS_GATE_TWOSHOT;
  const bool direct = bit & kDirect;
  bool skip = direct && *direct_dead;
  for (Comm* c : cs) skip = skip || (direct && (skipped(c->rank) & bit));
  if (skip) {
    for (unsigned& f : *fail) f |= kDirect;
    *direct_dead = true;
    return mccsSuccess;
  }
  std::vector<Route> routes;
  routes.reserve(cs.size());
  for (Comm* c : cs) routes.emplace_back(c, bit);
  const size_t count = path_count(cs[0], bit);
  const int reps = direct ? 2 : 3;
  std::vector<bool> ok(cs.size(), true), hung(cs.size(), false);
  for (int rep = 0; rep < reps; ++rep) {
    MCCS_CHECK(gate_allreduce(cs, bufs, count, rep, path_algo(bit), &ok, &hung));
    bool any_hung = false;
    for (size_t k = 0; k < cs.size(); ++k) {
      if (!ok[k]) (*fail)[k] |= bit;
      if (hung[k]) any_hung = true;
    }
    if (any_hung) {
      for (unsigned& f : *fail) f |= kDirect;
      *direct_dead = true;
      break;
    }
  }
  for (size_t k = 0; k < cs.size(); ++k) (*fail)[k] |= injected(cs[k]->rank) & bit;
  return mccsSuccess;
}

// One ring AllReduce(MAX) of kVoteWords uint32 (in/out `v`) over this
// process's one rank of the communicator, in the cached mode with
// system-scope fences (the reference's hand-off) whatever mode is configured,
// under a watchdog of `ticks` (0: none).
constexpr int kVoteWords = 32;
mccsResult_t ring_max(Comm* c, Buf& b, uint32_t* v, uint64_t ticks) {
  DeviceGuard g(c->device);
  MCCS_HIP(rt().Memcpy(b.send, v, kVoteWords * 4, hipMemcpyHostToDevice));
  Route route(c, 0);
  const mccsRingKernelCfg saved = c->kcfg;
  c->kcfg.fence_mode = MCCS_FENCE_SYSTEM;
  c->kcfg.timeout_ticks = ticks;
  mccsResult_t r = mccsAllReduce(b.send, b.recv, kVoteWords, mccsUint32, mccsDevMax, (mccsComm_t)c, nullptr);
  if (r == mccsSuccess) r = mccsCommSync((mccsComm_t)c);
  c->kcfg = saved;
  MCCS_CHECK(r);
  MCCS_HIP(rt().Memcpy(v, b.recv, kVoteWords * 4, hipMemcpyDeviceToHost));
  return mccsSuccess;
}

// Every rank's failure bits ORed, the same answer on every rank.  In one
// process: the host ORs them.  Across processes (cs.size() == 1 < nranks):
// one ring_max over one uint32 per bit.
mccsResult_t gate_vote(std::vector<Comm*>& cs, std::vector<Buf>& bufs, std::vector<unsigned>* fail,
                       unsigned* agreed) {
  StepScope st("vote");
  unsigned all = 0;
  for (unsigned f : *fail) all |= f;
  if ((int)cs.size() == cs[0]->nranks) {
    *agreed = all;
    return mccsSuccess;
  }
  uint32_t v[kVoteWords];
  for (int b = 0; b < kVoteWords; ++b) v[b] = (all >> b) & 1u;
  // a peer may still sit in a direct test launch until its own (5 s)
  // watchdog fires before this ring launch runs there: wait longer here
  MCCS_CHECK(ring_max(cs[0], bufs[0], v, 3ull * kGateTimeoutTicks));
  if (assume_pass()) {  // nothing ran: the local bits stand for the vote
    *agreed = all;
    return mccsSuccess;
  }
  unsigned out = 0;
  for (int b = 0; b < kVoteWords; ++b) {
    // a vote that is not 0/1 came back corrupted
    if (v[b] > 1) MCCS_FAIL(mccsInternalError, "vote word %d came back as %u", b, v[b]);
    out |= (v[b] & 1u) << b;
  }
  *agreed = out;
  return mccsSuccess;
}

// Across processes, the ranks enter Connect at different times (a peer still
// loading code objects, opening IPC handles, or on a loaded host).  The
// gate's test launches run under a 5 s watchdog counted from kernel start, so
// before them the ranks meet in one ring launch under the communicator's own
// watchdog (a peer 5 s late used to fail the connect with
// mccsTimeout, or vote a direct variant off).  After it the ranks are in step
// to within host jitter.  One fused launch (cs.size() == nranks) needs none.
mccsResult_t gate_barrier(std::vector<Comm*>& cs, std::vector<Buf>& bufs, uint64_t configured_ticks) {
  if ((int)cs.size() == cs[0]->nranks) return mccsSuccess;
  StepScope st("barrier");
  uint32_t v[kVoteWords] = {0};
  return ring_max(cs[0], bufs[0], v, configured_ticks);
}

}  // namespace

int gate_env() {
  const char* g = std::getenv("MCCS_GATE");
  return g ? std::atoi(g) : -1;
}

bool gate_wanted(bool distinct_gpus) {
  const int g = gate_env();
  if (g == 0) return false;
  if (g == 1) return true;
  return distinct_gpus;
}

// Runs the gate over `cs`: every rank of the communicator (one process) or
// this process's one rank.  `atomics_ok`: this process's view of peer atomics
// for each comm (voted on; the outcome becomes direct_ok).
mccsResult_t comm_gate(std::vector<Comm*>& cs, const std::vector<bool>& atomics_ok) {
  if (cs.empty()) return mccsSuccess;
  const size_t max_count = std::max<size_t>(kRingCount, (2u << 20) / 4);
  std::vector<Buf> bufs(cs.size());
  std::vector<uint64_t> saved_ticks(cs.size());
  mccsResult_t r = mccsSuccess;
  for (size_t k = 0; k < cs.size() && r == mccsSuccess; ++k) {
    DeviceGuard g(cs[k]->device);
    if (rt().Malloc((void**)&bufs[k].send, max_count * 4) != hipSuccess ||
        rt().Malloc((void**)&bufs[k].recv, max_count * 4) != hipSuccess) {
      err_note(__FILE__, __LINE__, "test buffers: Malloc of %zu bytes failed", max_count * 4);
      r = mccsUnhandledCudaError;
    }
    // a gate launch that hangs ends after 5 s, not the configured 30 s
    saved_ticks[k] = cs[k]->kcfg.timeout_ticks;
    if (saved_ticks[k] == 0 || saved_ticks[k] > kGateTimeoutTicks) cs[k]->kcfg.timeout_ticks = kGateTimeoutTicks;
  }
  unsigned failed = 0, disabled = 0;
  bool direct_dead = false;
  std::vector<unsigned> fail(cs.size(), 0);
  // peer atomics: a rank that cannot do them turns the count-based variants off everywhere
  for (size_t k = 0; k < cs.size(); ++k)
    if (!atomics_ok[k]) fail[k] |= MCCS_GATE_NO_ATOMICS;
  if (r == mccsSuccess) r = gate_barrier(cs, bufs, saved_ticks[0]);
  // 1. the ring, stepping down the hand-off ladder until every rank's sums are exact
  for (int attempt = 0; attempt < 3 && r == mccsSuccess; ++attempt) {
    const unsigned bit = ring_bit(cs[0]->kcfg.fence_mode);
    r = gate_path(cs, bufs, bit, &fail, &direct_dead);
    unsigned agreed = 0;
    if (r == mccsSuccess) r = gate_vote(cs, bufs, &fail, &agreed);
    if (r != mccsSuccess) break;
    for (unsigned& f : fail) f &= ~bit;
    if (agreed & MCCS_GATE_NO_ATOMICS)
      for (Comm* c : cs) c->direct_ok = false;
    for (unsigned& f : fail) f &= ~MCCS_GATE_NO_ATOMICS;
    if (!(agreed & bit)) break;
    failed |= bit;
    if (bit == MCCS_GATE_RING_SYSTEM) {
      err_note(__FILE__, __LINE__, "the ring AllReduce is wrong in every hand-off mode; refusing the communicator");
      r = mccsSystemError;
      break;
    }
    const int next = bit == MCCS_GATE_RING_UNCACHED ? MCCS_FENCE_UNCACHED_RELEASE : MCCS_FENCE_SYSTEM;
    MCCS_LOG("node gate: ring AllReduce wrong in hand-off mode %u; stepping down to %d", cs[0]->kcfg.fence_mode, next);
    for (Comm* c : cs) {
      c->gate_fence = next;
      const uint64_t t = c->kcfg.timeout_ticks;
      MCCS_CHECK(comm_set_kernel_cfg(c));
      c->kcfg.timeout_ticks = t;
    }
  }
  // 2. the direct variants that are on (after the ring's mode settled: they
  // inherit its fence mode), one vote for all of them
  if (r == mccsSuccess) {
    const unsigned bits[3] = {MCCS_GATE_LL, MCCS_GATE_ONESHOT, MCCS_GATE_TWOSHOT};
    bool any = false;
    for (unsigned b : bits) {
      if (!path_enabled(cs[0], b) || r != mccsSuccess) continue;
      any = true;
      r = gate_path(cs, bufs, b, &fail, &direct_dead);
    }
    unsigned agreed = 0;
    if (r == mccsSuccess && any) r = gate_vote(cs, bufs, &fail, &agreed);
    if (r == mccsSuccess && any) {
      failed |= agreed;
      for (unsigned b : bits) {
        if (!(agreed & b)) continue;
        disabled |= b;
        MCCS_LOG("node gate: %s AllReduce wrong on this node; disabled for the communicator",
                 b == MCCS_GATE_LL ? "LL one-shot" : b == MCCS_GATE_ONESHOT ? "one-shot" : "two-shot");
        for (Comm* c : cs) {
          if (b == MCCS_GATE_LL) c->cfg.ll_bytes = 0;
          if (b == MCCS_GATE_ONESHOT) c->cfg.oneshot_bytes = 0;
          if (b == MCCS_GATE_TWOSHOT) c->cfg.direct_bytes = 0;
        }
      }
    }
  }
  for (size_t k = 0; k < cs.size(); ++k) {
    DeviceGuard g(cs[k]->device);
    if (bufs[k].send) (void)rt().Free(bufs[k].send);
    if (bufs[k].recv) (void)rt().Free(bufs[k].recv);
    cs[k]->kcfg.timeout_ticks = saved_ticks[k];
    cs[k]->gate_ran = r == mccsSuccess;
    cs[k]->gate_failed = failed;
    cs[k]->gate_disabled = disabled;
    cs[k]->last_algo = -1;
  }
  return r;
}

}  // namespace mccs

extern "C" mccsResult_t mccsCommGateInfo(mccsComm_t comm, int* info4) {
  const mccs::Comm* c = (const mccs::Comm*)comm;
  if (!c || !info4) return mccsInvalidArgument;
  info4[0] = c->gate_ran ? 1 : 0;
  info4[1] = c->kcfg.fence_mode == MCCS_FENCE_SYSTEM             ? MCCS_FIFO_DEVICE
             : c->kcfg.fence_mode == MCCS_FENCE_UNCACHED_RELEASE ? MCCS_FIFO_UNCACHED_RELEASE
                                                                 : MCCS_FIFO_UNCACHED;
  info4[2] = (int)c->gate_failed;
  info4[3] = (int)c->gate_disabled;
  return mccsSuccess;
}

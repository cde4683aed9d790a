// host_ring.cpp — the ring AllReduce protocol run by host threads over host
// memory: BASELINE configs[0] ("2-rank loopback allreduce, 1 KiB fp32,
// host-side elementwise sum; plumbing, no GPU").
//
// Same protocol as the gfx950 kernels (ring.hip) and the reference
// (all_reduce.h:10-87 schedule; prims_simple.h:68-237 FIFO: 8 slots, slices of
// 2 steps, sender waits head + 8 >= step + 2, receiver waits tail >= step + 2,
// operand order fn(own input, received)), with one host thread per
// (rank, channel) and std::atomic head/tail counters.  The threads and the
// FIFOs persist across calls (HostRingPool): a call hands each task to its
// own parked worker, so a 1 KiB AllReduce costs no thread creation.  It exists so the FIFO
// protocol and schedule can be exercised end to end without a GPU; it is not
// a fallback for the device path (nothing on the device path calls it).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "mccs_devcomm.h"
#include "mccs_hip.h"

namespace {

float h2f(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16, exp = (h >> 10) & 0x1f, man = h & 0x3ffu;
  uint32_t u;
  if (exp == 0) {
    float v = std::ldexp((float)man, -24);
    return sign ? -v : v;
  }
  if (exp == 31) u = sign | 0x7f800000u | (man << 13);
  else u = sign | ((exp + 112) << 23) | (man << 13);
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

uint16_t f2h(float f) {  // round to nearest even
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u, a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0));
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);
  if (a < 0x38800000u) {
    float v;
    std::memcpy(&v, &a, 4);
    return (uint16_t)(sign | (uint32_t)std::nearbyint(v * 16777216.0f));
  }
  uint32_t h = (((a >> 23) - 112) << 10) | ((a & 0x7fffffu) >> 13);
  const uint32_t rem = a & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h += 1;
  return (uint16_t)(sign | h);
}

float b2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

uint16_t f2b(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

template <typename T>
T iop(int op, T x, T y) {
  using U = typename std::make_unsigned<T>::type;
  switch (op) {
    case mccsDevSum: return (T)((U)x + (U)y);
    case mccsDevProd: return (T)((U)x * (U)y);
    case mccsDevMax: return x < y ? y : x;
    default: return x < y ? x : y;
  }
}

template <typename T>
T fop(int op, T x, T y) {
  switch (op) {
    case mccsDevSum: return x + y;
    case mccsDevProd: return x * y;
    case mccsDevMax: return x < y ? y : x;
    default: return x < y ? x : y;
  }
}

float hop(int op, float x, float y) {
  switch (op) {
    case mccsDevSum: return x + y;
    case mccsDevProd: return x * y;
    case mccsDevMax: return std::fmax(x, y);
    default: return std::fmin(x, y);
  }
}

// out[i] = fn(x[i], y[i]); out may alias either input
void apply(int dt, int op, void* out, const void* x, const void* y, size_t n) {
#define INT_CASE(D, T)                                                                       \
  case D:                                                                                    \
    for (size_t i = 0; i < n; ++i) ((T*)out)[i] = iop<T>(op, ((const T*)x)[i], ((const T*)y)[i]); \
    break;
  switch (dt) {
    INT_CASE(mccsInt8, int8_t)
    INT_CASE(mccsUint8, uint8_t)
    INT_CASE(mccsInt32, int32_t)
    INT_CASE(mccsUint32, uint32_t)
    INT_CASE(mccsInt64, int64_t)
    INT_CASE(mccsUint64, uint64_t)
    case mccsFloat32:
      for (size_t i = 0; i < n; ++i) ((float*)out)[i] = fop<float>(op, ((const float*)x)[i], ((const float*)y)[i]);
      break;
    case mccsFloat64:
      for (size_t i = 0; i < n; ++i)
        ((double*)out)[i] = fop<double>(op, ((const double*)x)[i], ((const double*)y)[i]);
      break;
    case mccsFloat16:
      for (size_t i = 0; i < n; ++i)
        ((uint16_t*)out)[i] = f2h(hop(op, h2f(((const uint16_t*)x)[i]), h2f(((const uint16_t*)y)[i])));
      break;
    case mccsBfloat16:
      for (size_t i = 0; i < n; ++i)
        ((uint16_t*)out)[i] = f2b(hop(op, b2f(((const uint16_t*)x)[i]), b2f(((const uint16_t*)y)[i])));
      break;
  }
#undef INT_CASE
}

size_t esize(int dt) {
  return (dt == mccsInt8 || dt == mccsUint8) ? 1
         : (dt == mccsFloat16 || dt == mccsBfloat16) ? 2
         : (dt == mccsInt32 || dt == mccsUint32 || dt == mccsFloat32) ? 4
         : 8;
}

struct HostConn {  // one directed FIFO (rank -> next) of one channel
  // uninitialised: only the slots a call touches are ever faulted in (a
  // zero-filled 4 MiB FIFO per connector cost ms per 1 KiB call)
  std::unique_ptr<char[]> data;
  // written by different threads (head: receiver, tail: sender): one cache
  // line each, so a post does not invalidate the line the other side polls
  alignas(64) std::atomic<uint64_t> head{0};
  alignas(64) std::atomic<uint64_t> tail{0};
};

struct Ctx {
  int n, nch, dt, op, nthreads_ref, buff_size;
  size_t es, count;
  const void* const* send;
  void* const* recv;
  const int* rings;  // nch x n, nullptr = identity
  std::vector<HostConn>* conns;  // [ch * n + rank]: FIFO rank -> next on channel ch
  std::atomic<int> failed{0};
  double timeout_s;
};

// one (rank, channel) thread executing runRing
void run_rank_channel(Ctx* c, int rank, int ch) {
  const int n = c->n;
  int ring[64];  // n <= 64 (mccs_host_ring_allreduce)
  for (int i = 0; i < n; ++i) ring[i] = c->rings ? c->rings[ch * n + i] : i;
  int pos = 0, pos0 = 0;
  for (int i = 0; i < n; ++i) {
    if (ring[i] == rank) pos = i;
    if (ring[i] == 0) pos0 = i;
  }
  const int next = ring[(pos + 1) % n], prev = ring[(pos + n - 1) % n];
  const int ringIx = (pos - pos0 + n) % n;
  HostConn& out = (*c->conns)[ch * n + rank];
  HostConn& in = (*c->conns)[ch * n + prev];
  (void)next;
  const int64_t stepSize = c->buff_size / MCCS_BUFFER_SLOTS / (int64_t)c->es;
  const int64_t chunkSize = (int64_t)(int)(stepSize * ALLREDUCE_CHUNKSTEPS);
  const int64_t size = (int64_t)c->count;
  const int64_t loopSize = (int64_t)c->nch * n * chunkSize;
  int64_t gran = (int64_t)(c->nthreads_ref - WARP_SIZE) * 8 / (int64_t)c->es;
  if (gran < 1) gran = 1;
  const char* input = (const char*)c->send[rank];
  char* output = (char*)c->recv[rank];
  uint64_t rstep = 0, sstep = 0;
  thread_local std::vector<char> tmp_store;  // this worker's staging slice, kept across calls
  if (tmp_store.size() < (size_t)(2 * stepSize * c->es)) tmp_store.resize((size_t)(2 * stepSize * c->es));
  char* const tmp = tmp_store.data();
  const auto t0 = std::chrono::steady_clock::now();
  auto wait_geq = [&](std::atomic<uint64_t>& f, uint64_t target) {
    // the peer is a running thread: spin (pause) before giving up the core
    for (int spin = 0; spin < 4096; ++spin) {
      if (f.load(std::memory_order_acquire) >= target) return true;
      __builtin_ia32_pause();
    }
    while (f.load(std::memory_order_acquire) < target) {
      if (c->failed.load(std::memory_order_relaxed)) return false;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
        c->failed.store(1);
        return false;
      }
      std::this_thread::yield();
    }
    return true;
  };
  // genericOp: RECV/SEND/SRC(input)/DST(output) flags, two slices per call
  auto op = [&](bool RECV, bool SEND, bool SRC, bool DST, int64_t srcIx, int64_t dstIx, int64_t nelem) {
    if (nelem < 0) nelem = 0;
    int64_t sliceSize = stepSize * ALLREDUCE_SLICESTEPS;
    const int64_t s = (nelem + 32 - 1) / 32 * 16;
    sliceSize = s > sliceSize / 32 ? s : sliceSize / 32;
    int64_t offset = 0;
    for (int slice = 0; slice < 2; ++slice) {
      int64_t real = nelem - offset;
      real = real < sliceSize ? real : sliceSize;
      if (real < 0) real = 0;
      if (RECV && !wait_geq(in.tail, rstep + 2)) return false;
      if (SEND && !wait_geq(out.head, sstep + 2 > 8 ? sstep + 2 - 8 : 0)) return false;
      const size_t bytes = (size_t)real * c->es;
      const char* rslot = in.data.get() + (rstep % 8) * stepSize * c->es;
      char* sslot = out.data.get() + (sstep % 8) * stepSize * c->es;
      if (bytes) {
        // vals = srcs[0]; vals = fn(vals, srcs[1]) with srcs = [input?, recv?]
        if (SRC && RECV) apply(c->dt, c->op, tmp, input + (srcIx + offset) * c->es, rslot, (size_t)real);
        else if (SRC) std::memcpy(tmp, input + (srcIx + offset) * c->es, bytes);
        else std::memcpy(tmp, rslot, bytes);
        if (DST) std::memcpy(output + (dstIx + offset) * c->es, tmp, bytes);
        if (SEND) std::memcpy(sslot, tmp, bytes);
      }
      // a call whose elements all fit in this slice posts the steps of its
      // remaining (empty) slices with this one: the same step counts as a
      // post per slice, one cross-thread hand-off instead of two
      const int64_t adv = offset + sliceSize >= nelem ? 2 * (2 - slice) : 2;
      if (SEND) out.tail.store(sstep + adv, std::memory_order_release);
      if (RECV) in.head.store(rstep + adv, std::memory_order_release);
      if (RECV) rstep += adv;
      if (SEND) sstep += adv;
      if (adv > 2) break;
      offset += sliceSize;
    }
    return true;
  };
  auto mod = [&](int r) { return r >= n ? r - n : r; };
  for (int64_t g = 0; g < size; g += loopSize) {
    int64_t rcs = (size - g + (int64_t)c->nch * n - 1) / ((int64_t)c->nch * n);
    rcs = chunkSize < rcs ? chunkSize : rcs;
    rcs = (int64_t)(int)((rcs + gran - 1) / gran * gran);
    auto off = [&](int chunk) { return g + (int64_t)ch * n * rcs + (int64_t)chunk * rcs; };
    auto ne = [&](int64_t o) { return rcs < size - o ? rcs : size - o; };
    int chunk = mod(ringIx + n - 1);
    if (!op(false, true, true, false, off(chunk), 0, ne(off(chunk)))) return;
    for (int j = 2; j < n; ++j) {
      chunk = mod(ringIx + n - j);
      if (!op(true, true, true, false, off(chunk), 0, ne(off(chunk)))) return;
    }
    chunk = ringIx;
    if (!op(true, true, true, true, off(chunk), off(chunk), ne(off(chunk)))) return;
    for (int j = 1; j < n - 1; ++j) {
      chunk = mod(ringIx + n - j);
      if (!op(true, true, false, true, 0, off(chunk), ne(off(chunk)))) return;
    }
    chunk = mod(ringIx + 1);
    if (!op(true, false, false, true, 0, off(chunk), ne(off(chunk)))) return;
  }
}

// Parked worker threads, one per concurrent (rank, channel) task: every task
// of a call must run at the same time (they spin on each other's FIFO flags),
// so task i >= 1 always goes to worker i and task 0 runs on the caller.  Workers spin briefly after a call (back
// to back calls wake them in ~1 us) and then sleep on a condition variable.
class HostRingPool {
 public:
  static HostRingPool& get() {
    static HostRingPool* p = new HostRingPool();  // never destroyed: workers stay parked at exit
    return *p;
  }
  std::mutex call_mu;

  // FIFOs of `nconn` connectors of `bytes` each, counters reset
  std::vector<HostConn>& fifos(size_t nconn, size_t bytes) {
    if (conns_.size() != nconn || conn_bytes_ != bytes) {
      conns_ = std::vector<HostConn>(nconn);
      for (auto& hc : conns_) hc.data.reset(new char[bytes]);
      conn_bytes_ = bytes;
    }
    for (auto& hc : conns_) {
      hc.head.store(0, std::memory_order_relaxed);
      hc.tail.store(0, std::memory_order_relaxed);
    }
    return conns_;
  }

  // Task 0 runs on the calling thread; tasks 1.. go to parked workers 1..
  // (a 2-rank call wakes one worker).  The job, its task count and the
  // generation change together under mu_, and a worker reads them together
  // under mu_, so a worker that lagged behind a call it had no task in
  // cannot pair an old generation with a newer job.
  void run(Ctx* c, int ntasks) {
    while ((int)workers_.size() < ntasks - 1) {
      const int id = (int)workers_.size() + 1;
      workers_.emplace_back([this, id] { loop(id); });
    }
    remaining_.store(ntasks - 1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu_);  // also pairs with a sleeper's predicate check
      job_.store(c, std::memory_order_relaxed);
      ntasks_.store(ntasks, std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);
    }
    if (sleepers_.load(std::memory_order_acquire)) cv_.notify_all();
    run_rank_channel(c, 0, 0);
    for (int spin = 0; remaining_.load(std::memory_order_acquire) != 0; ++spin) {
      if (spin < 4096) __builtin_ia32_pause();
      else std::this_thread::yield();
    }
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      // spin ~200 us for the next call, then sleep
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; gen_.load(std::memory_order_acquire) == seen; ++i) {
        __builtin_ia32_pause();
        if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
      }
      if (gen_.load(std::memory_order_acquire) == seen) {
        std::unique_lock<std::mutex> lk(mu_);
        sleepers_.fetch_add(1, std::memory_order_acq_rel);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
        sleepers_.fetch_sub(1, std::memory_order_acq_rel);
      }
      Ctx* c;
      int ntasks;
      {
        std::lock_guard<std::mutex> lk(mu_);
        seen = gen_.load(std::memory_order_acquire);
        c = job_.load(std::memory_order_relaxed);
        ntasks = ntasks_.load(std::memory_order_relaxed);
      }
      if (id < ntasks) {
        run_rank_channel(c, id / c->nch, id % c->nch);
        remaining_.fetch_sub(1, std::memory_order_acq_rel);
      }
    }
  }

  std::vector<std::thread> workers_;
  std::vector<HostConn> conns_;
  size_t conn_bytes_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> remaining_{0};
  std::atomic<int> sleepers_{0};
  std::atomic<Ctx*> job_{nullptr};
  std::atomic<int> ntasks_{0};
};

}  // namespace

extern "C" mccsResult_t mccs_host_ring_allreduce(int nranks, const void* const* sendbufs, void* const* recvbufs,
                                                 size_t count, int dtype, int op, int nchannels, int nthreads_ref,
                                                 int buff_size, const int* rings) {
  if (nranks < 1 || nranks > 64 || !sendbufs || !recvbufs || dtype < 0 || dtype >= mccsNumTypes || op < 0 ||
      op > mccsDevMin || nchannels < 1 || nchannels > MCCS_MAX_NCHANNELS || nthreads_ref <= WARP_SIZE ||
      buff_size < 8192 || buff_size % 8192)
    return mccsInvalidArgument;
  const size_t es = esize(dtype);
  if (nranks == 1) {
    if (recvbufs[0] != sendbufs[0]) std::memmove(recvbufs[0], sendbufs[0], count * es);
    return mccsSuccess;
  }
  HostRingPool& pool = HostRingPool::get();
  std::lock_guard<std::mutex> call(pool.call_mu);  // one host-ring AllReduce at a time
  std::vector<HostConn>& conns = pool.fifos((size_t)nchannels * nranks, (size_t)buff_size);
  Ctx c;
  c.n = nranks;
  c.nch = nchannels;
  c.dt = dtype;
  c.op = op;
  c.nthreads_ref = nthreads_ref;
  c.buff_size = buff_size;
  c.es = es;
  c.count = count;
  c.send = sendbufs;
  c.recv = recvbufs;
  c.rings = rings;
  c.conns = &conns;
  c.timeout_s = 60.0;
  pool.run(&c, nranks * nchannels);
  return c.failed.load() ? mccsTimeout : mccsSuccess;
}

// rt.cpp — HIP implementation of the device-runtime seam (rt.h) and the
// recording fake CPU tests install to drive the multi-device path without
// GPUs.
#include "rt.h"

#include <dlfcn.h>
#include <signal.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "comm.h"

namespace mccs {

namespace {

// Every failing call's error is returned and also cleared from HIP's
// per-thread last error: callers see it once, through the return value, and
// no later hipGetLastError() (torch checks one after each of its kernel
// launches) reports a failure of ours that was already handled.
class HipRuntime final : public DeviceRuntime {
  static hipError_t ret(hipError_t e) {
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
  }

 public:
  hipError_t GetDeviceCount(int* n) override { return ret(hipGetDeviceCount(n)); }
  hipError_t GetDevice(int* d) override { return ret(hipGetDevice(d)); }
  hipError_t SetDevice(int d) override { return ret(hipSetDevice(d)); }
  hipError_t Malloc(void** p, size_t bytes) override { return ret(hipMalloc(p, bytes)); }
  hipError_t MallocUncached(void** p, size_t bytes) override {
    return ret(hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached));
  }
  bool IsUncached(void* p) override {
    hipPointerAttribute_t attr;
    std::memset(&attr, 0, sizeof(attr));
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return attr.allocationFlags == hipDeviceMallocUncached;
  }
  hipError_t Free(void* p) override { return ret(hipFree(p)); }
  hipError_t Memset(void* p, int v, size_t bytes) override { return ret(hipMemset(p, v, bytes)); }
  hipError_t Memcpy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind) override {
    return ret(hipMemcpy(dst, src, bytes, kind));
  }
  hipError_t HostMallocMapped(void** p, size_t bytes) override { return ret(hipHostMalloc(p, bytes, hipHostMallocMapped)); }
  hipError_t HostGetDevicePointer(void** d, void* h) override { return ret(hipHostGetDevicePointer(d, h, 0)); }
  hipError_t HostFree(void* p) override { return ret(hipHostFree(p)); }
  hipError_t DeviceSynchronize() override { return ret(hipDeviceSynchronize()); }
  hipError_t FlushCaches() override { return ret(ring_flush_caches(nullptr)); }
  hipError_t CanAccessPeer(int* can, int dev, int peer) override { return ret(hipDeviceCanAccessPeer(can, dev, peer)); }
  hipError_t P2PAtomics(int* ok, int dev, int peer) override {
    if (dev == peer) {
      *ok = 1;
      return hipSuccess;
    }
    return ret(hipDeviceGetP2PAttribute(ok, hipDevP2PAttrNativeAtomicSupported, dev, peer));
  }
  hipError_t EnablePeerAccess(int peer) override {
    hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) e = hipSuccess;
    (void)hipGetLastError();
    return e;
  }
  hipError_t EventCreate(hipEvent_t* e, unsigned flags) override { return ret(hipEventCreateWithFlags(e, flags)); }
  hipError_t EventDestroy(hipEvent_t e) override { return ret(hipEventDestroy(e)); }
  hipError_t EventRecord(hipEvent_t e, hipStream_t s) override { return ret(hipEventRecord(e, s)); }
  hipError_t EventSynchronize(hipEvent_t e) override { return ret(hipEventSynchronize(e)); }
  hipError_t EventQuery(hipEvent_t e) override { return ret(hipEventQuery(e)); }
  hipError_t StreamCreate(hipStream_t* s) override { return ret(hipStreamCreateWithFlags(s, hipStreamNonBlocking)); }
  hipError_t StreamDestroy(hipStream_t s) override { return ret(hipStreamDestroy(s)); }
  hipError_t StreamSynchronize(hipStream_t s) override { return ret(hipStreamSynchronize(s)); }
  hipError_t StreamWaitEvent(hipStream_t s, hipEvent_t e) override { return ret(hipStreamWaitEvent(s, e, 0)); }
  // hipStreamGetId is a ROCm 7.1 symbol: resolved at run time, since the
  // process may already hold an older libamdhip64 (torch's own, ROCm 7.0, on
  // this image).  Without it the stream's address stands in for its id; torch
  // never destroys its streams (a per-device pool), so there addresses do not
  // come back as new streams.
  using StreamIdFn = hipError_t (*)(hipStream_t, unsigned long long*);
  static StreamIdFn stream_id_fn() {
    static const StreamIdFn fn = (StreamIdFn)dlsym(RTLD_DEFAULT, "hipStreamGetId");
    return fn;
  }
  hipError_t StreamId(hipStream_t s, unsigned long long* id) override {
    const StreamIdFn fn = stream_id_fn();
    static const bool logged = [&] {  // which key tells streams apart, once per process
      if (std::getenv("MCCS_DEBUG"))
        std::fprintf(stderr, "[mccs] streams told apart by %s\n",
                     fn ? "hipStreamGetId" : "address (hipStreamGetId absent from the loaded HIP runtime)");
      return true;
    }();
    (void)logged;
    if (!fn) {
      *id = (unsigned long long)(uintptr_t)s;
      return hipSuccess;
    }
    return ret(fn(s, id));
  }
  hipError_t StreamIsCapturing(hipStream_t s, bool* capturing) override {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    hipError_t e = hipStreamIsCapturing(s, &st);
    *capturing = st == hipStreamCaptureStatusActive;
    return ret(e);
  }
  hipError_t CaptureGraph(hipStream_t s, hipGraph_t* g) override {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    *g = nullptr;
    return ret(hipStreamGetCaptureInfo_v2(s, &st, nullptr, g, nullptr, nullptr));
  }
  hipError_t GraphOnDestroy(hipGraph_t g, void (*fn)(void*), void* arg) override {
    hipUserObject_t obj = nullptr;
    hipError_t e = hipUserObjectCreate(&obj, arg, fn, 1, hipUserObjectNoDestructorSync);
    if (e != hipSuccess) return ret(e);
    // the graph takes over the one reference; on failure the object (and so
    // the callback) is left unreleased: what it guards stays held
    return ret(hipGraphRetainUserObject(g, obj, 1, hipGraphUserObjectMove));
  }
  hipError_t LaunchKernel(const void* fn, dim3 grid, dim3 block, void** args, hipStream_t s) override {
    return ret(hipLaunchKernel(fn, grid, block, args, 0, s));
  }
  hipError_t LaunchKernelExt(const void* fn, dim3 grid, dim3 block, void** args, hipStream_t s,
                             hipEvent_t stop) override {
    return ret(hipExtLaunchKernel(fn, grid, block, args, 0, s, nullptr, stop, 0));
  }
  hipError_t BlocksPerCu(int* per_cu, const void* fn, int block) override {
    return ret(hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, fn, block, 0));
  }
  hipError_t CuCount(int* ncu, int device) override {
    return ret(hipDeviceGetAttribute(ncu, hipDeviceAttributeMultiprocessorCount, device));
  }
  hipError_t IpcGetMemHandle(hipIpcMemHandle_t* h, void* p) override { return ret(hipIpcGetMemHandle(h, p)); }
  hipError_t IpcOpenMemHandle(void** p, hipIpcMemHandle_t h) override {
    return ret(hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess));
  }
  hipError_t IpcCloseMemHandle(void* p) override { return ret(hipIpcCloseMemHandle(p)); }
  hipError_t DeviceGetPCIBusId(char* id, int len, int device) override { return ret(hipDeviceGetPCIBusId(id, len, device)); }
  hipError_t DeviceGetByPCIBusId(int* device, const char* id) override { return ret(hipDeviceGetByPCIBusId(device, id)); }
  bool ProcessGone(int pid) override { return pid > 0 && kill(pid, 0) != 0 && errno == ESRCH; }
};

// Recording fake: "device" memory is host memory tagged with its device,
// nothing executes, and every call that orders work or makes the host wait
// is appended to a text log (one event per line):
//   launch dev=D grid=XxY block=B stream=S comms_on_dev=1
//   record dev=D event=E stream=S          stream_wait dev=D stream=S event=E event_dev=D2
//   host_wait what=event|stream|device|memcpy|error dev=D
//   peer dev=D peer=P                      flush dev=D
// Every call is also appended, by name, to a call trace, and any one call can
// be made to fail: arm(name, nth, err) fails the nth call of that name,
// counted from arming, with err (tests/test_setup_diag.py walks the setup path this way).
class FakeRuntime final : public DeviceRuntime {
 public:
  explicit FakeRuntime(int ndev) : ndev_(ndev) {}
  ~FakeRuntime() override {
    for (auto& kv : mem_) std::free(kv.first);
  }
  std::string log() {
    std::lock_guard<std::mutex> lk(mu_);
    return log_.str();
  }
  void clear() {
    std::lock_guard<std::mutex> lk(mu_);
    log_.str("");
  }
  std::string calls(bool clear) {
    std::lock_guard<std::mutex> lk(mu_);
    std::string s = calls_.str();
    if (clear) calls_.str("");
    return s;
  }
  void arm(const char* name, int nth, hipError_t err) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!name) {
      fail_.clear();
      return;
    }
    fail_[name] = Fail{nth, err, 0};
  }
  void delay(const char* name, int ms) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!name) delay_ms_.clear();
    else delay_ms_[name] = ms;
  }
  void live(int* blocks, int* events) {
    std::lock_guard<std::mutex> lk(mu_);
    if (blocks) *blocks = (int)mem_.size();
    if (events) *events = (int)events_.size();
  }
  hipError_t GetDeviceCount(int* n) override {
    if (hipError_t e = inj("GetDeviceCount")) return e;
    *n = ndev_;
    return hipSuccess;
  }
  hipError_t GetDevice(int* d) override {
    *d = cur_;
    return hipSuccess;
  }
  hipError_t SetDevice(int d) override {
    if (d < 0 || d >= ndev_) return hipErrorInvalidDevice;
    cur_ = d;
    return hipSuccess;
  }
  hipError_t Malloc(void** p, size_t bytes) override {
    if (hipError_t e = inj("Malloc")) return e;
    return alloc(p, bytes, false);
  }
  hipError_t MallocUncached(void** p, size_t bytes) override {
    if (hipError_t e = inj("MallocUncached")) return e;
    return alloc(p, bytes, true);
  }
  bool IsUncached(void* p) override {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = mem_.find(p);
    return it != mem_.end() && it->second.uncached;
  }
  hipError_t Free(void* p) override {
    if (hipError_t e = inj("Free")) return e;
    return release(p);
  }
  hipError_t Memset(void* p, int v, size_t bytes) override {
    if (hipError_t e = inj("Memset")) return e;
    std::memset(p, v, bytes);
    return hipSuccess;
  }
  hipError_t Memcpy(void* dst, const void* src, size_t bytes, hipMemcpyKind) override {
    if (hipError_t e = inj("Memcpy")) return e;
    std::memcpy(dst, src, bytes);
    note("host_wait what=memcpy dev=" + std::to_string(cur_));
    return hipSuccess;
  }
  hipError_t HostMallocMapped(void** p, size_t bytes) override {
    if (hipError_t e = inj("HostMallocMapped")) return e;
    return alloc(p, bytes, false);
  }
  hipError_t HostGetDevicePointer(void** d, void* h) override {
    if (hipError_t e = inj("HostGetDevicePointer")) return e;
    *d = h;
    return hipSuccess;
  }
  hipError_t HostFree(void* p) override {
    if (hipError_t e = inj("HostFree")) return e;
    return release(p);
  }
  hipError_t DeviceSynchronize() override {
    if (hipError_t e = inj("DeviceSynchronize")) return e;
    note("host_wait what=device dev=" + std::to_string(cur_));
    return hipSuccess;
  }
  hipError_t FlushCaches() override {
    if (hipError_t e = inj("FlushCaches")) return e;
    note("flush dev=" + std::to_string(cur_));
    return hipSuccess;
  }
  hipError_t CanAccessPeer(int* can, int dev, int peer) override {
    if (hipError_t e = inj("CanAccessPeer")) return e;
    *can = dev >= 0 && dev < ndev_ && peer >= 0 && peer < ndev_;
    return hipSuccess;
  }
  hipError_t EnablePeerAccess(int peer) override {
    if (hipError_t e = inj("EnablePeerAccess")) return e;
    note("peer dev=" + std::to_string(cur_) + " peer=" + std::to_string(peer));
    return hipSuccess;
  }
  hipError_t P2PAtomics(int* ok, int dev, int peer) override {
    if (hipError_t e = inj("P2PAtomics")) return e;
    *ok = dev >= 0 && dev < ndev_ && peer >= 0 && peer < ndev_ && !std::getenv("MCCS_TEST_NO_P2P_ATOMICS");
    return hipSuccess;
  }
  hipError_t EventCreate(hipEvent_t* e, unsigned) override {
    if (hipError_t r = inj("EventCreate")) return r;
    std::lock_guard<std::mutex> lk(mu_);
    const uintptr_t id = ++next_id_;
    events_[id] = cur_;
    *e = (hipEvent_t)id;
    return hipSuccess;
  }
  hipError_t EventDestroy(hipEvent_t e) override {
    if (hipError_t r = inj("EventDestroy")) return r;
    std::lock_guard<std::mutex> lk(mu_);
    events_.erase((uintptr_t)e);
    return hipSuccess;
  }
  hipError_t EventRecord(hipEvent_t e, hipStream_t s) override {
    if (hipError_t r = inj("EventRecord")) return r;
    if (quiet_) return hipSuccess;
    note("record dev=" + std::to_string(cur_) + " event=" + std::to_string((uintptr_t)e) + " stream=" + sid(s));
    return hipSuccess;
  }
  hipError_t EventSynchronize(hipEvent_t e) override {
    if (hipError_t r = inj("EventSynchronize")) return r;
    note("host_wait what=event dev=" + std::to_string(event_dev(e)) + " event=" + std::to_string((uintptr_t)e));
    return hipSuccess;
  }
  hipError_t EventQuery(hipEvent_t) override { return inj("EventQuery"); }
  hipError_t StreamCreate(hipStream_t* s) override {
    if (hipError_t e = inj("StreamCreate")) return e;
    std::lock_guard<std::mutex> lk(mu_);
    *s = (hipStream_t)(++next_id_);
    return hipSuccess;
  }
  hipError_t StreamDestroy(hipStream_t) override { return inj("StreamDestroy"); }
  hipError_t StreamSynchronize(hipStream_t s) override {
    if (hipError_t e = inj("StreamSynchronize")) return e;
    note("host_wait what=stream dev=" + std::to_string(cur_) + " stream=" + sid(s));
    return hipSuccess;
  }
  hipError_t StreamWaitEvent(hipStream_t s, hipEvent_t e) override {
    if (hipError_t r = inj("StreamWaitEvent")) return r;
    if (quiet_) return hipSuccess;
    note("stream_wait dev=" + std::to_string(cur_) + " stream=" + sid(s) + " event=" +
         std::to_string((uintptr_t)e) + " event_dev=" + std::to_string(event_dev(e)));
    return hipSuccess;
  }
  hipError_t StreamId(hipStream_t s, unsigned long long* id) override {
    if (hipError_t e = inj("StreamId")) return e;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = stream_ids_.find(s);
    if (it == stream_ids_.end()) it = stream_ids_.emplace(s, ++next_stream_id_).first;
    *id = it->second;
    return hipSuccess;
  }
  // A stream destroyed and created again at the same address: a new id.
  void recreate_stream(hipStream_t s) {
    std::lock_guard<std::mutex> lk(mu_);
    stream_ids_.erase(s);
  }
  hipError_t StreamIsCapturing(hipStream_t s, bool* capturing) override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      *capturing = capture_.count(s) > 0;
    }
    return inj("StreamIsCapturing");
  }
  hipError_t CaptureGraph(hipStream_t s, hipGraph_t* g) override {
    if (hipError_t e = inj("CaptureGraph")) return e;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = capture_.find(s);
    if (it == capture_.end()) return hipErrorStreamCaptureUnmatched;
    *g = (hipGraph_t)(uintptr_t)it->second;
    return hipSuccess;
  }
  hipError_t GraphOnDestroy(hipGraph_t g, void (*fn)(void*), void* arg) override {
    if (hipError_t e = inj("GraphOnDestroy")) return e;
    std::lock_guard<std::mutex> lk(mu_);
    on_destroy_[(int)(uintptr_t)g].emplace_back(fn, arg);
    return hipSuccess;
  }
  // test hooks: a stream "captures" into graph id `graph` (0 ends it), and a
  // "destroyed" graph runs the callbacks registered on it
  void capture(hipStream_t s, int graph) {
    std::lock_guard<std::mutex> lk(mu_);
    if (graph > 0) capture_[s] = graph;
    else capture_.erase(s);
  }
  int destroy_graph(int graph) {
    std::vector<std::pair<void (*)(void*), void*>> fns;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fns.swap(on_destroy_[graph]);
      on_destroy_.erase(graph);
    }
    for (auto& f : fns) f.first(f.second);
    return (int)fns.size();
  }
  hipError_t LaunchKernelExt(const void* fn, dim3 grid, dim3 block, void** args, hipStream_t s,
                             hipEvent_t stop) override {
    stop_ = stop;
    const hipError_t e = LaunchKernel(fn, grid, block, args, s);
    stop_ = nullptr;
    return e;
  }
  hipError_t LaunchKernel(const void* fn, dim3 grid, dim3 block, void** args, hipStream_t s) override {
    if (hipError_t e = inj("LaunchKernel")) return e;
    if (quiet_) {
      ack_fifo_works(fn, grid, args);
      return hipSuccess;
    }
    // every communicator of a fused ring launch must live on the launching device
    bool on_dev = true;
    unsigned inl = 0;
    std::string extra;
    bool direct = false;
    for (int dt = 0; dt < mccsNumTypes && fn; ++dt)
      for (int op = 0; op < 4; ++op) direct = direct || fn == direct_kernel_ptr(dt, op);
    if (fn && args && grid.y >= 1 && grid.y <= MCCS_MULTI_MAX_RANKS) {
      if (direct) {  // mccsDirectArgs: the walk it reproduces
        const mccsDirectArgs* da = (const mccsDirectArgs*)args[0];
        for (unsigned k = 0; k < grid.y; ++k) on_dev = on_dev && dev_of(da->r[k].comm) == cur_;
        extra = " count=" + std::to_string(da->count) + " nch=" + std::to_string(da->nch) +
                " nthr=" + std::to_string(da->nthr_ref) + " fence=" + std::to_string(da->fence_mode) +
                " mode=" + (da->mode == MCCS_DIRECT_ONE_SHOT      ? "oneshot"
                            : da->mode == MCCS_DIRECT_AG_ONE_SHOT ? "ag-oneshot"
                            : da->mode == MCCS_DIRECT_LL_ONE_SHOT ? "ll"
                            : da->mode == MCCS_DIRECT_LL_AG       ? "ll-ag"
                                                                  : "twoshot") +
                " gx=" + std::to_string(grid.x) + " llslot=" + std::to_string(da->ll_slot_bytes) +
                " piece=" + std::to_string(da->piece) + " piece2=" + std::to_string(da->piece2) +
                " guard_order=" + std::to_string(da->guard_order) + " no_guard=" + std::to_string(da->no_guard) +
                " owned=";
        for (unsigned t = 0; t < da->nranks && t < MCCS_DIRECT_MAX_RANKS; ++t)
          extra += (t ? "," : "") + std::to_string(da->owned[t]);
      } else {
        const mccsMultiLaunchArgs* ma = (const mccsMultiLaunchArgs*)args[0];
        for (unsigned k = 0; k < grid.y; ++k) on_dev = on_dev && dev_of(ma->comm[k]) == cur_;
        inl = ma->inline_works;
        extra = " fence=" + std::to_string(ma->cfg.fence_mode) + " guard_order=" + std::to_string(ma->guard_order) +
                " no_guard=" + std::to_string(ma->cfg.no_guard);
      }
    }
    note("launch dev=" + std::to_string(cur_) + " grid=" + std::to_string(grid.x) + "x" + std::to_string(grid.y) +
         " block=" + std::to_string(block.x) + " stream=" + sid(s) + " comms_on_dev=" + (on_dev ? "1" : "0") +
         " inline_works=" + std::to_string(inl) + " stop_event=" + std::to_string((uintptr_t)stop_) +
         " kind=" + (direct ? "direct" : "ring") + extra);
    return hipSuccess;
  }
  // Quiet fake: what a ring kernel reading its works from the work FIFO
  // does to the host (common.h:153-155): each channel's last work stores its
  // doneAcks, so a loop of FIFO launches does not fill the FIFO.
  void ack_fifo_works(const void* fn, dim3 grid, void** args) {
    if (!fn || !args || grid.y < 1 || grid.y > MCCS_MULTI_MAX_RANKS) return;
    for (int dt = 0; dt < mccsNumTypes; ++dt)
      for (int op = 0; op < 4; ++op)
        if (fn == direct_kernel_ptr(dt, op)) return;
    const mccsMultiLaunchArgs* ma = (const mccsMultiLaunchArgs*)args[0];
    if (ma->inline_works) return;
    const int nch = __builtin_popcountll(ma->channelMask);
    for (unsigned k = 0; k < grid.y; ++k) {
      const mccsDevCommAndChannels* cc = (const mccsDevCommAndChannels*)ma->comm[k];
      uint64_t m = ma->channelMask;
      for (int i = 0; i < nch; ++i, m &= m - 1) {
        const int ch = __builtin_ctzll(m);
        const mccsDevWork* w = ma->work[k] + i;
        while (!w->header.isLast) w = ma->work[k] + w->header.workNext;
        if (w->header.inFifo) *cc->channels[ch].workFifoDone = w->header.doneAcks;
      }
    }
  }
  hipError_t BlocksPerCu(int* per_cu, const void*, int) override {
    *per_cu = 1;
    return inj("BlocksPerCu");
  }
  hipError_t CuCount(int* ncu, int) override {
    *ncu = 256;
    return inj("CuCount");
  }
  // IPC within one process: the handle carries the block's address (every
  // fake "process" is this one), opening checks that the block is alive
  hipError_t IpcGetMemHandle(hipIpcMemHandle_t* h, void* p) override {
    if (hipError_t e = inj("IpcGetMemHandle")) return e;
    std::lock_guard<std::mutex> lk(mu_);
    if (!mem_.count(p)) return hipErrorInvalidValue;
    std::memset(h, 0, sizeof(*h));
    std::memcpy(h->reserved, "FAKEIPC", 8);
    std::memcpy(h->reserved + 8, &p, sizeof(p));
    return hipSuccess;
  }
  hipError_t IpcOpenMemHandle(void** p, hipIpcMemHandle_t h) override {
    if (hipError_t e = inj("IpcOpenMemHandle")) return e;
    void* q = nullptr;
    std::memcpy(&q, h.reserved + 8, sizeof(q));
    std::lock_guard<std::mutex> lk(mu_);
    if (std::memcmp(h.reserved, "FAKEIPC", 8) != 0 || !mem_.count(q)) return hipErrorInvalidValue;
    ++ipc_open_[q];
    *p = q;
    return hipSuccess;
  }
  hipError_t IpcCloseMemHandle(void* p) override {
    if (hipError_t e = inj("IpcCloseMemHandle")) return e;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = ipc_open_.find(p);
    if (it == ipc_open_.end()) return hipErrorInvalidValue;
    if (--it->second == 0) ipc_open_.erase(it);
    return hipSuccess;
  }
  hipError_t DeviceGetPCIBusId(char* id, int len, int device) override {
    if (hipError_t e = inj("DeviceGetPCIBusId")) return e;
    if (device < 0 || device >= ndev_) return hipErrorInvalidDevice;
    std::snprintf(id, (size_t)len, "0000:%02x:00.0", 0x10 + device);
    return hipSuccess;
  }
  hipError_t DeviceGetByPCIBusId(int* device, const char* id) override {
    if (hipError_t e = inj("DeviceGetByPCIBusId")) return e;
    unsigned bus = 0;
    if (std::sscanf(id, "0000:%x:00.0", &bus) != 1 || bus < 0x10 || (int)bus - 0x10 >= ndev_)
      return hipErrorInvalidValue;
    *device = (int)bus - 0x10;
    return hipSuccess;
  }
  // Every fake "process" is this one: a peer pid counts as exited only once a
  // test says so (mccs_test_fake_process_exit).
  bool ProcessGone(int pid) override {
    std::lock_guard<std::mutex> lk(mu_);
    return std::find(exited_.begin(), exited_.end(), pid) != exited_.end();
  }
  void process_exit(int pid) {
    std::lock_guard<std::mutex> lk(mu_);
    exited_.push_back(pid);
  }

 private:
  std::vector<int> exited_;
  struct Block {
    int device;
    bool uncached;
  };
  struct Fail {
    int nth;  // 1-based among this name's calls since arming; 0 = every call
    hipError_t err;
    int seen;
  };
  // Traces the call, sleeps for its armed delay (outside the lock: other
  // threads' calls go on meanwhile), and returns the armed error for it, if
  // this is the one.
  hipError_t inj(const char* name) {
    if (quiet_) return hipSuccess;
    int delay = 0;
    hipError_t e = hipSuccess;
    {
      std::lock_guard<std::mutex> lk(mu_);
      calls_ << name << '\n';
      auto d = delay_ms_.find(name);
      if (d != delay_ms_.end()) delay = d->second;
      auto it = fail_.find(name);
      if (it != fail_.end()) {
        Fail& f = it->second;
        ++f.seen;
        if (f.nth == 0 || f.seen == f.nth) e = f.err;
      }
    }
    if (delay > 0) std::this_thread::sleep_for(std::chrono::milliseconds(delay));
    return e;
  }
  hipError_t alloc(void** p, size_t bytes, bool uncached) {
    void* q = std::calloc(1, bytes ? bytes : 1);
    if (!q) return hipErrorOutOfMemory;
    std::lock_guard<std::mutex> lk(mu_);
    mem_[q] = Block{cur_, uncached};
    *p = q;
    return hipSuccess;
  }
  hipError_t release(void* p) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = mem_.find(p);
    if (it == mem_.end()) return hipErrorInvalidValue;
    std::free(p);
    mem_.erase(it);
    return hipSuccess;
  }
  int dev_of(const void* p) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = mem_.find(const_cast<void*>(p));
    return it == mem_.end() ? -1 : it->second.device;
  }
  int event_dev(hipEvent_t e) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = events_.find((uintptr_t)e);
    return it == events_.end() ? -1 : it->second;
  }
  static std::string sid(hipStream_t s) { return std::to_string((uintptr_t)s); }
  void note(const std::string& line) {
    if (quiet_) return;
    std::lock_guard<std::mutex> lk(mu_);
    log_ << line << '\n';
  }

 public:
  std::atomic<bool> quiet_{false};  // no event log (host-cost measurements of the library itself)

 private:
  int ndev_, cur_ = 0;
  hipEvent_t stop_ = nullptr;  // the stop event of the launch being logged (LaunchKernelExt)
  uintptr_t next_id_ = 0;
  std::mutex mu_;
  std::map<void*, Block> mem_;
  std::map<uintptr_t, int> events_;
  std::map<void*, int> ipc_open_;
  std::map<std::string, Fail> fail_;
  std::map<std::string, int> delay_ms_;
  std::map<hipStream_t, int> capture_;
  std::map<hipStream_t, unsigned long long> stream_ids_;
  unsigned long long next_stream_id_ = 0;
  std::map<int, std::vector<std::pair<void (*)(void*), void*>>> on_destroy_;
  std::ostringstream log_, calls_;
};

HipRuntime g_hip;
// The installed fake (owned by g_fake_owner) is published through an atomic
// pointer so rt() never reads a half-swapped unique_ptr; install / removal is
// serialised by g_fake_mu.  Test-only contract: no communicator created under
// one runtime is used or destroyed under another.
std::mutex g_fake_mu;
std::unique_ptr<FakeRuntime> g_fake_owner;
std::atomic<FakeRuntime*> g_fake{nullptr};
// 0 = the HIP runtime; every fake install gets a fresh nonzero id, so arenas
// pooled under HIP stay reusable across fake install / remove cycles
std::atomic<unsigned> g_generation{0};
unsigned g_fake_serial = 0;

}  // namespace

DeviceRuntime& rt() {
  FakeRuntime* f = g_fake.load(std::memory_order_acquire);
  return f ? (DeviceRuntime&)*f : (DeviceRuntime&)g_hip;
}

void rt_use_fake(int ndevices) {
  std::lock_guard<std::mutex> lk(g_fake_mu);
  const unsigned old = g_generation.load();
  std::unique_ptr<FakeRuntime> next(ndevices > 0 ? new FakeRuntime(ndevices) : nullptr);
  g_fake.store(next.get(), std::memory_order_release);
  g_generation.store(ndevices > 0 ? ++g_fake_serial : 0u);
  g_fake_owner.swap(next);  // the previous fake (if any) dies with `next` below
  if (old != 0) comm_pool_drop_generation(old);  // its arenas were its host memory
}

unsigned rt_generation() { return g_generation.load(); }

bool rt_stream_ids_native() { return HipRuntime::stream_id_fn() != nullptr; }

}  // namespace mccs

// ---- test-only C-ABI (tests/test_multidevice_launch.py) -------------------
// Installs (ndevices > 0) or removes (0) the recording fake runtime.  Only
// communicators created while it is installed may be used with it.  Refused
// (mccsInvalidUsage) unless MCCS_TEST_HOOKS=1 is set in the environment, so
// no production caller can swap the device runtime by accident.
extern "C" mccsResult_t mccs_test_fake_runtime(int ndevices) {
  const char* hooks = std::getenv("MCCS_TEST_HOOKS");
  if (!hooks || std::atoi(hooks) != 1) return mccsInvalidUsage;
  if (ndevices < 0 || ndevices > 64) return mccsInvalidArgument;
  mccs::rt_use_fake(ndevices);
  return mccsSuccess;
}

// Copies the fake runtime's event log (NUL-terminated, truncated to cap) and
// optionally clears it; returns the log length, or -1 without a fake.
extern "C" int mccs_test_fake_log(char* buf, int cap, int clear) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  const std::string s = f->log();
  if (buf && cap > 0) {
    const size_t n = std::min(s.size(), (size_t)cap - 1);
    std::memcpy(buf, s.data(), n);
    buf[n] = '\0';
  }
  if (clear) f->clear();
  return (int)s.size();
}

// Fails the nth call (1-based, counted from now; 0 = every call) of the fake
// runtime's method `call` (its DeviceRuntime name, e.g. "HostMallocMapped")
// with hipError_t `err`; call = NULL disarms every injection.  -1 without a fake.
extern "C" int mccs_test_fake_fail(const char* call, int nth, int err) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  f->arm(call, nth, (hipError_t)err);
  return 0;
}

// The fake's call trace (method names, one a line) since the last clear; same
// contract as mccs_test_fake_log.
extern "C" int mccs_test_fake_calls(char* buf, int cap, int clear) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  const std::string s = f->calls(clear != 0);
  if (buf && cap > 0) {
    const size_t n = std::min(s.size(), (size_t)cap - 1);
    std::memcpy(buf, s.data(), n);
    buf[n] = '\0';
  }
  return (int)s.size();
}

// Live fake allocations (device + host blocks) and events, and the FIFO
// arenas the process pool holds (pooled arenas stay allocated by design).
extern "C" int mccs_test_fake_live(int* blocks, int* events, int* pooled) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  f->live(blocks, events);
  if (pooled) *pooled = mccs::comm_pool_count(mccs::rt_generation());
  return 0;
}

// Makes every call of the fake's method `call` sleep `ms` milliseconds before
// returning (lock-holding tests: ADVICE r04); call = NULL clears all delays.
extern "C" int mccs_test_fake_delay(const char* call, int ms) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  f->delay(call, ms);
  return 0;
}

// Simulates hipStreamDestroy + hipStreamCreate returning the same address:
// the fake stream `stream` gets a new id.
extern "C" int mccs_test_fake_recreate_stream(void* stream) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  f->recreate_stream((hipStream_t)stream);
  return 0;
}

// Quiet fake (1): no event log, no call trace, no injected failures or
// delays, so a loop of collectives on it times the library's own host path
// (tools/host_overhead.c --fake).  -1 without a fake.
extern "C" int mccs_test_fake_quiet(int quiet) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  f->quiet_ = quiet != 0;
  return 0;
}

// Marks the fake stream `stream` (a handle value as the library's callers
// pass it) as capturing into graph id `graph` (> 0), or ends its capture (0).
extern "C" int mccs_test_fake_capture(void* stream, int graph) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  f->capture((hipStream_t)stream, graph);
  return 0;
}

// "Destroys" fake graph `graph`: runs the callbacks registered on it (the HIP
// user objects' destructors); returns how many ran, -1 without a fake.
extern "C" int mccs_test_fake_destroy_graph(int graph) {
  mccs::FakeRuntime* f;
  {
    std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
    f = mccs::g_fake.load();
  }
  return f ? f->destroy_graph(graph) : -1;
}

// Marks fake peer process `pid` as exited and reaped (the arena pool's
// liveness check, DeviceRuntime::ProcessGone); -1 without a fake.
extern "C" int mccs_test_fake_process_exit(int pid) {
  std::lock_guard<std::mutex> lk(mccs::g_fake_mu);
  mccs::FakeRuntime* f = mccs::g_fake.load();
  if (!f) return -1;
  f->process_exit(pid);
  return 0;
}

// Pooled FIFO arenas of the current runtime still awaiting a peer's release
// (comm.cpp pool; tests of the release protocol).
extern "C" int mccs_test_pool_waiting(void) { return mccs::comm_pool_waiting(mccs::rt_generation()); }

// 1 when streams are told apart by hipStreamGetId (the loaded HIP runtime has
// it: ROCm >= 7.1), 0 when by address (an older runtime, e.g. torch's ROCm 7.0
// libamdhip64 loaded first).  plan.cpp orders a comm's launch on another stream
// after its previous one by this key.
extern "C" int mccs_stream_id_native(void) { return mccs::rt_stream_ids_native() ? 1 : 0; }

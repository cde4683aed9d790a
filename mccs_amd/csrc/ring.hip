// ring.hip — AllGather ring kernel, kernel tables and device-wide helpers of
// the ring path.  The device engine is ring_kernel.h; the forty AllReduce
// kernels live in ring_ar_{sum,prod,max,min}.hip (one translation unit per
// reduction op, compiled in parallel).
#include "ring_kernel.h"

namespace mccs {
int comm_fifo_slots_of(const void* d_comm);  // host/comm.cpp
}

#include <hip/hip_ext.h>

#include <mutex>
#include <vector>

extern "C" __global__ void __launch_bounds__(MCCS_RING_MAX_THREADS)
    mccsKernel_AllGather_RING_SIMPLE_Sum_int8_t(mccsDevComm* comm, uint64_t channelMask, mccsDevWork* workHead) {
  mccs::ring_kernel_body<mccsFuncAllGather, mccsInt8, mccs::OpSum>(comm, channelMask, workHead, blockIdx.x,
                                                                    gridDim.x, mccs::kRefCfg);
}

MCCS_RING_TU_ACCESSORS(ag)

// ---- host-side kernel tables ------------------------------------------------
namespace mccs {

const void* ring_ar_kernel_Sum(int dtype, bool multi);
const void* ring_ar_kernel_Prod(int dtype, bool multi);
const void* ring_ar_kernel_Max(int dtype, bool multi);
const void* ring_ar_kernel_Min(int dtype, bool multi);
hipError_t ring_tu_ar_sum_read_profile(unsigned long long* out, bool reset);
hipError_t ring_tu_ar_prod_read_profile(unsigned long long* out, bool reset);
hipError_t ring_tu_ar_max_read_profile(unsigned long long* out, bool reset);
hipError_t ring_tu_ar_min_read_profile(unsigned long long* out, bool reset);
hipError_t ring_tu_ag_set_ref_watchdog(unsigned long long ticks);
hipError_t ring_tu_ar_sum_set_ref_watchdog(unsigned long long ticks);
hipError_t ring_tu_ar_prod_set_ref_watchdog(unsigned long long ticks);
hipError_t ring_tu_ar_max_set_ref_watchdog(unsigned long long ticks);
hipError_t ring_tu_ar_min_set_ref_watchdog(unsigned long long ticks);

static const void* ar_kernel(int dtype, int op, bool multi) {
  if (dtype < 0 || dtype >= mccsNumTypes) return nullptr;
  switch (op) {
    case OpSum: return ring_ar_kernel_Sum(dtype, multi);
    case OpProd: return ring_ar_kernel_Prod(dtype, multi);
    case OpMax: return ring_ar_kernel_Max(dtype, multi);
    case OpMin: return ring_ar_kernel_Min(dtype, multi);
  }
  return nullptr;
}

const void* ring_kernel_ptr(int func, int dtype, int op) {
  if (func == mccsFuncAllGather) return (const void*)&mccsKernel_AllGather_RING_SIMPLE_Sum_int8_t;
  if (func != mccsFuncAllReduce) return nullptr;
  return ar_kernel(dtype, op, false);
}

const void* ring_multi_kernel_ptr(int func, int dtype, int op) {
  if (func == mccsFuncAllGather) return (const void*)&ring_multi_kernel<mccsFuncAllGather, mccsInt8, OpSum>;
  if (func != mccsFuncAllReduce) return nullptr;
  return ar_kernel(dtype, op, true);
}

// Writes back and invalidates every XCD's L2 and the CUs' L1 (system-scope
// release + acquire in many workgroups so all eight XCDs run one).  Used after
// (re)allocating FIFO arenas: a freshly mapped range may still have lines in
// an L2 from its previous life under another memory type.
__global__ void cache_flush_kernel() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
}

// Returns the launch's own status.  It used to return hipGetLastError(),
// which also reports any failure an earlier call left on the calling thread
// (the caller's, torch's, a handled one of ours): communicator setup then
// failed on an error that was not its own (tests/test_setup_diag.py).
hipError_t ring_flush_caches(hipStream_t st) {
  return hipLaunchKernel((const void*)cache_flush_kernel, dim3(2048), dim3(64), nullptr, 0, st);
}

// Reads (and optionally zeroes) the current device's ring profile counters,
// summed over the translation units that hold ring kernels.
hipError_t ring_read_profile(unsigned long long* out, bool reset) {
  for (int i = 0; i < MCCS_PROF_N; ++i) out[i] = 0;
  hipError_t (*const readers[])(unsigned long long*, bool) = {
      ring_tu_ag_read_profile, ring_tu_ar_sum_read_profile, ring_tu_ar_prod_read_profile,
      ring_tu_ar_max_read_profile, ring_tu_ar_min_read_profile};
  for (auto rd : readers) {
    hipError_t e = rd(out, reset);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace mccs

extern "C" const void* mccs_hip_coll_kernel(int func, int dtype, int op) {
  return mccs::ring_kernel_ptr(func, dtype, op);
}

namespace {
// External launches still in flight, per device: a rank of another
// communicator on the same device must not be launched beside them
// (mccs_hip.h: co-located ranks need one fused launch).
struct ExtLaunch {
  int device;
  const mccsDevComm* comm;
  hipEvent_t done;
};
std::mutex g_ext_mu;
std::vector<ExtLaunch> g_ext;

// true if another communicator's external launch on `device` is unfinished;
// forgets finished ones
bool colocated_launch_running(int device, const mccsDevComm* comm) {
  bool busy = false;
  for (size_t i = 0; i < g_ext.size();) {
    ExtLaunch& x = g_ext[i];
    if (x.device == device && x.comm != comm) {
      const hipError_t q = hipEventQuery(x.done);
      if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        busy = true;
        ++i;
        continue;
      }
      if (q != hipSuccess) (void)hipGetLastError();  // a failed launch's event: forget it, leave no stale error
      (void)hipEventDestroy(x.done);
      g_ext.erase(g_ext.begin() + i);
      continue;
    }
    ++i;
  }
  return busy;
}
}  // namespace

// The reference-named kernels' watchdog on the current device (every
// translation unit holds its own copy): ms without FIFO progress before a
// kernel raises abortFlag; 0 = the 10 min default, < 0 = none.
extern "C" mccsResult_t mccs_hip_set_ref_watchdog(int timeout_ms) {
  const unsigned long long ticks =
      timeout_ms < 0 ? 0ull : (unsigned long long)(timeout_ms == 0 ? 600000 : timeout_ms) * 100000ull;
  hipError_t (*const set[])(unsigned long long) = {
      mccs::ring_tu_ag_set_ref_watchdog, mccs::ring_tu_ar_sum_set_ref_watchdog, mccs::ring_tu_ar_prod_set_ref_watchdog,
      mccs::ring_tu_ar_max_set_ref_watchdog, mccs::ring_tu_ar_min_set_ref_watchdog};
  for (auto f : set)
    if (f(ticks) != hipSuccess) {
      (void)hipGetLastError();
      return mccsUnhandledCudaError;
    }
  return mccsSuccess;
}

extern "C" mccsResult_t mccs_hip_launch_coll(int func, int dtype, int op, mccsDevComm* comm, uint64_t channelMask,
                                             mccsDevWork* workHead, unsigned grid, unsigned block,
                                             hipStream_t stream) {
  const void* fn = mccs::ring_kernel_ptr(func, dtype, op);
  // blocks of one wave have no control wave (ring_kernel.h); the reference
  // host never launches fewer than 96 threads (get_task_schema, plan.rs:602-635)
  if (!fn || !comm || !workHead || grid == 0 || block <= 64 || block > MCCS_RING_MAX_THREADS) return mccsInvalidArgument;
  // a communicator of this library with a deeper FIFO ring: the kernels below
  // index the reference's 8 slots (kRefCfg), its peers' launches would not
  const int fs = mccs::comm_fifo_slots_of(comm);
  if (fs != 0 && fs != MCCS_BUFFER_SLOTS) return mccsInvalidUsage;
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return mccsUnhandledCudaError;
  std::lock_guard<std::mutex> lk(g_ext_mu);
  if (colocated_launch_running(device, comm)) return mccsInvalidUsage;
  void* args[3] = {&comm, &channelMask, &workHead};
  // the co-location guard's event rides on the dispatch's completion signal
  // (no marker packet behind the kernel, tools/launch_cost.hip); a capturing
  // stream gets a plain kernel node and a recorded event
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) != hipSuccess) return mccsUnhandledCudaError;
  const bool capturing = cap == hipStreamCaptureStatusActive;
  // this comm's entry (its latest launch) is reused eagerly: re-recording the
  // event moves it to the newest launch, which is what the guard asks about
  ExtLaunch* mine = nullptr;
  for (auto& x : g_ext)
    if (x.device == device && x.comm == comm) mine = &x;
  hipEvent_t done = (mine && !capturing) ? mine->done : nullptr;
  if (!done && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) return mccsUnhandledCudaError;
  hipError_t e = capturing ? hipLaunchKernel(fn, dim3(grid), dim3(block), args, 0, stream)
                           : hipExtLaunchKernel(fn, dim3(grid), dim3(block), args, 0, stream, nullptr, done, 0);
  if (e == hipSuccess && capturing) e = hipEventRecord(done, stream);
  if (e != hipSuccess) {
    if (!mine || done != mine->done) (void)hipEventDestroy(done);
    return mccsUnhandledCudaError;
  }
  if (mine && mine->done != done) {  // a captured launch replaced the entry's event
    (void)hipEventDestroy(mine->done);
    mine->done = done;
  } else if (!mine) {
    g_ext.push_back(ExtLaunch{device, comm, done});
  }
  return mccsSuccess;
}

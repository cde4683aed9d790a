// launch_cost.hip — device-side cost of the completion-tracking choices for
// back-to-back stream-ordered launches on MI355X (the question behind the
// ring's comm event, DESIGN.md §1 "Comm events only when consumed").
//
// A one-block kernel spins for ~8 us (s_memrealtime, 100 MHz); N launches go
// back to back on one stream in each mode, wall time per launch after a
// warm-up:
//   plain        hipLaunchKernel
//   +record      hipLaunchKernel + hipEventRecord(ev) after every launch
//   ext-stop     hipExtLaunchKernel(..., stopEvent = ev): the event rides on
//                the dispatch packet's completion signal
//   ext-stop-t   the same with a timing-enabled event
//   graph        the N plain launches captured in one graph and replayed
//
//   hipcc --offload-arch=gfx950 -O2 -o launch_cost tools/launch_cost.hip && ./launch_cost
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  const unsigned long long ticks = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 800;  // 8 us
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev, evt;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreate(&evt));
  void* args[1] = {(void*)&ticks};
  const void* fn = (const void*)&spin_kernel;
  auto run = [&](int mode, int count) -> hipError_t {
    for (int i = 0; i < count; ++i) {
      hipError_t e = hipSuccess;
      if (mode == 0 || mode == 1) e = hipLaunchKernel(fn, dim3(1), dim3(64), args, 0, st);
      if (mode == 1 && e == hipSuccess) e = hipEventRecord(ev, st);
      if (mode == 2) e = hipExtLaunchKernel(fn, dim3(1), dim3(64), args, 0, st, nullptr, ev, 0);
      if (mode == 3) e = hipExtLaunchKernel(fn, dim3(1), dim3(64), args, 0, st, nullptr, evt, 0);
      if (e != hipSuccess) return e;
    }
    return hipStreamSynchronize(st);
  };
  const char* names[] = {"plain", "+record", "ext-stop", "ext-stop-t"};
  std::printf("{\"tool\": \"launch_cost\", \"launches\": %d, \"kernel_us\": %.1f, \"us_per_launch\": {", n,
              ticks / 100.0);
  for (int rep = 0; rep < 2; ++rep) {
    for (int mode = 0; mode < 4; ++mode) {
      CK(run(mode, 50));
      const auto t0 = std::chrono::steady_clock::now();
      CK(run(mode, n));
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
      std::printf("%s\"%s_r%d\": %.2f", (rep || mode) ? ", " : "", names[mode], rep, us);
    }
    // graph of n plain launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; ++i) CK(hipLaunchKernel(fn, dim3(1), dim3(64), args, 0, st));
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    const auto t0 = std::chrono::steady_clock::now();
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    std::printf(", \"graph_r%d\": %.2f", rep, us);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  std::printf("}");
  // semantics of the stop event: not complete while the kernel runs, complete
  // after it; another stream waiting on it starts after the kernel
  {
    const unsigned long long long_ticks = 20000000ull;  // 200 ms
    void* largs[1] = {(void*)&long_ticks};
    CK(hipStreamSynchronize(st));
    const auto t0 = std::chrono::steady_clock::now();
    CK(hipExtLaunchKernel(fn, dim3(1), dim3(64), largs, 0, st, nullptr, ev, 0));
    const hipError_t q0 = hipEventQuery(ev);
    hipStream_t st2;
    CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
    CK(hipStreamWaitEvent(st2, ev, 0));
    hipEvent_t ev2;
    CK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
    CK(hipEventRecord(ev2, st2));
    const hipError_t q2 = hipEventQuery(ev2);  // st2 waits on ev: not done while the kernel runs
    CK(hipEventSynchronize(ev));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const hipError_t q1 = hipEventQuery(ev);
    CK(hipEventSynchronize(ev2));
    std::printf(", \"stop_event\": {\"query_while_running_not_ready\": %s, \"sync_waited_ms\": %.1f, "
                "\"query_after_success\": %s, \"waiting_stream_held\": %s}}\n",
                q0 == hipErrorNotReady ? "true" : "false", ms, q1 == hipSuccess ? "true" : "false",
                q2 == hipErrorNotReady ? "true" : "false");
    (void)hipGetLastError();
  }
  return 0;
}

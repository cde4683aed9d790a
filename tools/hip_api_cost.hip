// hip_api_cost.hip — HOST microseconds per HIP runtime call on the eager
// launch path of a collective (GroupEnd costs 11.4 us
// for the ring, the raw launch 2.5-4.2 us; which calls make up the rest?).
//
// Each call is issued `n` times on one non-blocking stream (kernels are
// empty, 1 workgroup) and timed alone on the host; the median is reported.  Launch variants carry a 1 KiB argument block (the ring's
// mccsMultiLaunchArgs is 832 B) or 8 B:
//   launch            hipLaunchKernel
//   launch+stop       hipExtLaunchKernel with a stop event (the library's
//                     default: the comm event rides on the dispatch)
//   launch+record     hipLaunchKernel + hipEventRecord
//   module            hipModuleLaunchKernel on the kernel's hipFunction_t
//                     (hipGetFuncBySymbol once; no per-call symbol lookup)
//   module+stop       hipExtModuleLaunchKernel with a stop event
//   GetDevice, SetDevice(current), StreamIsCapturing, StreamGetId,
//   EventQuery (a completed event), StreamWaitEvent (completed event)
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/hip_api_cost tools/hip_api_cost.hip && tools/hip_api_cost
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <vector>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

struct Big {
  unsigned long long w[128];  // 1 KiB
};

__global__ void empty_big(Big b) {
  if (threadIdx.x == 1024) b.w[0] = 0;  // never: keeps the argument alive
}
__global__ void empty_small(unsigned long long x) {
  if (threadIdx.x == 1024 && x == 7) __builtin_trap();
}
// spins `ticks` of the 100 MHz constant clock (s_memrealtime): a kernel of a
// known device time, so the next call is issued while it runs
__global__ void busy(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

// Median host time of one call: each call timed alone, the stream drained
// every 16 calls outside the timed calls (so the device never falls behind
// and no call waits for queue space).
template <class F>
static double per_call_us(int n, F f, hipStream_t st) {
  for (int i = 0; i < 64; ++i) f();  // warm
  CK(hipStreamSynchronize(st));
  std::vector<double> t(n);
  for (int i = 0; i < n; ++i) {
    if (i % 16 == 0) CK(hipStreamSynchronize(st));
    const auto t0 = std::chrono::steady_clock::now();
    f();
    t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  CK(hipStreamSynchronize(st));
  std::sort(t.begin(), t.end());
  return t[n / 2];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 400;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev, done;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  CK(hipEventRecord(done, st));
  CK(hipStreamSynchronize(st));
  Big big{};
  unsigned long long small = 1;
  void* abig[1] = {&big};
  void* asmall[1] = {&small};
  const void* fb = (const void*)&empty_big;
  const void* fs = (const void*)&empty_small;
  hipFunction_t mb = nullptr, ms = nullptr;
  CK(hipGetFuncBySymbol(&mb, fb));
  CK(hipGetFuncBySymbol(&ms, fs));
  int dev = 0;
  CK(hipGetDevice(&dev));
  using Fn = hipError_t (*)(hipStream_t, unsigned long long*);
  Fn get_id = (Fn)hipStreamGetId;
  std::printf("{\"tool\": \"hip_api_cost\", \"calls\": %d, \"host_us_per_call\": {", n);
  bool first = true;
  auto row = [&](const char* name, double us) {
    std::printf("%s\"%s\": %.3f", first ? "" : ", ", name, us);
    first = false;
  };
  for (int big_args = 1; big_args >= 0; --big_args) {
    void** a = big_args ? abig : asmall;
    const void* f = big_args ? fb : fs;
    hipFunction_t m = big_args ? mb : ms;
    char nm[64];
    std::snprintf(nm, sizeof nm, "launch %s", big_args ? "1KiB" : "8B");
    row(nm, per_call_us(n, [&] { CK(hipLaunchKernel(f, dim3(1), dim3(64), a, 0, st)); }, st));
    std::snprintf(nm, sizeof nm, "launch+stop %s", big_args ? "1KiB" : "8B");
    row(nm, per_call_us(n, [&] { CK(hipExtLaunchKernel(f, dim3(1), dim3(64), a, 0, st, nullptr, ev, 0)); }, st));
    std::snprintf(nm, sizeof nm, "launch+record %s", big_args ? "1KiB" : "8B");
    row(nm, per_call_us(n, [&] {
          CK(hipLaunchKernel(f, dim3(1), dim3(64), a, 0, st));
          CK(hipEventRecord(ev, st));
        }, st));
    std::snprintf(nm, sizeof nm, "module %s", big_args ? "1KiB" : "8B");
    row(nm, per_call_us(n, [&] { CK(hipModuleLaunchKernel(m, 1, 1, 1, 64, 1, 1, 0, st, a, nullptr)); }, st));
    std::snprintf(nm, sizeof nm, "module+stop %s", big_args ? "1KiB" : "8B");
    row(nm, per_call_us(n, [&] {
          CK(hipExtModuleLaunchKernel(m, 64, 1, 1, 64, 1, 1, 0, st, a, nullptr, nullptr, ev, 0));
        }, st));
  }
  // launch+stop of kernels running 2 / 8 / 20 us, back to back on one event
  // (the LL one-shot's device time is ~8 us, the 8 MiB ring's ~21 us): does
  // the host cost depend on whether the previous dispatch is still running?
  for (unsigned long long us : {2ull, 8ull, 20ull}) {
    unsigned long long ticks = us * 100;
    void* ab[1] = {&ticks};
    char nm[64];
    std::snprintf(nm, sizeof nm, "launch+stop busy %lluus", us);
    row(nm, per_call_us(n, [&] { CK(hipExtLaunchKernel((const void*)&busy, dim3(1), dim3(64), ab, 0, st, nullptr, ev, 0)); }, st));
    std::snprintf(nm, sizeof nm, "launch busy %lluus", us);
    row(nm, per_call_us(n, [&] { CK(hipLaunchKernel((const void*)&busy, dim3(1), dim3(64), ab, 0, st)); }, st));
  }
  row("GetDevice", per_call_us(4 * n, [&] { int d; CK(hipGetDevice(&d)); }, st));
  row("SetDevice(current)", per_call_us(4 * n, [&] { CK(hipSetDevice(dev)); }, st));
  row("StreamIsCapturing", per_call_us(4 * n, [&] {
        hipStreamCaptureStatus s;
        CK(hipStreamIsCapturing(st, &s));
      }, st));
  row("StreamGetId", per_call_us(4 * n, [&] {
        unsigned long long id;
        CK(get_id(st, &id));
      }, st));
  row("EventQuery(done)", per_call_us(4 * n, [&] { CK(hipEventQuery(done)); }, st));
  row("StreamWaitEvent(done)", per_call_us(4 * n, [&] { CK(hipStreamWaitEvent(st, done, 0)); }, st));
  std::printf("}}\n");
  return 0;
}

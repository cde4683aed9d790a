// wg_stream.hip — how fast can ONE ring workgroup stream on MI355X?
//
// The reference launch shape (plan.rs:648-652, mccs.toml channel_count = 2)
// gives a 128 MiB AllReduce two 544-thread workgroups, so the depth-A drop-in
// is bound by one CU's streaming rate (VERDICT r03 "what's weak" 2).  This
// tool isolates that rate: G workgroups of 544 threads (8 data waves + a
// half wave that only waits, as the ring's control wave does), each streaming
// its own HBM region through the ring's slice shapes
//   RRCS  2 sources -> 2 destinations (recvReduceCopySend)
//   RRS   2 sources -> 1 destination  (recvReduceSend)
//   RCS   1 source  -> 2 destinations (recvCopySend)
// in slices of SL bytes per operand with a drain (vmcnt(0)) + workgroup
// barrier between slices, as the ring drains and counts out each slice.
// Loop designs:
//   reg   reduce_copy_rows (ring_kernel.h today): U packs per source per lane
//         loaded, reduced, stored, next pass
//   regpp the same with the next pass's loads issued before this pass's
//         stores (register double buffer)
//   lds   per-wave LDS-DMA ring: S stages of U KiB per source, S-1 tiles in
//         flight, counted vmcnt waits (lds_dma.h)
// Prints GB/s of HBM traffic per workgroup (loads + stores) per design.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I mccs_amd/csrc -I tools \
//       -o wg_stream tools/wg_stream.hip && ./wg_stream [G] [MiB per WG] [slice KiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lds_dma.h"
#include "reduce_copy.h"
#include "ring_stream.h"
#include "wg_stream_rows.h"

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

using namespace mccs;

constexpr int kBlock = 544;

// design: 0 reg, 1 regpp, 2 lds, 3 reg with dynamic wave units (ring_stream.h).  NTM: nt mask of the loads (bit 0 source 0,
// bit 1 source 1); P0 / P1: store policy of destination 0 / 1 (reduce_copy.h)
template <int DES, int U, int S, int NS, int ND, int NTM = 1, int P0 = kNonTemporal, int P1 = kPlain>
__global__ void __launch_bounds__(576) stream_kernel(const float* s0, const float* s1, float* d0, float* d1,
                                                     long per_wg, long slice) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t ctr[2];  // design 3: per-parity unit counters
  uint32_t cbase[2] = {0, 0};
  if (threadIdx.x == 0) ctr[0] = ctr[1] = 0;
  __syncthreads();
  int t = 0;
  const long base = (long)blockIdx.x * per_wg;
  const int nthr = blockDim.x;
  const int ndthr = (nthr / 64) * 64 == nthr ? nthr - 64 : (nthr / 64) * 64;  // whole waves, minus control
  const int wave = threadIdx.x >> 6;
  const bool data = threadIdx.x < ndthr;
  for (long off = 0; off < per_wg; off += slice) {
    const long n = slice < per_wg - off ? slice : per_wg - off;
    const float* a = s0 + base + off;
    const float* b = s1 + base + off;
    float* x = d0 + base + off;
    float* y = d1 + base + off;
    if (data) {
      if constexpr (DES == 0) {
        reduce_copy_rows<mccsFloat32, OpSum, U, NS, ND, NTM, P0, P1>(a, b, x, y, n, threadIdx.x, ndthr);
      } else if constexpr (DES == 1) {
        reduce_copy_rows_pp<mccsFloat32, OpSum, U, NS, ND, NTM, P0, P1>(a, b, x, y, n, threadIdx.x, ndthr);
      } else if constexpr (DES == 3) {
        cbase[t & 1] += reduce_copy_rows_dyn<mccsFloat32, OpSum, U, NS, ND, NTM, P0, P1>(
            a, b, x, y, n, threadIdx.x, ndthr, &ctr[t & 1], cbase[t & 1]);
      } else {
        const uint32_t lds = (uint32_t)(uintptr_t)smem + (uint32_t)(wave * S * NS * U * 1024);
        lds_stream_rows<mccsFloat32, OpSum, U, S, NS, ND, NTM, P0, P1>(a, b, x, y, n, threadIdx.x, ndthr, lds);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    ++t;
  }
}

struct Bufs {
  float *s0, *s1, *d0, *d1;
};

template <int DES, int U, int S, int NS, int ND, int NTM = 1, int P0 = kNonTemporal, int P1 = kPlain>
static void run(const char* name, const Bufs& b, int G, long per_wg, long slice, int iters) {
  auto k = stream_kernel<DES, U, S, NS, ND, NTM, P0, P1>;
  const size_t lds = DES == 2 ? (size_t)8 * S * NS * U * 1024 : 0;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k, dim3(G), dim3(kBlock), lds, 0, b.s0, b.s1, b.d0, b.d1, per_wg, slice);
  CK(hipGetLastError());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL(k, dim3(G), dim3(kBlock), lds, 0, b.s0, b.s1, b.d0, b.d1, per_wg, slice);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)per_wg * 4 * (NS + ND);  // per workgroup per launch
  std::printf("{\"design\": \"%s\", \"NS\": %d, \"ND\": %d, \"U\": %d, \"S\": %d, \"ntmask\": %d, \"st\": [%d, %d], "
              "\"G\": %d, \"slice_KiB\": %ld, \"us\": %.1f, \"GBps_per_wg\": %.1f}\n",
              name, NS, ND, U, S, NTM, P0, P1, G, slice * 4 / 1024, ms * 1e3 / iters, bytes / (ms * 1e-3 / iters) / 1e9);
  std::fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

// correctness of each design on one shape (RRCS, ragged length)
template <int DES, int U, int S>
static bool check(const Bufs& b, long n) {
  auto k = stream_kernel<DES, U, S, 2, 2>;
  const size_t lds = DES == 2 ? (size_t)8 * S * 2 * U * 1024 : 0;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  CK(hipMemset(b.d0, 0, n * 4));
  CK(hipMemset(b.d1, 0, n * 4));
  hipLaunchKernelGGL(k, dim3(1), dim3(kBlock), lds, 0, b.s0, b.s1, b.d0, b.d1, n, (long)(300001));
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<float> a(n), c(n), x(n), y(n);
  CK(hipMemcpy(a.data(), b.s0, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), b.s1, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(x.data(), b.d0, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), b.d1, n * 4, hipMemcpyDeviceToHost));
  for (long i = 0; i < n; ++i)
    if (x[i] != a[i] + c[i] || y[i] != x[i]) {
      std::printf("{\"check\": \"FAIL\", \"design\": %d, \"U\": %d, \"S\": %d, \"at\": %ld}\n", DES, U, S, i);
      return false;
    }
  return true;
}

__global__ void fill(float* p, long n, float k) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = (float)((i * 7 + (long)k) % 1000) * 0.25f;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? std::atoi(argv[1]) : 4;
  const long mib = argc > 2 ? std::atol(argv[2]) : 64;
  const long slice_kib = argc > 3 ? std::atol(argv[3]) : 1024;
  const int iters = argc > 4 ? std::atoi(argv[4]) : 3;
  const long per_wg = mib * (1L << 20) / 4;
  const long slice = slice_kib * 1024 / 4;
  const long total = per_wg * G;
  Bufs b;
  CK(hipMalloc(&b.s0, total * 4));
  CK(hipMalloc(&b.s1, total * 4));
  CK(hipMalloc(&b.d0, total * 4));
  CK(hipMalloc(&b.d1, total * 4));
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, b.s0, total, 1.0f);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, b.s1, total, 5.0f);
  CK(hipDeviceSynchronize());
  bool ok = check<0, 8, 1>(b, 1000003) && check<3, 8, 1>(b, 1000003) && check<3, 16, 1>(b, 3000017) &&
            check<1, 4, 1>(b, 1000003) && check<1, 8, 1>(b, 1000003) &&
            check<2, 4, 2>(b, 1000003) && check<2, 2, 4>(b, 1000003) && check<2, 2, 3>(b, 1000003);
  std::printf("{\"check\": \"%s\"}\n", ok ? "ok" : "FAIL");
  std::fflush(stdout);
  if (!ok) return 1;
  const int set = argc > 5 ? std::atoi(argv[5]) : 0;
  if (set == 0) {
    run<0, 8, 1, 2, 2>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2>("reg", b, G, per_wg, slice, iters);
    run<1, 8, 1, 2, 2>("regpp", b, G, per_wg, slice, iters);
    run<2, 4, 2, 2, 2>("lds", b, G, per_wg, slice, iters);
    run<0, 8, 1, 2, 1>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 1>("reg", b, G, per_wg, slice, iters);
    run<0, 8, 1, 1, 2>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 1, 2>("reg", b, G, per_wg, slice, iters);
  } else if (set == 3) {
    // static rows vs dynamic wave units, per slice shape
    run<0, 8, 1, 2, 2>("reg", b, G, per_wg, slice, iters);
    run<3, 8, 1, 2, 2>("dyn", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2>("reg", b, G, per_wg, slice, iters);
    run<3, 16, 1, 2, 2>("dyn", b, G, per_wg, slice, iters);
    run<0, 16, 1, 1, 1>("reg", b, G, per_wg, slice, iters);
    run<3, 16, 1, 1, 1>("dyn", b, G, per_wg, slice, iters);
    run<0, 16, 1, 1, 2>("reg", b, G, per_wg, slice, iters);
    run<3, 16, 1, 1, 2>("dyn", b, G, per_wg, slice, iters);
  } else if (set == 2) {
    // single-source slices (send 1 -> 1, recvCopySend 1 -> 2, recv 1 -> 1) at
    // the register budget of a 2-source pass: twice the packs
    run<0, 8, 1, 1, 1>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 1, 1>("reg", b, G, per_wg, slice, iters);
    run<0, 32, 1, 1, 1>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 1, 2>("reg", b, G, per_wg, slice, iters);
    run<0, 32, 1, 1, 2>("reg", b, G, per_wg, slice, iters);
    run<2, 8, 2, 1, 1>("lds", b, G, per_wg, slice, iters);
    run<2, 8, 2, 1, 2>("lds", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 1>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2>("reg", b, G, per_wg, slice, iters);
  } else {
    // cache policies at U = 16, 2 -> 2: loads (nt mask), stores (output, FIFO)
    run<0, 16, 1, 2, 2, 0, kPlain, kPlain>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2, 1, kNonTemporal, kPlain>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2, 3, kNonTemporal, kPlain>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2, 3, kNonTemporal, kNonTemporal>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2, 1, kWriteThrough, kPlain>("reg", b, G, per_wg, slice, iters);
    run<0, 16, 1, 2, 2, 1, kNonTemporal, kWriteThrough>("reg", b, G, per_wg, slice, iters);
    run<0, 12, 1, 2, 2>("reg", b, G, per_wg, slice, iters);
    run<0, 8, 1, 2, 2, 0, kPlain, kPlain>("reg", b, G, per_wg, slice, iters);
    run<0, 8, 1, 2, 2, 3, kNonTemporal, kNonTemporal>("reg", b, G, per_wg, slice, iters);
  }
  return 0;
}

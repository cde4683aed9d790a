// handoff_bench.hip — what one ring hop costs on MI355X, measured, for the
// protocol choice in DESIGN.md §9: two workgroups on one GPU ping-pong a
// payload through uncached (fine-grained) memory, the way ring neighbours
// hand slices over.
//
//   SIMPLE (the mCCS protocol, prims_simple.h): the producer streams the
//     payload with 16-byte stores, drains them (s_waitcnt vmcnt(0)), then
//     stores a step flag; the consumer polls the flag, then loads the payload.
//   LL (flag in data, NCCL's LL idea): every 8-byte word carries 4 bytes of
//     payload and a 4-byte step tag, so there is no drain and no separate
//     flag; the consumer polls the words themselves (2x the bytes moved).
//
// One round trip = A hands off to B, B hands the same amount back.  Reported:
// microseconds per one-way hop, averaged over `iters` round trips, for
// payloads of 1 KiB .. 256 KiB.  Build: hipcc --offload-arch=gfx950 -O3 -o
// tools/handoff_bench tools/handoff_bench.hip; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t ld_flag(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_flag(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Args {
  char* buf[2];       // payload buffer written by side s (read by the other side)
  uint64_t* flag[2];  // flag posted by side s
  uint64_t* ll[2];    // LL lines written by side s
  int bytes;
  int iters;
  int mode;  // 0 SIMPLE, 1 LL
  unsigned long long* out_ticks;
  unsigned long long* sink;
};

// side 0 = block 0, side 1 = block 1; 256 threads each.
__global__ void __launch_bounds__(256) pingpong(Args a) {
  const int side = blockIdx.x;
  const int tid = threadIdx.x;
  const int peer = side ^ 1;
  __shared__ int stop;
  if (tid == 0) stop = 0;
  __syncthreads();
  uint64_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < a.iters; ++it) {
    const uint64_t step = (uint64_t)it + 1;
    // side 0 sends first in every round trip, side 1 answers
    for (int phase = 0; phase < 2; ++phase) {
      const bool sending = (phase == 0) == (side == 0);
      if (a.mode == 0) {
        if (sending) {
          u32x4* dst = (u32x4*)a.buf[side];
          const int n16 = a.bytes / 16;
          for (int i = tid; i < n16; i += 256) {
            u32x4 v = {(unsigned)step, (unsigned)i, 0u, 0u};
            dst[i] = v;
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0) st_flag(a.flag[side], step);
        } else {
          if (tid == 0) {
            uint64_t spins = 0;
            while (ld_flag(a.flag[peer]) < step) {
              if (++spins > (1ull << 22)) { stop = 1; break; }
            }
          }
          __syncthreads();
          if (stop) break;
          const u32x4* src = (const u32x4*)a.buf[peer];
          const int n16 = a.bytes / 16;
          for (int i = tid; i < n16; i += 256) acc += __builtin_nontemporal_load(&src[i]).x;
        }
      } else {
        // LL: 8-byte words {payload (4 B), step tag (4 B)}; bytes of payload
        // -> bytes/4 words
        uint64_t* lines = a.ll[sending ? side : peer];
        const int nw = a.bytes / 4;
        if (sending) {
          for (int i = tid; i < nw; i += 256) {
            const uint64_t w = ((uint64_t)(uint32_t)step << 32) | (uint32_t)(i * 3 + 1);
            __hip_atomic_store(&lines[i], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        } else {
          for (int i = tid; i < nw; i += 256) {
            uint64_t w;
            uint64_t spins = 0;
            do {
              w = __hip_atomic_load(&lines[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              if (++spins > (1ull << 22)) break;
            } while ((uint32_t)(w >> 32) < (uint32_t)step);
            acc += (uint32_t)w;
          }
        }
        __syncthreads();
      }
    }
    if (stop) break;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) a.out_ticks[side] = t1 - t0;
  if (acc == 0x12345678ull) a.sink[0] = acc;  // keep the loads
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int sizes[] = {1024, 4096, 16384, 65536, 262144};
  Args a{};
  const size_t maxb = 262144;
  for (int s = 0; s < 2; ++s) {
    CHECK(hipExtMallocWithFlags((void**)&a.buf[s], maxb, hipDeviceMallocUncached));
    CHECK(hipExtMallocWithFlags((void**)&a.flag[s], 4096, hipDeviceMallocUncached));
    CHECK(hipExtMallocWithFlags((void**)&a.ll[s], maxb * 2, hipDeviceMallocUncached));
  }
  CHECK(hipMalloc(&a.out_ticks, 2 * sizeof(unsigned long long)));
  CHECK(hipMalloc(&a.sink, sizeof(unsigned long long)));
  std::printf("{\"iters\": %d, \"rows\": [", iters);
  bool first = true;
  for (int mode = 0; mode < 2; ++mode) {
    for (int bytes : sizes) {
      for (int s = 0; s < 2; ++s) {
        CHECK(hipMemset(a.buf[s], 0, maxb));
        CHECK(hipMemset(a.flag[s], 0, 4096));
        CHECK(hipMemset(a.ll[s], 0, maxb * 2));
      }
      CHECK(hipDeviceSynchronize());
      a.bytes = bytes;
      a.iters = iters;
      a.mode = mode;
      hipLaunchKernelGGL(pingpong, dim3(2), dim3(256), 0, 0, a);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      unsigned long long t[2];
      CHECK(hipMemcpy(t, a.out_ticks, sizeof(t), hipMemcpyDeviceToHost));
      // s_memrealtime: 100 MHz; a round trip is two hops
      const double hop_us = (double)t[0] / 100.0 / iters / 2.0;
      std::printf("%s{\"protocol\": \"%s\", \"payload_bytes\": %d, \"hop_us\": %.3f}", first ? "" : ", ",
                  mode == 0 ? "SIMPLE" : "LL", bytes, hop_us);
      first = false;
    }
  }
  std::printf("]}\n");
  return 0;
}

/*
 * host_overhead.c — host time per collective call through the C-ABI, the way
 * a Rust / C service issues them (no Python): mccsGroupStart, one
 * mccsAllReduce per rank of a 2-rank virtual node, mccsGroupEnd, repeated
 * without waiting, then one sync.  Reports the host microseconds per call
 * (issue rate) and the wall microseconds per call including the device
 * (back-to-back rate), for an LL-sized bucket (16 KiB), a one-shot-sized one
 * (512 KiB) and a ring one (8 MiB) at the library defaults.
 *
 *   gcc -std=c11 -O2 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/host_overhead.c \
 *       -Lmccs_amd -lmccs_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/mccs_amd -o tools/host_overhead
 *   tools/host_overhead [calls per size] [--fake]
 *
 * --fake (MCCS_TEST_HOOKS=1 in the environment; no GPU): the library's own
 * host path on the quiet recording fake runtime, every HIP call a no-op --
 * what the planner, the group state and the launch bookkeeping cost.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mccs_hip.h"

/* test hooks of libmccs_hip.so (csrc/host/rt.cpp), not part of the header:
   looked up at run time, so the tool also runs against a library without them */
typedef int (*hook_fn)(int);

enum { MAXS = 4096 };
static double one[MAXS];
static int cmp_double(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main(int argc, char** argv) {
  enum { NR = 2 };
  /* calls per size (default 2000); fewer than the HIP queue holds keeps the
     host from waiting for the device, so host_us_per_call is the issue cost */
  const int CALLS = argc > 1 ? atoi(argv[1]) : 2000;
  const int fake = argc > 2 && strcmp(argv[2], "--fake") == 0;
  if (fake) {
    hook_fn rt = (hook_fn)dlsym(RTLD_DEFAULT, "mccs_test_fake_runtime");
    hook_fn quiet = (hook_fn)dlsym(RTLD_DEFAULT, "mccs_test_fake_quiet");
    if (!rt || !quiet || rt(1) != mccsSuccess || quiet(1) != 0) return 6;
  }
  mccsComm_t comms[NR];
  int devices[NR] = {0, 0};
  if (mccsCommInitAll(comms, NR, devices, NULL) != mccsSuccess) return 1;
  hipStream_t st = (hipStream_t)0x7000;  /* a fake stream handle under --fake */
  if (!fake && hipStreamCreate(&st) != hipSuccess) return 1;
  const size_t sizes[3] = {16 << 10, 512 << 10, 8 << 20};
  void *buf[NR][2];
  for (int r = 0; r < NR; ++r)
    for (int k = 0; k < 2; ++k)
      if (fake) buf[r][k] = (void*)(uintptr_t)(0x10000000ull * (2 * r + k + 1));
      else if (hipMalloc(&buf[r][k], 8 << 20) != hipSuccess) return 1;
  printf("{\"what\": \"host time per call: GroupStart + 2 x mccsAllReduce + GroupEnd, 2-rank virtual node, fp32, library defaults\", \"rows\": [");
  for (int s = 0; s < 3; ++s) {
    const size_t count = sizes[s] / 4;
    for (int warm = 0; warm < 2; ++warm) {
      double t0 = now_us(), issue = 0, launch = 0;
      for (int i = 0; i < CALLS; ++i) {
        double a = now_us();
        mccsGroupStart();
        for (int r = 0; r < NR; ++r)
          if (mccsAllReduce(buf[r][0], buf[r][1], count, mccsFloat32, mccsDevSum, comms[r], st) != mccsSuccess) return 2;
        double b = now_us();
        if (mccsGroupEnd() != mccsSuccess) return 3;
        double e = now_us();
        issue += e - a;
        launch += e - b;
        if (i < MAXS) one[i] = e - a;
      }
      if (!fake && hipStreamSynchronize(st) != hipSuccess) return 4;
      for (int r = 0; r < NR; ++r)
        if (mccsCommSync(comms[r]) != mccsSuccess) return 5;
      const double wall = now_us() - t0;
      /* median of single calls, the device drained every 16 calls outside
         them: the issue cost with no wait for queue space */
      double med = 0;
      {
        const int m = 400;
        for (int i = 0; i < m; ++i) {
          if (i % 16 == 0) {
            if (!fake && hipStreamSynchronize(st) != hipSuccess) return 4;
          }
          double a = now_us();
          mccsGroupStart();
          for (int r = 0; r < NR; ++r)
            if (mccsAllReduce(buf[r][0], buf[r][1], count, mccsFloat32, mccsDevSum, comms[r], st) != mccsSuccess)
              return 2;
          if (mccsGroupEnd() != mccsSuccess) return 3;
          one[i] = now_us() - a;
        }
        if (!fake && hipStreamSynchronize(st) != hipSuccess) return 4;
        qsort(one, m, sizeof(double), cmp_double);
        med = one[m / 2];
      }
      if (warm)
        printf("%s{\"bytes\": %zu, \"algo\": %d, \"host_us_per_call\": %.2f, \"group_end_us\": %.2f, "
               "\"wall_us_per_call\": %.2f, \"host_us_median_drained\": %.2f}", s ? ", " : "", sizes[s],
               mccsCommLastAlgo(comms[0]), issue / CALLS, launch / CALLS, wall / CALLS, med);
    }
  }
  printf("]}\n");
  for (int r = 0; r < NR; ++r) mccsCommDestroy(comms[r]);
  return 0;
}

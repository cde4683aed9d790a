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
 */
#define _POSIX_C_SOURCE 199309L
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <time.h>

#include "mccs_hip.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main(void) {
  enum { NR = 2, CALLS = 2000 };
  mccsComm_t comms[NR];
  int devices[NR] = {0, 0};
  if (mccsCommInitAll(comms, NR, devices, NULL) != mccsSuccess) return 1;
  hipStream_t st;
  if (hipStreamCreate(&st) != hipSuccess) return 1;
  const size_t sizes[3] = {16 << 10, 512 << 10, 8 << 20};
  void *buf[NR][2];
  for (int r = 0; r < NR; ++r)
    for (int k = 0; k < 2; ++k)
      if (hipMalloc(&buf[r][k], 8 << 20) != hipSuccess) return 1;
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
      }
      if (hipStreamSynchronize(st) != hipSuccess) return 4;
      for (int r = 0; r < NR; ++r)
        if (mccsCommSync(comms[r]) != mccsSuccess) return 5;
      const double wall = now_us() - t0;
      if (warm)
        printf("%s{\"bytes\": %zu, \"algo\": %d, \"host_us_per_call\": %.2f, \"group_end_us\": %.2f, "
               "\"wall_us_per_call\": %.2f}", s ? ", " : "", sizes[s], mccsCommLastAlgo(comms[0]), issue / CALLS,
               launch / CALLS, wall / CALLS);
    }
  }
  printf("]}\n");
  for (int r = 0; r < NR; ++r) mccsCommDestroy(comms[r]);
  return 0;
}

/*
 * capi_allreduce.c — the C-ABI of libmccs_hip.so driven from plain C (what a
 * Rust / cgo / JNI binding of include/mccs_hip.h would do), no Python or torch:
 *
 *   1. mccsCommInitAll: two ranks on device 0 (the reference service model,
 *      one process driving every rank);
 *   2. the allreduce_proto known answer (src/mccs_examples/allreduce_proto/
 *      src/main.rs:27,75-116): rank r sends 2042 + r (int32, Sum), every
 *      element of every result must be 2042 * n + n (n - 1) / 2;
 *   3. an fp32 AllReduce of k/64 inputs (exact in any order) against the
 *      host sum;
 *   4. mccs_hip_reduce (the standalone chunk reduce) against the host sum;
 *   5. a stream destroyed with a collective still queued on it, a new stream
 *      created at once (HIP hands it the same address) and a collective
 *      issued on it: the library must tell the two streams apart by id
 *      (hipStreamGetId, which this process's ROCm 7.2 runtime has, unlike
 *      torch's ROCm 7.0 one) and order the second launch after the first,
 *      so the launch guard never sees the two overlap.
 *
 * Built by mccs_amd/build.py (gcc, C11) into tests/capi/capi_allreduce;
 * run by tests/test_gpu_capi.py.  Prints "capi ok" and exits 0 on success.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mccs_hip.h"

#define CHECK_MCCS(x)                                                            \
  do {                                                                           \
    mccsResult_t r_ = (x);                                                       \
    if (r_ != mccsSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, mccsGetErrorString(r_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)
#define CHECK_HIP(x)                                                             \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

enum { NR = 2, COUNT = 1000003 };

int main(void) {
  mccsComm_t comms[NR];
  int devices[NR] = {0, 0};
  CHECK_MCCS(mccsCommInitAll(comms, NR, devices, NULL));
  hipStream_t stream;
  CHECK_HIP(hipStreamCreate(&stream));

  /* 2. int32 known answer */
  int32_t* host = (int32_t*)malloc(sizeof(int32_t) * COUNT);
  void *send[NR], *recv[NR];
  for (int r = 0; r < NR; ++r) {
    CHECK_HIP(hipMalloc(&send[r], sizeof(int32_t) * COUNT));
    CHECK_HIP(hipMalloc(&recv[r], sizeof(int32_t) * COUNT));
    for (int i = 0; i < COUNT; ++i) host[i] = 2042 + r;
    CHECK_HIP(hipMemcpy(send[r], host, sizeof(int32_t) * COUNT, hipMemcpyHostToDevice));
  }
  CHECK_MCCS(mccsGroupStart());
  for (int r = 0; r < NR; ++r)
    CHECK_MCCS(mccsAllReduce(send[r], recv[r], COUNT, mccsInt32, mccsDevSum, comms[r], stream));
  CHECK_MCCS(mccsGroupEnd());
  for (int r = 0; r < NR; ++r) CHECK_MCCS(mccsCommSync(comms[r]));
  const int32_t kat = 2042 * NR + NR * (NR - 1) / 2;
  for (int r = 0; r < NR; ++r) {
    CHECK_HIP(hipMemcpy(host, recv[r], sizeof(int32_t) * COUNT, hipMemcpyDeviceToHost));
    for (int i = 0; i < COUNT; ++i)
      if (host[i] != kat) {
        fprintf(stderr, "int32 rank %d elem %d: %d != %d\n", r, i, host[i], kat);
        return 1;
      }
  }

  /* 3. fp32 exact-sum AllReduce */
  float* hf = (float*)malloc(sizeof(float) * COUNT);
  float* expf_ = (float*)calloc(COUNT, sizeof(float));
  for (int r = 0; r < NR; ++r) {
    for (int i = 0; i < COUNT; ++i) {
      hf[i] = (float)(((i * 7 + r * 13) % 511) - 255) / 64.0f;
      expf_[i] += hf[i];
    }
    CHECK_HIP(hipMemcpy(send[r], hf, sizeof(float) * COUNT, hipMemcpyHostToDevice));
  }
  CHECK_MCCS(mccsGroupStart());
  for (int r = 0; r < NR; ++r)
    CHECK_MCCS(mccsAllReduce(send[r], recv[r], COUNT, mccsFloat32, mccsDevSum, comms[r], stream));
  CHECK_MCCS(mccsGroupEnd());
  for (int r = 0; r < NR; ++r) CHECK_MCCS(mccsCommSync(comms[r]));
  for (int r = 0; r < NR; ++r) {
    CHECK_HIP(hipMemcpy(hf, recv[r], sizeof(float) * COUNT, hipMemcpyDeviceToHost));
    if (memcmp(hf, expf_, sizeof(float) * COUNT) != 0) {
      fprintf(stderr, "fp32 AllReduce rank %d differs from the exact sum\n", r);
      return 1;
    }
  }

  /* 4. standalone chunk reduce: recv[0] = send[0] + send[1] */
  const void* srcs[2] = {send[0], send[1]};
  CHECK_MCCS(mccs_hip_reduce(recv[0], srcs, 2, COUNT, mccsFloat32, mccsDevSum, stream));
  CHECK_HIP(hipStreamSynchronize(stream));
  CHECK_HIP(hipMemcpy(hf, recv[0], sizeof(float) * COUNT, hipMemcpyDeviceToHost));
  if (memcmp(hf, expf_, sizeof(float) * COUNT) != 0) {
    fprintf(stderr, "mccs_hip_reduce differs from the host sum\n");
    return 1;
  }

  /* 5. stream recreated at the same address */
  {
    enum { BIG = 1 << 24 };
    const int native = mccs_stream_id_native();
    printf("stream ids: %s\n", native ? "native" : "address");
    float *bs[NR], *br[NR], *cs[NR], *cr[NR];
    float* hb = (float*)malloc(sizeof(float) * BIG);
    float* eb = (float*)calloc(BIG, sizeof(float));
    float* ec = (float*)calloc(BIG, sizeof(float));
    for (int r = 0; r < NR; ++r) {
      CHECK_HIP(hipMalloc((void**)&bs[r], sizeof(float) * BIG));
      CHECK_HIP(hipMalloc((void**)&br[r], sizeof(float) * BIG));
      CHECK_HIP(hipMalloc((void**)&cs[r], sizeof(float) * BIG));
      CHECK_HIP(hipMalloc((void**)&cr[r], sizeof(float) * BIG));
      for (int i = 0; i < BIG; ++i) {
        hb[i] = (float)(((i * 5 + r * 11) % 509) - 254) / 64.0f;
        eb[i] += hb[i];
      }
      CHECK_HIP(hipMemcpy(bs[r], hb, sizeof(float) * BIG, hipMemcpyHostToDevice));
      for (int i = 0; i < BIG; ++i) {
        hb[i] = (float)(((i * 3 + r * 17) % 503) - 251) / 64.0f;
        ec[i] += hb[i];
      }
      CHECK_HIP(hipMemcpy(cs[r], hb, sizeof(float) * BIG, hipMemcpyHostToDevice));
    }
    unsigned long long waits0 = 0, waits1 = 0;
    uint64_t gi[4];
    for (int r = 0; r < NR; ++r) {
      CHECK_MCCS(mccsCommGuardInfo(comms[r], gi));
      waits0 += gi[3];
    }
    hipStream_t s1, s2;
    CHECK_HIP(hipStreamCreate(&s1));
    CHECK_MCCS(mccsGroupStart());
    for (int r = 0; r < NR; ++r)
      CHECK_MCCS(mccsAllReduce(bs[r], br[r], BIG, mccsFloat32, mccsDevSum, comms[r], s1));
    CHECK_MCCS(mccsGroupEnd());
    CHECK_HIP(hipStreamDestroy(s1)); /* the AllReduce is still queued or running */
    CHECK_HIP(hipStreamCreate(&s2));
    printf("recreated stream at the same address: %s\n", s2 == s1 ? "yes" : "no");
    CHECK_MCCS(mccsGroupStart());
    for (int r = 0; r < NR; ++r)
      CHECK_MCCS(mccsAllReduce(cs[r], cr[r], BIG, mccsFloat32, mccsDevSum, comms[r], s2));
    CHECK_MCCS(mccsGroupEnd());
    for (int r = 0; r < NR; ++r) CHECK_MCCS(mccsCommSync(comms[r]));
    CHECK_HIP(hipDeviceSynchronize());
    for (int r = 0; r < NR; ++r) {
      CHECK_MCCS(mccsCommGuardInfo(comms[r], gi));
      waits1 += gi[3];
      if (gi[0] || gi[1] || gi[2]) {
        fprintf(stderr, "rank %d's launch guard is not free after the sync\n", r);
        return 1;
      }
      CHECK_HIP(hipMemcpy(hb, br[r], sizeof(float) * BIG, hipMemcpyDeviceToHost));
      if (memcmp(hb, eb, sizeof(float) * BIG) != 0) {
        fprintf(stderr, "rank %d: the AllReduce on the destroyed stream differs from the exact sum\n", r);
        return 1;
      }
      CHECK_HIP(hipMemcpy(hb, cr[r], sizeof(float) * BIG, hipMemcpyDeviceToHost));
      if (memcmp(hb, ec, sizeof(float) * BIG) != 0) {
        fprintf(stderr, "rank %d: the AllReduce on the recreated stream differs from the exact sum\n", r);
        return 1;
      }
      CHECK_HIP(hipFree(bs[r]));
      CHECK_HIP(hipFree(br[r]));
      CHECK_HIP(hipFree(cs[r]));
      CHECK_HIP(hipFree(cr[r]));
    }
    /* ordered by the host (id branch): the second launch never waited on the guard */
    printf("guard waits: %llu\n", waits1 - waits0);
    if (native && waits1 != waits0) {
      fprintf(stderr, "the launch on the recreated stream overlapped the one on the destroyed stream\n");
      return 1;
    }
    CHECK_HIP(hipStreamDestroy(s2));
    free(hb);
    free(eb);
    free(ec);
  }

  for (int r = 0; r < NR; ++r) {
    CHECK_HIP(hipFree(send[r]));
    CHECK_HIP(hipFree(recv[r]));
    CHECK_MCCS(mccsCommDestroy(comms[r]));
  }
  CHECK_HIP(hipStreamDestroy(stream));
  free(host);
  free(hf);
  free(expf_);
  printf("capi ok (%s)\n", mccs_hip_version());
  return 0;
}

// shared.cpp — the application <-> backend bridge of libmccs, for callers
// that run the collectives in a separate backend process (the reference's
// mCCS service model):
//   cuda_malloc   (libmccs memory.rs:12-37)      -> mccsMemAllocShared / mccsMemOpenShared
//   register_stream (communicator.rs:47-66)      -> mccsEventCreateShared / mccsEventOpenShared
//   backend_event (communicator.rs:35-38)        -> mccsCommEventHandle
//   wait_user_event (proxy/engine.rs:1185-1189)  -> mccsCommWaitEvent (+ mccsCommStream)
// Handles are the 64-byte hipIpcMemHandle_t / hipIpcEventHandle_t, passed as
// opaque bytes so callers need no HIP headers.
#include <hip/hip_runtime.h>

#include <cstring>

#include "comm.h"

using namespace mccs;

static_assert(sizeof(hipIpcMemHandle_t) == MCCS_IPC_HANDLE_BYTES, "hipIpcMemHandle_t size");
static_assert(sizeof(hipIpcEventHandle_t) == MCCS_IPC_HANDLE_BYTES, "hipIpcEventHandle_t size");

extern "C" mccsResult_t mccsMemAllocShared(int device, size_t bytes, void** dptr, void* handle_out) {
  if (!dptr || !handle_out || bytes == 0) return mccsInvalidArgument;
  DeviceGuard g(device);
  void* p = nullptr;
  MCCS_HIP(hipMalloc(&p, bytes));
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipFree(p);
    return mccsUnhandledCudaError;
  }
  std::memcpy(handle_out, &h, sizeof(h));
  *dptr = p;
  return mccsSuccess;
}

extern "C" mccsResult_t mccsMemFreeShared(int device, void* dptr) {
  if (!dptr) return mccsInvalidArgument;
  DeviceGuard g(device);
  MCCS_HIP(hipFree(dptr));
  return mccsSuccess;
}

extern "C" mccsResult_t mccsMemOpenShared(int device, const void* handle, void** dptr) {
  if (!handle || !dptr) return mccsInvalidArgument;
  DeviceGuard g(device);
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  MCCS_HIP(hipIpcOpenMemHandle(dptr, h, hipIpcMemLazyEnablePeerAccess));
  return mccsSuccess;
}

extern "C" mccsResult_t mccsMemCloseShared(int device, void* dptr) {
  if (!dptr) return mccsInvalidArgument;
  DeviceGuard g(device);
  MCCS_HIP(hipIpcCloseMemHandle(dptr));
  return mccsSuccess;
}

extern "C" mccsResult_t mccsEventCreateShared(int device, void** event, void* handle_out) {
  if (!event || !handle_out) return mccsInvalidArgument;
  DeviceGuard g(device);
  hipEvent_t e = nullptr;
  MCCS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventInterprocess));
  hipIpcEventHandle_t h;
  if (hipIpcGetEventHandle(&h, e) != hipSuccess) {
    (void)hipEventDestroy(e);
    return mccsUnhandledCudaError;
  }
  std::memcpy(handle_out, &h, sizeof(h));
  *event = e;
  return mccsSuccess;
}

extern "C" mccsResult_t mccsEventOpenShared(int device, const void* handle, void** event) {
  if (!handle || !event) return mccsInvalidArgument;
  DeviceGuard g(device);
  hipIpcEventHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  hipEvent_t e = nullptr;
  MCCS_HIP(hipIpcOpenEventHandle(&e, h));
  *event = e;
  return mccsSuccess;
}

extern "C" mccsResult_t mccsEventDestroyShared(void* event) {
  if (!event) return mccsInvalidArgument;
  MCCS_HIP(hipEventDestroy((hipEvent_t)event));
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommEventHandle(mccsComm_t comm, void* handle_out) {
  Comm* c = (Comm*)comm;
  if (!c || !handle_out) return mccsInvalidArgument;
  DeviceGuard g(c->device);
  MCCS_CHECK(comm_make_event_ipc(c));
  hipIpcEventHandle_t h;
  MCCS_HIP(hipIpcGetEventHandle(&h, c->event));
  std::memcpy(handle_out, &h, sizeof(h));
  return mccsSuccess;
}

extern "C" mccsResult_t mccsCommStream(mccsComm_t comm, hipStream_t* stream) {
  Comm* c = (Comm*)comm;
  if (!c || !stream) return mccsInvalidArgument;
  return comm_stream(c, stream);
}

extern "C" mccsResult_t mccsCommWaitEvent(mccsComm_t comm, void* event) {
  Comm* c = (Comm*)comm;
  if (!c || !event) return mccsInvalidArgument;
  DeviceGuard g(c->device);
  hipStream_t st = nullptr;
  MCCS_CHECK(comm_stream(c, &st));
  MCCS_HIP(hipStreamWaitEvent(st, (hipEvent_t)event, 0));
  return mccsSuccess;
}

// The two stream-order calls of libmccs's bridge (collectives.rs:86,134), so
// an application needs no HIP bindings of its own.
extern "C" mccsResult_t mccsEventRecordShared(void* event, hipStream_t stream) {
  if (!event) return mccsInvalidArgument;
  MCCS_HIP(hipEventRecord((hipEvent_t)event, stream));
  return mccsSuccess;
}

extern "C" mccsResult_t mccsStreamWaitShared(hipStream_t stream, void* event) {
  if (!event) return mccsInvalidArgument;
  MCCS_HIP(hipStreamWaitEvent(stream, (hipEvent_t)event, 0));
  return mccsSuccess;
}

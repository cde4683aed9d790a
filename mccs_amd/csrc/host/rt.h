// rt.h — the device-runtime seam of the host path (internal).
//
// Every HIP call the communicator lifecycle makes on the single-process path
// (mccsCommInitAll -> group launch -> mccsCommSync -> destroy) goes through
// rt(): the HIP runtime in production, or a recording fake with N pretend
// devices (host memory, no kernels run) that CPU tests install with
// mccs_test_fake_runtime() to check how launches are issued across devices
// (tests/test_multidevice_launch.py).  Per-rank setup and connect (one rank
// per process) go through it too, so the fake can fail any one of their calls
// (mccs_test_fake_fail, tests/test_setup_diag.py).  The shared-memory service
// path calls HIP directly: it needs a real GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace mccs {

class DeviceRuntime {
 public:
  virtual ~DeviceRuntime() = default;
  virtual hipError_t GetDeviceCount(int* n) = 0;
  virtual hipError_t GetDevice(int* d) = 0;
  virtual hipError_t SetDevice(int d) = 0;
  virtual hipError_t Malloc(void** p, size_t bytes) = 0;
  virtual hipError_t MallocUncached(void** p, size_t bytes) = 0;
  virtual bool IsUncached(void* p) = 0;  // the runtime reports hipDeviceMallocUncached
  virtual hipError_t Free(void* p) = 0;
  virtual hipError_t Memset(void* p, int v, size_t bytes) = 0;
  virtual hipError_t Memcpy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind) = 0;
  virtual hipError_t HostMallocMapped(void** p, size_t bytes) = 0;
  virtual hipError_t HostGetDevicePointer(void** d, void* h) = 0;
  virtual hipError_t HostFree(void* p) = 0;
  virtual hipError_t DeviceSynchronize() = 0;
  virtual hipError_t FlushCaches() = 0;  // ring_flush_caches on the null stream of the current device
  virtual hipError_t CanAccessPeer(int* can, int dev, int peer) = 0;
  virtual hipError_t EnablePeerAccess(int peer) = 0;  // from the current device; already-enabled is success
  // Whether `dev` can perform atomics on `peer`'s memory (same device: yes).
  virtual hipError_t P2PAtomics(int* ok, int dev, int peer) = 0;
  virtual hipError_t EventCreate(hipEvent_t* e, unsigned flags) = 0;
  virtual hipError_t EventDestroy(hipEvent_t e) = 0;
  virtual hipError_t EventRecord(hipEvent_t e, hipStream_t s) = 0;
  virtual hipError_t EventSynchronize(hipEvent_t e) = 0;
  virtual hipError_t EventQuery(hipEvent_t e) = 0;
  virtual hipError_t StreamCreate(hipStream_t* s) = 0;  // non-blocking
  virtual hipError_t StreamDestroy(hipStream_t s) = 0;
  virtual hipError_t StreamSynchronize(hipStream_t s) = 0;
  virtual hipError_t StreamWaitEvent(hipStream_t s, hipEvent_t e) = 0;
  // A stream's process-unique id: HIP hands a destroyed stream's address to
  // the next stream it creates (tools/stream_id_probe.c), so the address does
  // not tell two streams apart; the id does.
  virtual hipError_t StreamId(hipStream_t s, unsigned long long* id) = 0;
  virtual hipError_t StreamIsCapturing(hipStream_t s, bool* capturing) = 0;
  // The graph a capturing stream records into, and a host callback run once
  // that graph and every executable graph instantiated from it are destroyed
  // (a HIP user object the graph retains; the callback may run on a runtime
  // thread and must make no HIP call).
  virtual hipError_t CaptureGraph(hipStream_t s, hipGraph_t* g) = 0;
  virtual hipError_t GraphOnDestroy(hipGraph_t g, void (*fn)(void*), void* arg) = 0;
  virtual hipError_t LaunchKernel(const void* fn, dim3 grid, dim3 block, void** args, hipStream_t s) = 0;
  // The same launch with `stop` recorded by the dispatch's own completion
  // signal (hipExtLaunchKernel): no marker packet behind the kernel.
  virtual hipError_t LaunchKernelExt(const void* fn, dim3 grid, dim3 block, void** args, hipStream_t s,
                                     hipEvent_t stop) = 0;
  virtual hipError_t BlocksPerCu(int* per_cu, const void* fn, int block) = 0;
  virtual hipError_t CuCount(int* ncu, int device) = 0;
  // one rank per process (mccsCommSetupRank / mccsCommConnect)
  virtual hipError_t IpcGetMemHandle(hipIpcMemHandle_t* h, void* p) = 0;
  virtual hipError_t IpcOpenMemHandle(void** p, hipIpcMemHandle_t h) = 0;  // lazy peer access
  virtual hipError_t IpcCloseMemHandle(void* p) = 0;
  virtual hipError_t DeviceGetPCIBusId(char* id, int len, int device) = 0;
  virtual hipError_t DeviceGetByPCIBusId(int* device, const char* id) = 0;
  // True only when process `pid` (of this host and pid namespace) has exited
  // and been reaped: its GPU queues are gone, so none of its kernels can still
  // write a peer's FIFO arena (the arena pool stops waiting for its release).
  virtual bool ProcessGone(int pid) = 0;
};

DeviceRuntime& rt();
// Installs a recording fake with `ndevices` devices (0 restores HIP).
void rt_use_fake(int ndevices);
// Identity of the current runtime: 0 for HIP, a fresh nonzero id per
// installed fake.  Memory pooled under one runtime is never handed out under
// another; a removed fake's pooled arenas are dropped (its memory died with it).
unsigned rt_generation();
bool rt_stream_ids_native();  // the HIP runtime tells streams apart by hipStreamGetId (else by address)

}  // namespace mccs

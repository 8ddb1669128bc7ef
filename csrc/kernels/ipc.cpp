// HIP IPC buffers for the parameter-server data plane (parallel/ps_device.py).
//
// A parameter-server task allocates its variable shard and the workers' gradient mailboxes with
// hipMalloc (its own allocations, never torch's caching allocator, so one handle maps exactly one
// buffer at offset 0), exports them with hipIpcGetMemHandle, and the workers map them with
// hipIpcOpenMemHandle: on an 8-GPU node that is a peer mapping over xGMI (the copy engines and
// kernels of the worker's GPU read/write the owner's HBM directly), on one GPU a second mapping
// of the same HBM.  The buffers are handed to torch as DLPack capsules whose deleter unmaps /
// frees them, so their lifetime is the tensor's.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace {
void ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    ok(hipGetDevice(&prev), "hipGetDevice");
    if (dev != prev) ok(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};
}  // namespace

uintptr_t dtf_ipc_alloc(size_t bytes, int device) {
  DeviceGuard g(device);
  void* p = nullptr;
  ok(hipMalloc(&p, bytes ? bytes : 256), "hipMalloc");
  ok(hipMemset(p, 0, bytes ? bytes : 256), "hipMemset");
  ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return reinterpret_cast<uintptr_t>(p);
}

std::string dtf_ipc_handle(uintptr_t ptr, int device) {
  DeviceGuard g(device);
  hipIpcMemHandle_t h;
  ok(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

uintptr_t dtf_ipc_open(const std::string& handle, int device) {
  if (handle.size() != sizeof(hipIpcMemHandle_t))
    throw std::invalid_argument("ipc_open: handle has the wrong size");
  DeviceGuard g(device);
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  void* p = nullptr;
  ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return reinterpret_cast<uintptr_t>(p);
}

void dtf_ipc_close(uintptr_t ptr, int device) {
  DeviceGuard g(device);
  (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr));
}

void dtf_ipc_free(uintptr_t ptr, int device) {
  DeviceGuard g(device);
  (void)hipDeviceSynchronize();
  (void)hipFree(reinterpret_cast<void*>(ptr));
}

// Native RCCL communicator (SURVEY.md §5.8 "data plane: a C++ wrapper over rccl.h").
//
// One process per GPU; the communicator is created with ncclCommInitRank from a unique id the
// Python side exchanges through the cluster's TCPStore.  Every collective is enqueued on the
// HIP stream the caller passes (the strategy's dedicated comm stream, ordered against the
// compute stream with hipEvents by the caller) -- no c10d work objects, no watchdog thread.
//
// RCCL is bound at run time with dlopen/dlsym: the process already has torch's librccl.so.1
// (its ProcessGroupNCCL links it), and a second copy of the library in one process would be two
// independent transports on the same GPUs.  `dtf_rccl_load(path)` opens the library torch
// ships (RTLD_NOLOAD first: the already-mapped copy) and resolves the entry points below; the
// types come from the system rccl.h (the API and ncclUniqueId layout are stable across
// 2.26 / 2.27).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace {

struct RcclApi {
  void* lib = nullptr;
  ncclResult_t (*GetVersion)(int*) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t,
                                ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int,
                         ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
};

RcclApi g_api;

template <typename F>
void bind(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g_api.lib, name));
  if (!f) throw std::runtime_error(std::string("rccl: symbol ") + name + " not found");
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("rccl ") + what + ": " +
                             (g_api.GetErrorString ? g_api.GetErrorString(r) : "error") +
                             " (" + std::to_string((int)r) + ")");
}

void need() {
  if (!g_api.lib) throw std::runtime_error("rccl: call rccl_load(path) first");
}

}  // namespace

int dtf_rccl_load(const std::string& path) {
  if (g_api.lib) {
    int v = 0;
    g_api.GetVersion(&v);
    return v;
  }
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);     // torch's copy, already mapped
  if (!h) h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!h) throw std::runtime_error(std::string("rccl: dlopen ") + path + ": " + dlerror());
  g_api.lib = h;
  bind(g_api.GetVersion, "ncclGetVersion");
  bind(g_api.GetErrorString, "ncclGetErrorString");
  bind(g_api.GetUniqueId, "ncclGetUniqueId");
  bind(g_api.CommInitRank, "ncclCommInitRank");
  bind(g_api.CommDestroy, "ncclCommDestroy");
  bind(g_api.CommAbort, "ncclCommAbort");
  bind(g_api.CommGetAsyncError, "ncclCommGetAsyncError");
  bind(g_api.AllReduce, "ncclAllReduce");
  bind(g_api.ReduceScatter, "ncclReduceScatter");
  bind(g_api.AllGather, "ncclAllGather");
  bind(g_api.Broadcast, "ncclBroadcast");
  bind(g_api.Reduce, "ncclReduce");
  bind(g_api.GroupStart, "ncclGroupStart");
  bind(g_api.GroupEnd, "ncclGroupEnd");
  int v = 0;
  check(g_api.GetVersion(&v), "GetVersion");
  return v;
}

std::string dtf_rccl_unique_id() {
  need();
  ncclUniqueId id;
  check(g_api.GetUniqueId(&id), "GetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

// opaque handle (the ncclComm_t pointer) as an integer for the Python wrapper
long dtf_rccl_comm_init(const std::string& uid, int nranks, int rank, int device) {
  need();
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("rccl: bad unique id size");
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl: hipSetDevice failed");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  check(g_api.CommInitRank(&comm, nranks, id, rank), "CommInitRank");
  return reinterpret_cast<long>(comm);
}

void dtf_rccl_comm_destroy(long comm, int abort) {
  need();
  auto c = reinterpret_cast<ncclComm_t>(comm);
  check(abort ? g_api.CommAbort(c) : g_api.CommDestroy(c), abort ? "CommAbort" : "CommDestroy");
}

int dtf_rccl_async_error(long comm) {
  need();
  ncclResult_t r = ncclSuccess;
  check(g_api.CommGetAsyncError(reinterpret_cast<ncclComm_t>(comm), &r), "CommGetAsyncError");
  return (int)r;
}

void dtf_rccl_all_reduce(long comm, long send, long recv, long count, int dtype, int op,
                         long stream) {
  need();
  check(g_api.AllReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                        (size_t)count, (ncclDataType_t)dtype, (ncclRedOp_t)op,
                        reinterpret_cast<ncclComm_t>(comm), reinterpret_cast<hipStream_t>(stream)),
        "AllReduce");
}

void dtf_rccl_reduce_scatter(long comm, long send, long recv, long recvcount, int dtype, int op,
                             long stream) {
  need();
  check(g_api.ReduceScatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                            (size_t)recvcount, (ncclDataType_t)dtype, (ncclRedOp_t)op,
                            reinterpret_cast<ncclComm_t>(comm),
                            reinterpret_cast<hipStream_t>(stream)),
        "ReduceScatter");
}

void dtf_rccl_all_gather(long comm, long send, long recv, long sendcount, int dtype,
                         long stream) {
  need();
  check(g_api.AllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                        (size_t)sendcount, (ncclDataType_t)dtype,
                        reinterpret_cast<ncclComm_t>(comm), reinterpret_cast<hipStream_t>(stream)),
        "AllGather");
}

void dtf_rccl_broadcast(long comm, long send, long recv, long count, int dtype, int root,
                        long stream) {
  need();
  check(g_api.Broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                        (size_t)count, (ncclDataType_t)dtype, root,
                        reinterpret_cast<ncclComm_t>(comm), reinterpret_cast<hipStream_t>(stream)),
        "Broadcast");
}

void dtf_rccl_reduce(long comm, long send, long recv, long count, int dtype, int op, int root,
                     long stream) {
  need();
  check(g_api.Reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                     (size_t)count, (ncclDataType_t)dtype, (ncclRedOp_t)op, root,
                     reinterpret_cast<ncclComm_t>(comm), reinterpret_cast<hipStream_t>(stream)),
        "Reduce");
}

void dtf_rccl_group(int start) {
  need();
  check(start ? g_api.GroupStart() : g_api.GroupEnd(), start ? "GroupStart" : "GroupEnd");
}

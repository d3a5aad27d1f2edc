// Native RCCL communicator for the training hot path (host C++).
//
// Capability parity: the reference's MPI transport (mpi4py over MPI_COMM_WORLD,
// data_parallelism_train.py:10,60-62,118,135,210,227).  Here each rank owns an
// ncclComm_t created with ncclCommInitRank from a unique id exchanged through the
// rendezvous TCPStore (python side), and the per-step gradient all-reduce is an
// ncclAllReduce launched straight onto the engine's HIP stream - no per-collective
// framework objects, no extra stream hops, and it is captured into the step hipGraph
// as a plain kernel node.  ncclCommAbort + a fresh ncclCommInitRank re-form the group
// after a rank drop (torch's bundled RCCL 2.26 has no ncclCommShrink).
//
// RCCL is resolved at run time with dlopen/dlsym from the SAME librccl.so that torch
// already loaded (path passed from python), so exactly one RCCL lives in the process.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace dnn {

namespace {
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*GetVersion)(int*) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
RcclApi g;

template <typename F>
void sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g.h, name));
  if (!f) throw std::runtime_error(std::string("RCCL symbol not found: ") + name);
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const char* s = g.GetErrorString ? g.GetErrorString(r) : "?";
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + s);
  }
}

void need() {
  if (!g.h) throw std::runtime_error("RCCL not opened: call rccl_open(path) first");
}
}  // namespace

int rccl_open(const std::string& path) {
  if (g.h) return 0;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) throw std::runtime_error(std::string("dlopen failed: ") + dlerror());
  g.h = h;
  sym(g.GetUniqueId, "ncclGetUniqueId");
  sym(g.CommInitRank, "ncclCommInitRank");
  sym(g.AllReduce, "ncclAllReduce");
  sym(g.Broadcast, "ncclBroadcast");
  sym(g.CommAbort, "ncclCommAbort");
  sym(g.CommDestroy, "ncclCommDestroy");
  sym(g.CommGetAsyncError, "ncclCommGetAsyncError");
  sym(g.GetVersion, "ncclGetVersion");
  sym(g.GetErrorString, "ncclGetErrorString");
  int v = 0;
  g.GetVersion(&v);
  return v;
}

std::string rccl_unique_id() {
  need();
  ncclUniqueId id;
  check(g.GetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

uintptr_t rccl_init(const std::string& id_bytes, int nranks, int rank, int device) {
  need();
  if (id_bytes.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad ncclUniqueId size");
  ncclUniqueId id;
  std::memcpy(id.internal, id_bytes.data(), NCCL_UNIQUE_ID_BYTES);
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  ncclComm_t c = nullptr;
  check(g.CommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
  return reinterpret_cast<uintptr_t>(c);
}

// dtype: 0 = fp32, 1 = bf16;  op: 0 = sum, 1 = avg, 2 = max
void rccl_allreduce(uintptr_t comm, uintptr_t buf, size_t count, int dtype, int op, uintptr_t stream) {
  need();
  const ncclDataType_t dt = dtype == 1 ? ncclBfloat16 : ncclFloat32;
  const ncclRedOp_t ro = op == 1 ? ncclAvg : (op == 2 ? ncclMax : ncclSum);
  void* p = reinterpret_cast<void*>(buf);
  check(g.AllReduce(p, p, count, dt, ro, reinterpret_cast<ncclComm_t>(comm), reinterpret_cast<hipStream_t>(stream)),
        "ncclAllReduce");
}

void rccl_broadcast(uintptr_t comm, uintptr_t buf, size_t count, int root, uintptr_t stream) {
  need();
  void* p = reinterpret_cast<void*>(buf);
  check(g.Broadcast(p, p, count, ncclFloat32, root, reinterpret_cast<ncclComm_t>(comm),
                    reinterpret_cast<hipStream_t>(stream)),
        "ncclBroadcast");
}

int rccl_async_error(uintptr_t comm) {
  need();
  ncclResult_t r = ncclSuccess;
  g.CommGetAsyncError(reinterpret_cast<ncclComm_t>(comm), &r);
  return static_cast<int>(r);
}

void rccl_abort(uintptr_t comm) {
  need();
  if (comm) g.CommAbort(reinterpret_cast<ncclComm_t>(comm));
}

void rccl_destroy(uintptr_t comm) {
  need();
  if (comm) g.CommDestroy(reinterpret_cast<ncclComm_t>(comm));
}

}  // namespace dnn

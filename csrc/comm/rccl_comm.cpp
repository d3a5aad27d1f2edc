// Native RCCL communicator for the training hot path (host C++).
//
// Capability parity: the reference's MPI transport (mpi4py over MPI_COMM_WORLD,
// data_parallelism_train.py:10,60-62,118,135,210,227).  Here each rank owns an
// ncclComm_t created with ncclCommInitRank from a unique id exchanged through the
// rendezvous TCPStore (python side), and the per-step gradient all-reduce is an
// ncclAllReduce launched straight onto the engine's HIP stream - no per-collective
// framework objects, no extra stream hops, and it is captured into the step hipGraph
// as a plain kernel node.  ncclCommAbort + a fresh communicator re-form the group after a rank
// drop.  (ncclCommShrink is not used: torch's bundled RCCL 2.26 does not export it, and the
// recovery path must ncclCommAbort first anyway - that is what releases RCCL kernels spinning
// on the dead peer - and an aborted communicator cannot be shrunk.)
//
// Communicators are created NON-BLOCKING (ncclCommInitRankConfig, config.blocking = 0) and
// the init is polled through ncclCommGetAsyncError with a deadline: a peer that dies during
// the (re-)init turns into an error after the timeout instead of a hang inside RCCL.  A
// collective that returns ncclInProgress (non-blocking enqueue) is polled to completion of
// its enqueue the same way.
//
// RCCL is resolved at run time with dlopen/dlsym from the SAME librccl.so that torch
// already loaded (path passed from python), so exactly one RCCL lives in the process.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace dnn {

namespace {
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
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
  sym(g.CommInitRankConfig, "ncclCommInitRankConfig");
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

// Poll a non-blocking communicator until its pending operation left ncclInProgress, at most
// timeout_s seconds.  Returns the final state (ncclInProgress: timed out).
ncclResult_t wait_ready(ncclComm_t c, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  ncclResult_t st = ncclInProgress;
  while (true) {
    if (g.CommGetAsyncError(c, &st) != ncclSuccess) return ncclInternalError;
    if (st != ncclInProgress) return st;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return st;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// blocking = 0: ncclCommInitRankConfig in non-blocking mode, polled with a deadline (the
// default); 1: plain ncclCommInitRank (no deadline).
uintptr_t rccl_init(const std::string& id_bytes, int nranks, int rank, int device, int blocking, double timeout_s) {
  need();
  if (id_bytes.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad ncclUniqueId size");
  ncclUniqueId id;
  std::memcpy(id.internal, id_bytes.data(), NCCL_UNIQUE_ID_BYTES);
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  ncclComm_t c = nullptr;
  if (blocking) {
    check(g.CommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
    return reinterpret_cast<uintptr_t>(c);
  }
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  const ncclResult_t r = g.CommInitRankConfig(&c, nranks, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) check(r, "ncclCommInitRankConfig");
  const ncclResult_t st = wait_ready(c, timeout_s);
  if (st != ncclSuccess) {
    g.CommAbort(c);
    if (st == ncclInProgress)
      throw std::runtime_error("ncclCommInitRankConfig timed out after " + std::to_string(timeout_s) +
                               " s (a peer never joined)");
    check(st, "ncclCommInitRankConfig (async)");
  }
  return reinterpret_cast<uintptr_t>(c);
}

// a collective's return code on a non-blocking communicator: ncclInProgress = still being
// enqueued; wait (bounded) until the enqueue finished before anything else touches the comm
void check_enqueue(ncclComm_t c, ncclResult_t r, const char* what) {
  if (r == ncclInProgress) r = wait_ready(c, 60.0);
  if (r == ncclInProgress) throw std::runtime_error(std::string("RCCL ") + what + ": enqueue timed out");
  check(r, what);
}

// dtype: 0 = fp32, 1 = bf16;  op: 0 = sum, 1 = avg, 2 = max
void rccl_allreduce(uintptr_t comm, uintptr_t buf, size_t count, int dtype, int op, uintptr_t stream) {
  need();
  const ncclDataType_t dt = dtype == 1 ? ncclBfloat16 : ncclFloat32;
  const ncclRedOp_t ro = op == 1 ? ncclAvg : (op == 2 ? ncclMax : ncclSum);
  void* p = reinterpret_cast<void*>(buf);
  ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
  check_enqueue(c, g.AllReduce(p, p, count, dt, ro, c, reinterpret_cast<hipStream_t>(stream)), "ncclAllReduce");
}

void rccl_broadcast(uintptr_t comm, uintptr_t buf, size_t count, int root, uintptr_t stream) {
  need();
  void* p = reinterpret_cast<void*>(buf);
  ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
  check_enqueue(c, g.Broadcast(p, p, count, ncclFloat32, root, c, reinterpret_cast<hipStream_t>(stream)),
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

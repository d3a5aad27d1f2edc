// One-shot gradient all-reduce over xGMI peer mappings, fused with momentum SGD (gfx950).
//
// Capability parity: the reference averages models through rank 0 with pickled mpi4py
// sends (data_parallelism_train.py:118,210,227,238-240); the per-step gradient
// all-reduce is its future work (Project_Report.pdf p.4 §6.2).  The step-allreduce
// policy's collective is tiny (62,006 fp32 = 248 KB) and therefore LATENCY-bound: a ring
// (RCCL) pays 2 (N-1) dependent hops over single xGMI links.  An 8x MI355X node is a full
// xGMI mesh (7 links per GPU), so this kernel does it in ONE hop instead:
//
//   1. publish - every workgroup copies its 1024-element slice of the local gradient into
//      this rank's shared region (double-buffered by step parity), then pushes a step
//      flag into EVERY peer's region (remote stores over xGMI; the peer polls locally);
//   2. wait    - lanes 0..N-1 poll the N flags of this slice in local memory;
//   3. reduce  - the workgroup reads the slice from all N regions (7 xGMI links in
//      parallel), sums them in RANK ORDER (so every replica computes bit-identical
//      values - no float atomics, deterministic run to run), scales by 1/N and applies
//      the momentum-SGD update + the bf16 weight-image refresh (the work sgd_apply does
//      after an RCCL all-reduce), or writes the averaged gradient (plain all-reduce).
//
// Regions come from hipExtMallocWithFlags(hipDeviceMallocUncached) and are shared with
// hipIpcGetMemHandle / hipIpcOpenMemHandle (dmabuf IPC); every access to shared bytes is
// a system-scope atomic (sc0 sc1), ordered by system-scope release/acquire fences around
// the flag hand-off.  Double buffering makes one flag per slice and step enough: a rank
// overwrites slot (s & 1) at step s + 2 only after every peer published step s + 1, which
// each does only after finishing its step s reads.
//
// Never hangs: a wait that exceeds the timeout (or sees the host abort word set - the
// fault watchdog sets it when a peer dies) sets a sticky error word and the kernel
// completes; later launches skip the wait.  The host checks the word at epoch end.
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "../kernels/common.h"
#include "xgmi_layout.h"

namespace dnn {

constexpr int XG_THREADS = 256;
constexpr int XG_PER_THREAD = XG_CHUNK / XG_THREADS;  // 4

struct XgmiArgs {
  unsigned char* region[XG_MAX_RANKS];  // every rank's shared region, mapped here (own included)
  int rank, nranks;
  int n;                 // elements to reduce
  int max_blocks;        // flag rows per writer (capacity / XG_CHUNK)
  long long slot_bytes;  // bytes per parity slot
  long long flag_bytes;  // bytes of the flag area at the start of a region
  const float* grad;     // local input
  float* out;            // mode 0: averaged gradient (may alias grad)
  float* master;
  float* mom;
  bf16* shadow;
  float lr, momentum, scale;
  int mode;                 // 0: all-reduce (avg) -> out; 1: + momentum SGD + bf16 shadow; 2: + SGD (no shadow)
  unsigned* ctr;            // local: [max_blocks] per-workgroup step counters, [max_blocks] error word
  const unsigned* abort_w;  // host-mapped abort word (fault watchdog)
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
  int fences;               // bit 0: system release before the flag push, bit 1: system acquire after the wait
  int prepub;               // 1: the previous kernel (grad_reduce) already stored this step's gradients in
                            //    the own slot (system-coherent): no publish copy, flags go out at once
};

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(XG_THREADS) xgmi_allreduce_kernel(XgmiArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  unsigned* err_w = a.ctr + a.max_blocks;
  const unsigned step = a.ctr[b] + 1u;
  const bool failed = a.ctr[a.max_blocks] != 0u;
  const int par = step & 1u;
  const int lo = b * XG_CHUNK;
  auto slot = [&](int r) {
    return reinterpret_cast<unsigned*>(a.region[r] + a.flag_bytes + par * a.slot_bytes);
  };

  // 1. publish this slice (system-coherent stores), then release + push the step flag
  // (the optimizer state is local and only this thread touches it: prefetch it now, so the
  //  update after the wait costs no extra memory latency)
  const unsigned* g = reinterpret_cast<const unsigned*>(a.grad);
  unsigned mine[XG_PER_THREAD];
  float p_old[XG_PER_THREAD], m_old[XG_PER_THREAD];
  unsigned* my_slot = slot(a.rank);
#pragma unroll
  for (int k = 0; k < XG_PER_THREAD; ++k) {
    const int e = min(lo + k * XG_THREADS + tid, a.n - 1);
    mine[k] = a.prepub ? ld_sys(my_slot + e) : g[e];
    if (a.mode != 0) {
      p_old[k] = a.master[e];
      m_old[k] = a.mom[e];
    }
  }
  if (!a.prepub) {
#pragma unroll
    for (int k = 0; k < XG_PER_THREAD; ++k) {
      const int e = lo + k * XG_THREADS + tid;
      if (e < a.n) st_sys(my_slot + e, mine[k]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (tid < 64) {
    if (a.fences & 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    if (tid < a.nranks && tid != a.rank) {  // (own data stays in registers: no own flag)
      unsigned* flags = reinterpret_cast<unsigned*>(a.region[tid]);
      st_sys(flags + a.rank * a.max_blocks + b, step);
    }
  }

  // 2. wait for the N flags of this slice (bounded)
  if (tid < a.nranks && tid != a.rank && !failed) {
    const unsigned* f = reinterpret_cast<const unsigned*>(a.region[a.rank]) + tid * a.max_blocks + b;
    const long long t0 = wall_clock64();
    int spins = 0;
    while ((int)(ld_sys(f) - step) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 255) == 0) {
        if (wall_clock64() - t0 > a.timeout_ticks || ld_sys(a.abort_w) != 0u) {
          st_sys(err_w, 1u);
          break;
        }
      }
    }
  }
  if (tid < 64 && (a.fences & 2)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // 3. gather all ranks' slices (every load in flight before the first use), sum in rank order
  float v[XG_MAX_RANKS][XG_PER_THREAD];
#pragma unroll
  for (int r = 0; r < XG_MAX_RANKS; ++r) {
    if (r < a.nranks) {
      const unsigned* src = slot(r);
#pragma unroll
      for (int k = 0; k < XG_PER_THREAD; ++k) {
        const int e = min(lo + k * XG_THREADS + tid, a.n - 1);
        v[r][k] = __uint_as_float(r == a.rank ? mine[k] : ld_sys(src + e));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < XG_PER_THREAD; ++k) {
    const int e = lo + k * XG_THREADS + tid;
    if (e >= a.n) continue;
    float s = v[0][k];
#pragma unroll
    for (int r = 1; r < XG_MAX_RANKS; ++r)
      if (r < a.nranks) s += v[r][k];
    const float gr = s * a.scale;
    if (a.mode == 0) {
      a.out[e] = gr;
    } else {
      float p, m;
      sgd_update(gr, p_old[k], m_old[k], a.lr, a.momentum, p, m);
      a.mom[e] = m;
      a.master[e] = p;
      if (a.mode == 1) write_shadow(a.shadow, e, p);
    }
  }
  __syncthreads();
  if (tid == 0) a.ctr[b] = step;
}

// ---- host side ------------------------------------------------------------------------
namespace {
void xcheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

// Allocates this rank's shared region (zeroed) and returns (device pointer, IPC handle
// bytes, memory kind).  Uncached (fine-grained) memory first; plain device memory if the
// driver refuses to export that kind.
std::tuple<uintptr_t, std::string, std::string> xgmi_alloc(long long capacity) {
  const long long bytes = xgmi_region_bytes(capacity);
  void* p = nullptr;
  std::string kind = "uncached";
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    kind = "device";
    xcheck(hipMalloc(&p, bytes), "hipMalloc(xgmi region)");
  }
  xcheck(hipMemset(p, 0, bytes), "hipMemset(xgmi region)");
  xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess && kind == "uncached") {
    (void)hipGetLastError();
    xcheck(hipFree(p), "hipFree");
    kind = "device";
    xcheck(hipMalloc(&p, bytes), "hipMalloc(xgmi region)");
    xcheck(hipMemset(p, 0, bytes), "hipMemset(xgmi region)");
    xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
    e = hipIpcGetMemHandle(&h, p);
  }
  xcheck(e, "hipIpcGetMemHandle");
  return {reinterpret_cast<uintptr_t>(p), std::string(h.reserved, HIP_IPC_HANDLE_SIZE), kind};
}

// zero both data slots (keeps the flags): elements a pre-published step never writes (arena
// padding) must read as 0 after the self-test filled the slots
void xgmi_clear_slots(uintptr_t region, long long capacity) {
  xcheck(hipMemset(reinterpret_cast<unsigned char*>(region) + xgmi_flag_bytes(capacity), 0,
                   2 * xgmi_slot_bytes(capacity)), "hipMemset(xgmi slots)");
  xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

uintptr_t xgmi_open(const std::string& handle) {
  if (handle.size() != HIP_IPC_HANDLE_SIZE) throw std::runtime_error("bad IPC handle size");
  hipIpcMemHandle_t h;
  std::memcpy(h.reserved, handle.data(), HIP_IPC_HANDLE_SIZE);
  void* p = nullptr;
  xcheck(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return reinterpret_cast<uintptr_t>(p);
}

// physical identity of the current device ("domain:bus:device.function"): ranks that share
// one GPU (single-GPU rehearsals) and ranks on distinct GPUs need different fence defaults
std::string xgmi_device_id() {
  int dev = 0;
  xcheck(hipGetDevice(&dev), "hipGetDevice");
  char buf[64] = {0};
  xcheck(hipDeviceGetPCIBusId(buf, sizeof(buf) - 1, dev), "hipDeviceGetPCIBusId");
  return std::string(buf);
}

void xgmi_close(uintptr_t p) {
  if (p) (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(p));
}

void xgmi_free(uintptr_t p) {
  if (p) (void)hipFree(reinterpret_cast<void*>(p));
}

// host-mapped abort word: (host pointer, device pointer)
std::pair<uintptr_t, uintptr_t> xgmi_abort_word() {
  void* h = nullptr;
  xcheck(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc(abort word)");
  std::memset(h, 0, 64);
  void* d = nullptr;
  xcheck(hipHostGetDevicePointer(&d, h, 0), "hipHostGetDevicePointer");
  return {reinterpret_cast<uintptr_t>(h), reinterpret_cast<uintptr_t>(d)};
}

void xgmi_set_abort(uintptr_t host_word, unsigned v) {
  __atomic_store_n(reinterpret_cast<unsigned*>(host_word), v, __ATOMIC_SEQ_CST);
}

void xgmi_free_abort_word(uintptr_t host_word) {
  if (host_word) (void)hipHostFree(reinterpret_cast<void*>(host_word));
}

void launch_xgmi_allreduce(const std::vector<uintptr_t>& regions, int rank, long long capacity, int n,
                           const float* grad, float* out, float* master, float* mom, bf16* shadow, float lr,
                           float momentum, float scale, int mode, unsigned* ctr, const unsigned* abort_w,
                           double timeout_s, int fences, int prepub, hipStream_t stream) {
  const int nranks = (int)regions.size();
  if (nranks < 1 || nranks > XG_MAX_RANKS) throw std::runtime_error("xgmi all-reduce: 1..8 ranks");
  if (rank < 0 || rank >= nranks) throw std::runtime_error("xgmi all-reduce: bad rank");
  if (n <= 0 || n > capacity) throw std::runtime_error("xgmi all-reduce: n exceeds the region capacity");
  if (mode < 0 || mode > 2) throw std::runtime_error("xgmi all-reduce: bad mode");
  if (mode == 1 && n > ARENA) throw std::runtime_error("xgmi all-reduce: shadow mode is for the fused arena");
  XgmiArgs a{};
  for (int r = 0; r < nranks; ++r) a.region[r] = reinterpret_cast<unsigned char*>(regions[r]);
  a.rank = rank;
  a.nranks = nranks;
  a.n = n;
  a.max_blocks = xgmi_max_blocks(capacity);
  a.slot_bytes = xgmi_slot_bytes(capacity);
  a.flag_bytes = xgmi_flag_bytes(capacity);
  a.grad = grad;
  a.out = out;
  a.master = master;
  a.mom = mom;
  a.shadow = shadow;
  a.lr = lr;
  a.momentum = momentum;
  a.scale = scale;
  a.mode = mode;
  a.ctr = ctr;
  a.abort_w = abort_w;
  a.timeout_ticks = (long long)(timeout_s * 1.0e8);
  a.fences = fences;
  a.prepub = prepub;
  const int nblk = (n + XG_CHUNK - 1) / XG_CHUNK;
  hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(nblk), dim3(XG_THREADS), 0, stream, a);
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

// One-shot gradient all-reduce over xGMI peer mappings, fused with momentum SGD (gfx950).
//
// Capability parity: the reference averages models through rank 0 with pickled mpi4py
// sends (data_parallelism_train.py:118,210,227,238-240); the per-step gradient
// all-reduce is its future work (Project_Report.pdf p.4 §6.2).  The step-allreduce
// policy's collective is tiny (62,006 fp32 = 248 KB) and therefore LATENCY-bound: a ring
// (RCCL) pays 2 (N-1) dependent hops over single xGMI links.  An 8x MI355X node is a full
// xGMI mesh (7 links per GPU), so this kernel does it in ONE hop instead:
//
//   1. publish - every workgroup writes its 1024-element slice of the local gradient into
//      this rank's shared region as data-tagged granules: ONE 8-byte {fp32 value, step}
//      word per element (double-buffered by step parity);
//   2. gather  - every lane reads its elements' granules from all N regions (7 xGMI links
//      in parallel, every load in flight before the first check) until each tag shows the
//      current step: the value and its tag are one atomic word, so no flag, fence or barrier
//      has to order the hand-off - on one device and across GPUs alike;
//   3. reduce  - sums them in RANK ORDER (so every replica computes bit-identical values - no
//      float atomics, deterministic run to run), scales by 1/N and applies the momentum-SGD
//      update + the bf16 weight-image refresh (the work sgd_apply does after an RCCL
//      all-reduce), or writes the averaged gradient (plain all-reduce).
//
// Regions come from hipExtMallocWithFlags(hipDeviceMallocUncached) and are shared with
// hipIpcGetMemHandle / hipIpcOpenMemHandle (dmabuf IPC); every access to shared bytes is a
// system-scope 64-bit atomic (sc0 sc1).  Double buffering by parity makes the tags safe: a
// rank overwrites element e of slot (s & 1) at step s + 2 only after it read every peer's
// step s + 1 granule of e, which each peer wrote only after reading this rank's step s one.
// (The one-launch path - kernels/reduce_sgd.hip xp_exchange - is the same protocol run by
// the batch-reduction lanes on their own elements; this kernel is its two-launch fallback
// and the all-reduce of the generic layer engine.)
//
// Never hangs: a wait that exceeds the timeout (or sees the host abort word set - the
// fault watchdog sets it when a peer dies) sets a sticky error word and the kernel
// completes; later launches skip the wait.  The host checks the word at epoch end.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <tuple>
#include <map>
#include <mutex>

#include <cstring>
#include <stdexcept>
#include <string>

#include "../kernels/common.h"
#include "xgmi_layout.h"

namespace dnn {

constexpr int XG_THREADS = 256;
constexpr int XG_PER_THREAD = XG_CHUNK / XG_THREADS;  // 4

__device__ __forceinline__ unsigned long long ld_sys64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct XgmiArgs {
  unsigned char* region[XG_MAX_RANKS];  // every rank's shared region, mapped here (own included)
  int rank, nranks;
  int n;                 // elements to reduce
  long long gslot_bytes; // bytes per parity slot of granules
  const float* grad;     // local input
  float* out;            // mode 0: averaged gradient (may alias grad)
  float* master;
  float* mom;
  bf16* shadow;
  float lr, momentum, scale;
  int mode;                 // 0: all-reduce (avg) -> out; 1: + momentum SGD + bf16 shadow; 2: + SGD (no shadow)
  unsigned* ctr;            // local: [max_blocks] per-workgroup step counters, [max_blocks] error word
  int max_blocks;
  const unsigned* abort_w;  // host-mapped abort word (fault watchdog)
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
  int form;                 // 0 one-hop pull, 2 two-hop pull (reduce-scatter + all-gather); + 4: bf16 granules
  long long ag_off;         // all-gather slot offset in every region (xgmi_layout.h)
  unsigned long long* wait; // optional: per-step wait ring, as ReduceArgs::xp_wait
};

// The two-hop form shares its ag slot with grad_reduce's: this kernel's tags carry bit 31 of
// the step word, so a granule of one path never matches a wait of the other, and an owner
// overwrites its ag slot only after every peer contributed to the new exchange, i.e. finished
// reading the previous one.
constexpr unsigned XG_PATH_BIT = 0x80000000u;

template <int NR>
__device__ __forceinline__ long long xg_wait(const XgmiArgs& a, const unsigned long long* const (&src)[NR],
                                             unsigned pending, float (&v)[NR][XG_PER_THREAD],
                                             const int (&e)[XG_PER_THREAD], unsigned want, bool failed,
                                             unsigned* err_w) {
  const long long t0 = wall_clock64();
  while (pending != 0u) {
    unsigned long long x[NR][XG_PER_THREAD];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int k = 0; k < XG_PER_THREAD; ++k)
        if (pending & (1u << (4 * r + k))) x[r][k] = ld_sys64(src[r] + e[k]);
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int k = 0; k < XG_PER_THREAD; ++k)
        if ((pending & (1u << (4 * r + k))) && (unsigned)(x[r][k] >> 32) == want) {
          v[r][k] = __uint_as_float((unsigned)x[r][k]);
          pending &= ~(1u << (4 * r + k));
        }
    if (pending == 0u || failed) break;
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > a.timeout_ticks ||
        __hip_atomic_load(a.abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
      __hip_atomic_store(err_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
  return wall_clock64() - t0;
}

// per-wave max wait of this step into the ring (see ReduceArgs::xp_wait)
__device__ __forceinline__ void xg_record_wait(const XgmiArgs& a, unsigned step, long long ticks) {
  if (a.wait == nullptr) return;
  unsigned t = (unsigned)min(ticks, 0xffffffffll);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t = max(t, (unsigned)__shfl_xor((int)t, off));
  if ((threadIdx.x & 63) == 0)
    a.wait[((size_t)(step % XP_WAIT_RING) * XP_MAX_BLOCKS + blockIdx.x) * (XG_THREADS / 64) + (threadIdx.x >> 6)] =
        ((unsigned long long)step << 32) | t;
}

// bf16 granules (PK, form bit 4): a thread's elements k = (0, 1) and (2, 3) travel as ONE word
// {bf16 | bf16 << 16, step} at the index of the pair's first element, exactly as the one-launch
// exchange's pairs (kernels/reduce_sgd.hip pack_pairs): every rank sums the same bf16-rounded
// values in fp32, rank order; the two-hop owner all-gathers its sum as bf16 too.
template <bool PK>
__device__ __forceinline__ void xg_pack(float (&x)[XG_PER_THREAD], const bool (&ok)[XG_PER_THREAD],
                                        const int (&e)[XG_PER_THREAD], unsigned long long* dst,
                                        unsigned long long tag) {
#pragma unroll
  for (int k = 0; k < XG_PER_THREAD; k += 2) {
    if (!ok[k]) continue;
    const unsigned lo = bf16_bits(x[k]), hi = ok[k + 1] ? bf16_bits(x[k + 1]) : 0u;
    x[k] = bf16_lo(lo);
    x[k + 1] = bf16_lo(hi);
    if (dst != nullptr)
      __hip_atomic_store(dst + e[k], tag | (unsigned long long)(lo | (hi << 16)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <bool PK>
__device__ __forceinline__ void xg_unpack(float (&x)[XG_PER_THREAD], const bool (&ok)[XG_PER_THREAD]) {
  if constexpr (PK) {
#pragma unroll
    for (int k = 0; k < XG_PER_THREAD; k += 2)
      if (ok[k]) {
        const unsigned w = __float_as_uint(x[k]);
        x[k] = bf16_lo(w);
        x[k + 1] = bf16_hi(w);
      }
  }
}

// NR: group-size bucket (2, 4, 8 >= nranks; 1 for a 1-rank group) sizing the register arrays
template <int NR, bool PK = false>
__global__ void __launch_bounds__(XG_THREADS) xgmi_allreduce_kernel(XgmiArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  unsigned* err_w = a.ctr + a.max_blocks;
  const unsigned step = a.ctr[b] + 1u;
  const bool failed = a.ctr[a.max_blocks] != 0u;
  const int par = step & 1u;
  const int lo = b * XG_CHUNK;
  const bool two_hop = (a.form & 2) != 0;
  const int owner = two_hop ? b % a.nranks : a.rank;
  // two-hop tags carry the path bit (its ag slot is shared with grad_reduce's)
  const unsigned want = two_hop ? (step | XG_PATH_BIT) : step;
  const unsigned long long tag = (unsigned long long)want << 32;

  // 1. publish this slice as granules into this rank's own pull slot (two-hop: non-owners
  //    only); the optimizer state is local and only this thread touches it: prefetch it now,
  //    so the update after the gather costs no extra latency
  float v[NR][XG_PER_THREAD];
  float p_old[XG_PER_THREAD], m_old[XG_PER_THREAD], g[XG_PER_THREAD];
  int e[XG_PER_THREAD];
  bool ok[XG_PER_THREAD];
  unsigned long long* mine = reinterpret_cast<unsigned long long*>(a.region[a.rank] + par * a.gslot_bytes);
  const bool publish = !two_hop || owner != a.rank;
#pragma unroll
  for (int k = 0; k < XG_PER_THREAD; ++k) {
    ok[k] = lo + k * XG_THREADS + tid < a.n;
    e[k] = min(lo + k * XG_THREADS + tid, a.n - 1);
    g[k] = a.grad[e[k]];
    if (a.mode != 0) {
      p_old[k] = a.master[e[k]];
      m_old[k] = a.mom[e[k]];
    }
    if (!PK && ok[k] && publish)
      __hip_atomic_store(mine + e[k], tag | __float_as_uint(g[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if constexpr (PK) xg_pack<PK>(g, ok, e, publish ? mine : nullptr, tag);
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int k = 0; k < XG_PER_THREAD; ++k) v[r][k] = g[k];

  // 2. gather: the one-hop form (and the two-hop owner) reads every peer's pull slot, a two-hop
  //    non-owner the owner's ag slot; all loads of a round in flight before the first check
  const unsigned long long* src[NR];
  unsigned pending = 0;  // bit 4 r + k
  const bool gather_all = !two_hop || owner == a.rank;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    src[r] = reinterpret_cast<const unsigned long long*>(
        gather_all ? a.region[r] + par * a.gslot_bytes : a.region[owner] + a.ag_off + par * a.gslot_bytes);
#pragma unroll
    for (int k = 0; k < XG_PER_THREAD; ++k) {
      const bool need = gather_all ? (r < a.nranks && r != a.rank) : r == 0;
      if (need && ok[k] && (!PK || (k & 1) == 0)) pending |= 1u << (4 * r + k);
    }
  }
  xg_record_wait(a, step, xg_wait<NR>(a, src, pending, v, e, want, failed, err_w));
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (gather_all ? (r < a.nranks && r != a.rank) : r == 0) xg_unpack<PK>(v[r], ok);

  // 3. rank-order sum (two-hop non-owner: the owner's sum), publish (two-hop owner), scale,
  //    optimizer
  float sum[XG_PER_THREAD];
#pragma unroll
  for (int k = 0; k < XG_PER_THREAD; ++k) {
    sum[k] = v[0][k];
    if (gather_all) {
#pragma unroll
      for (int r = 1; r < NR; ++r)
        if (r < a.nranks) sum[k] += v[r][k];
    }
  }
  if (two_hop && owner == a.rank) {
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.region[a.rank] + a.ag_off + par * a.gslot_bytes);
    if constexpr (PK) {
      xg_pack<PK>(sum, ok, e, dst, tag);
    } else {
#pragma unroll
      for (int k = 0; k < XG_PER_THREAD; ++k)
        if (ok[k]) __hip_atomic_store(dst + e[k], tag | __float_as_uint(sum[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
#pragma unroll
  for (int k = 0; k < XG_PER_THREAD; ++k) {
    if (!ok[k]) continue;
    const float gr = sum[k] * a.scale;
    if (a.mode == 0) {
      a.out[e[k]] = gr;
    } else {
      float p, m;
      sgd_update(gr, p_old[k], m_old[k], a.lr, a.momentum, p, m);
      a.mom[e[k]] = m;
      a.master[e[k]] = p;
      if (a.mode == 1) write_shadow(a.shadow, e[k], p);
    }
  }
  __syncthreads();  // every thread read this workgroup's counter before it advances
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

// Uncached (fine-grained) device memory, zeroed, for on-GPU hand-offs by tagged granules
// between concurrently running kernels (the pipelined / persistent step's control words): every access bypasses
// the per-XCD L2s, as the xGMI regions' do.  Freed with xgmi_free.
//
// Pooled: a block given back with uncached_free is kept for the next request of its size class
// ON THE SAME DEVICE (zeroed again on reuse), never returned to the driver - an engine's control
// words and flags are re-allocated by every engine a process builds (tests, A/B candidates), and
// each hipFree / hipExtMallocWithFlags pair of fine-grained memory cost a device-wide
// synchronisation and a page-table update while other engines' kernels were queued.
namespace {
std::mutex g_uc_mu;
using UcKey = std::pair<int, long long>;       // (device, size class)
std::multimap<UcKey, void*> g_uc_free;         // (device, size class) -> free blocks
std::map<void*, UcKey> g_uc_size;              // every pooled block -> its device and size class
long long g_uc_violations = 0;                 // reused blocks whose canary was overwritten while free
long long uc_class(long long bytes) { return std::max<long long>(4096, (bytes + 4095) / 4096 * 4096); }
constexpr unsigned char UC_CANARY = 0xA5;
// A free block holds the canary byte everywhere: a kernel that still wrote to its old owner's
// control words after that owner was destroyed (a use-after-free) would show up as a broken
// canary when the block is handed out again (DNN_UNCACHED_CANARY=0 skips the check).
bool uc_check_canary() {
  const char* v = std::getenv("DNN_UNCACHED_CANARY");
  return v == nullptr || v[0] != '0';
}
}  // namespace

uintptr_t uncached_alloc(long long bytes) {
  const long long cls = uc_class(bytes);
  int dev = 0;
  xcheck(hipGetDevice(&dev), "hipGetDevice");
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_uc_mu);
    auto it = g_uc_free.find(UcKey{dev, cls});
    if (it != g_uc_free.end()) {
      p = it->second;
      g_uc_free.erase(it);
    }
  }
  if (p != nullptr && uc_check_canary()) {
    std::vector<unsigned char> h((size_t)cls);
    xcheck(hipMemcpy(h.data(), p, (size_t)cls, hipMemcpyDeviceToHost), "hipMemcpy(uncached canary)");
    long long bad = 0;
    for (unsigned char c : h) bad += c != UC_CANARY;
    if (bad) {
      std::lock_guard<std::mutex> lk(g_uc_mu);
      ++g_uc_violations;
      std::fprintf(stderr, "[uncached pool] %lld bytes of a free %lld-byte block were written after its free\n", bad,
                   cls);
    }
  }
  if (p == nullptr) {
    xcheck(hipExtMallocWithFlags(&p, cls, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
    std::lock_guard<std::mutex> lk(g_uc_mu);
    g_uc_size[p] = UcKey{dev, cls};
  }
  xcheck(hipMemset(p, 0, cls), "hipMemset(uncached)");
  xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return reinterpret_cast<uintptr_t>(p);
}

// Give an uncached_alloc block back to the pool (the caller has synchronised: no kernel uses it).
void uncached_free(uintptr_t p) {
  if (!p) return;
  UcKey key{0, 0};
  {
    std::lock_guard<std::mutex> lk(g_uc_mu);
    auto it = g_uc_size.find(reinterpret_cast<void*>(p));
    if (it == g_uc_size.end()) throw std::runtime_error("uncached_free: not a pooled uncached block");
    key = it->second;
  }
  const long long cls = key.second;
  if (uc_check_canary()) {
    xcheck(hipMemset(reinterpret_cast<void*>(p), UC_CANARY, cls), "hipMemset(uncached canary)");
    xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }
  std::lock_guard<std::mutex> lk(g_uc_mu);
  g_uc_free.emplace(key, reinterpret_cast<void*>(p));
}

// (diagnostic) pooled blocks: (total, free, canary violations seen on reuse)
std::tuple<long long, long long, long long> uncached_pool_stats() {
  std::lock_guard<std::mutex> lk(g_uc_mu);
  return {(long long)g_uc_size.size(), (long long)g_uc_free.size(), g_uc_violations};
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
                           double timeout_s, hipStream_t stream, int form, unsigned long long* wait) {
  const int nranks = (int)regions.size();
  if (nranks < 1 || nranks > XG_MAX_RANKS) throw std::runtime_error("xgmi all-reduce: 1..8 ranks");
  if (rank < 0 || rank >= nranks) throw std::runtime_error("xgmi all-reduce: bad rank");
  if (n <= 0 || n > capacity) throw std::runtime_error("xgmi all-reduce: n exceeds the region capacity");
  if (mode < 0 || mode > 2) throw std::runtime_error("xgmi all-reduce: bad mode");
  if (mode == 1 && n > ARENA) throw std::runtime_error("xgmi all-reduce: shadow mode is for the fused arena");
  static_assert(XG_PER_THREAD * XG_MAX_RANKS <= 32, "pending mask bits");
  XgmiArgs a{};
  for (int r = 0; r < nranks; ++r) a.region[r] = reinterpret_cast<unsigned char*>(regions[r]);
  a.rank = rank;
  a.nranks = nranks;
  a.n = n;
  a.gslot_bytes = xgmi_gslot_bytes(capacity);
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
  a.max_blocks = xgmi_max_blocks(capacity);
  a.abort_w = abort_w;
  a.timeout_ticks = (long long)(timeout_s * 1.0e8);
  if (form < 0 || form > 6 || (form & 1))
    throw std::runtime_error("xgmi all-reduce: form 0 (pull) or 2 (two-hop pull), + 4 for bf16 granules");
  a.form = nranks > 1 ? form : (form & 4);  // (one rank: no two-hop; bf16 rounding as the exchange does)
  a.ag_off = xgmi_ag_off(capacity);
  a.wait = wait;
  const int nblk = (n + XG_CHUNK - 1) / XG_CHUNK;
  if (wait != nullptr && nblk > XP_MAX_BLOCKS) throw std::runtime_error("xgmi all-reduce: wait ring holds 128 blocks");
  const bool pk = (a.form & 4) != 0;
  auto* kern = nranks == 1 ? (pk ? &xgmi_allreduce_kernel<1, true> : &xgmi_allreduce_kernel<1>)
               : pk ? (nranks <= 2 ? &xgmi_allreduce_kernel<2, true>
                                   : (nranks <= 4 ? &xgmi_allreduce_kernel<4, true> : &xgmi_allreduce_kernel<8, true>))
                    : (nranks <= 2 ? &xgmi_allreduce_kernel<2>
                                   : (nranks <= 4 ? &xgmi_allreduce_kernel<4> : &xgmi_allreduce_kernel<8>));
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(XG_THREADS), 0, stream, a);
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

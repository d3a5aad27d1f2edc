// Direct AQL dispatch (aql_dispatch.h).
#include "runtime/aql_dispatch.h"

#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace dnn {

namespace {

constexpr uint32_t QUEUE_SIZE = 64;       // packets (power of two)
constexpr size_t KARG_BYTES = 4096;       // one kernarg buffer (the fused kernel's block is 648 B)

std::string hsa_err(hsa_status_t s) {
  const char* m = nullptr;
  hsa_status_string(s, &m);
  return m ? m : ("status " + std::to_string((int)s));
}

struct AgentFind {
  uint32_t bdf = 0, domain = 0;
  hsa_agent_t gpu{0}, cpu{0};
  bool have_gpu = false, have_cpu = false;
};

hsa_status_t find_agents(hsa_agent_t a, void* data) {
  auto* f = static_cast<AgentFind*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) {
    f->cpu = a;
    f->have_cpu = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !f->have_gpu) {
    uint32_t bdf = 0, dom = 0;
    hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
    hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
    if (bdf == f->bdf && dom == f->domain) {
      f->gpu = a;
      f->have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg_pool(hsa_amd_memory_pool_t p, void* data) {
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
    *static_cast<hsa_amd_memory_pool_t*>(data) = p;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct SymFind {
  hsa_agent_t agent;
  std::string part;
  std::vector<AqlKernel> hits;
};

hsa_status_t on_symbol(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void* data) {
  auto* f = static_cast<SymFind*>(data);
  hsa_symbol_kind_t kind;
  if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
      kind != HSA_SYMBOL_KIND_KERNEL)
    return HSA_STATUS_SUCCESS;
  uint32_t len = 0;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
  std::string name(len, '\0');
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, name.data());
  if (name.find(f->part) == std::string::npos) return HSA_STATUS_SUCCESS;
  AqlKernel k;
  k.name = name;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group_static);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.private_bytes);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg_bytes);
  for (const auto& h : f->hits)  // (one code object can be listed by more than one executable view)
    if (h.object == k.object) return HSA_STATUS_SUCCESS;
  f->hits.push_back(k);
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_executable(hsa_executable_t e, void* data) {
  auto* f = static_cast<SymFind*>(data);
  hsa_executable_iterate_agent_symbols(e, f->agent, on_symbol, data);
  return HSA_STATUS_SUCCESS;
}

inline void cpu_relax() {
#if defined(__x86_64__)
  _mm_pause();
#endif
}

}  // namespace

class AqlQueue {
 public:
  hsa_agent_t gpu{0};
  hsa_queue_t* queue = nullptr;
  hsa_signal_t done{0};
  void* kernarg = nullptr;
  bool broken = false, in_flight = false;
  std::chrono::steady_clock::time_point t_start, t_doorbell;
  double timeout_s = 0.0;
  std::string name;
  // acquire at agent scope: a dispatched kernel reads device memory only (its arguments included),
  // which the agent-scope invalidate covers - the system scope adds host-memory coherence
  // (15.98 vs 16.10 us/step over 6 bench pairs: profiles/r6/aql/fence/); release at system
  // scope, so host reads and every later queue see the kernel's writes
  unsigned acq_scope = HSA_FENCE_SCOPE_AGENT, rel_scope = HSA_FENCE_SCOPE_SYSTEM;
  double last_wait_us = 0.0, last_whole_us = 0.0;
  std::mutex mu;

  ~AqlQueue() {
    // (process exit: the runtime tears the queue down itself; freeing here would race HIP's
    // own teardown order, so a live process never destroys a queue - one per device)
  }
};

AqlQueue* aql_queue(int hip_device, std::string* why) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<AqlQueue>> queues;
  static std::map<int, std::string> failed;
  std::lock_guard<std::mutex> lock(mu);
  auto it = queues.find(hip_device);
  if (it != queues.end()) return it->second.get();
  auto fit = failed.find(hip_device);
  if (fit != failed.end()) {
    if (why) *why = fit->second;
    return nullptr;
  }
  auto fail = [&](const std::string& m) -> AqlQueue* {
    failed[hip_device] = m;
    if (why) *why = m;
    return nullptr;
  };
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, hip_device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, hip_device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, hip_device) != hipSuccess)
    return fail("the HIP device's PCI address is not available");
  hsa_status_t s = hsa_init();  // (reference-counted: HIP initialised it already)
  if (s != HSA_STATUS_SUCCESS) return fail("hsa_init: " + hsa_err(s));
  AgentFind af;
  af.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
  af.domain = (uint32_t)dom;
  hsa_iterate_agents(find_agents, &af);
  if (!af.have_gpu || !af.have_cpu) return fail("no HSA GPU agent at the HIP device's PCI address");
  auto q = std::make_unique<AqlQueue>();
  q->gpu = af.gpu;
  s = hsa_queue_create(af.gpu, QUEUE_SIZE, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q->queue);
  if (s != HSA_STATUS_SUCCESS) return fail("hsa_queue_create: " + hsa_err(s));
  s = hsa_signal_create(0, 0, nullptr, &q->done);
  if (s != HSA_STATUS_SUCCESS) return fail("hsa_signal_create: " + hsa_err(s));
  hsa_amd_memory_pool_t pool{0};
  hsa_amd_agent_iterate_memory_pools(af.cpu, find_kernarg_pool, &pool);
  if (pool.handle == 0) return fail("no kernarg memory pool");
  s = hsa_amd_memory_pool_allocate(pool, KARG_BYTES, 0, &q->kernarg);
  if (s != HSA_STATUS_SUCCESS) return fail("kernarg allocation: " + hsa_err(s));
  s = hsa_amd_agents_allow_access(1, &af.gpu, nullptr, q->kernarg);
  if (s != HSA_STATUS_SUCCESS) return fail("kernarg access: " + hsa_err(s));
  if (const char* f = std::getenv("DNN_AQL_FENCE"); f != nullptr && std::strlen(f) == 2) {
    auto scope = [](char c) -> unsigned {
      return c == 'n' ? HSA_FENCE_SCOPE_NONE : c == 'a' ? HSA_FENCE_SCOPE_AGENT : HSA_FENCE_SCOPE_SYSTEM;
    };
    q->acq_scope = scope(f[0]);
    q->rel_scope = scope(f[1]);
  }
  AqlQueue* raw = q.get();
  queues[hip_device] = std::move(q);
  return raw;
}

AqlKernel aql_kernel(AqlQueue* q, const void* host_fn, const char* name_part) {
  if (q == nullptr) throw std::runtime_error("aql_kernel: no queue");
  hipFuncAttributes attr;
  if (hipFuncGetAttributes(&attr, host_fn) != hipSuccess)  // makes HIP load the code object
    throw std::runtime_error("aql_kernel: hipFuncGetAttributes failed");
  SymFind f;
  f.agent = q->gpu;
  f.part = name_part;
  // the loader's executable iteration comes from the AMD loader extension table (version 1.03)
  hsa_ven_amd_loader_1_03_pfn_t table;
  std::memset(&table, 0, sizeof(table));
  hsa_status_t s = hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(table), &table);
  if (s != HSA_STATUS_SUCCESS || table.hsa_ven_amd_loader_iterate_executables == nullptr)
    throw std::runtime_error("aql_kernel: no AMD loader extension (1.03): " + hsa_err(s));
  s = table.hsa_ven_amd_loader_iterate_executables(on_executable, &f);
  if (s != HSA_STATUS_SUCCESS) throw std::runtime_error("aql_kernel: executable iteration: " + hsa_err(s));
  if (f.hits.size() != 1)
    throw std::runtime_error("aql_kernel: " + std::to_string(f.hits.size()) + " kernel symbols match '" + name_part + "'");
  return f.hits[0];
}

void aql_dispatch(AqlQueue* q, const AqlKernel& k, const void* args, size_t bytes, unsigned grid_x,
                  unsigned block_x, unsigned dyn_lds, double timeout_s, bool args_on_device) {
  if (q == nullptr || q->broken) throw std::runtime_error("aql_dispatch: the queue is unusable");
  if (q->in_flight) throw std::runtime_error("aql_dispatch: the previous dispatch was not waited for");
  if (k.object == 0) throw std::runtime_error("aql_dispatch: no kernel object");
  if (bytes != k.kernarg_bytes || bytes > KARG_BYTES)
    throw std::runtime_error("aql_dispatch: " + std::to_string(bytes) + " argument bytes for a kernarg segment of " +
                             std::to_string(k.kernarg_bytes) + " (" + k.name + ")");
  if (grid_x == 0 || block_x == 0 || block_x > 1024 || k.group_static + dyn_lds > 163840)
    throw std::runtime_error("aql_dispatch: bad launch shape");
  std::lock_guard<std::mutex> lock(q->mu);
  using clk = std::chrono::steady_clock;
  q->t_start = clk::now();
  // kernel arguments: the caller's device-resident block as it is (the kernel re-reads its arguments
  // in its loops - from system memory each of those reads crosses the host link), or a copy in
  // this queue's host kernarg buffer (the previous dispatch completed: one dispatch in flight)
  const void* karg = args;
  if (!args_on_device) {
    std::memcpy(q->kernarg, args, bytes);
    karg = q->kernarg;
  }
  hsa_signal_store_relaxed(q->done, 1);
  hsa_queue_t* hq = q->queue;
  const uint64_t idx = hsa_queue_add_write_index_relaxed(hq, 1);
  while (idx - hsa_queue_load_read_index_scacquire(hq) >= hq->size) cpu_relax();
  auto* pkt = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(hq->base_address) + (idx & (hq->size - 1));
  pkt->workgroup_size_x = (uint16_t)block_x;
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->reserved0 = 0;
  pkt->grid_size_x = grid_x * block_x;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = k.private_bytes;
  pkt->group_segment_size = k.group_static + dyn_lds;
  pkt->kernel_object = k.object;
  pkt->kernarg_address = const_cast<void*>(karg);
  pkt->reserved2 = 0;
  pkt->completion_signal = q->done;
  // acquire / release fences (AqlQueue: agent / system): the kernel reads what HIP kernels and
  // copies wrote before it and HIP work after it reads what it wrote (the packet is the only
  // ordering between the two queues).  (DNN_AQL_FENCE=<acquire><release>, each n / a / s for
  // none / agent / system: measurement)
  const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                     (1u << HSA_PACKET_HEADER_BARRIER) |
                                     (q->acq_scope << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                     (q->rel_scope << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  const uint16_t setup = (uint16_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(hq->doorbell_signal, (hsa_signal_value_t)idx);
  q->t_doorbell = clk::now();
  q->timeout_s = timeout_s;
  q->name = k.name;
  q->in_flight = true;
}

void aql_wait(AqlQueue* q) {
  if (q == nullptr || !q->in_flight) return;
  using clk = std::chrono::steady_clock;
  const auto limit = q->t_doorbell + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(q->timeout_s));
  unsigned n = 0;
  while (hsa_signal_load_scacquire(q->done) != 0) {
    cpu_relax();
    if ((++n & 1023u) == 0 && clk::now() > limit) {
      q->broken = true;
      q->in_flight = false;
      throw std::runtime_error("aql_wait: " + q->name + " did not complete within " + std::to_string(q->timeout_s) + " s");
    }
  }
  const auto t2 = clk::now();
  q->in_flight = false;
  q->last_wait_us = std::chrono::duration<double, std::micro>(t2 - q->t_doorbell).count();
  q->last_whole_us = std::chrono::duration<double, std::micro>(t2 - q->t_start).count();
}

void aql_run(AqlQueue* q, const AqlKernel& k, const void* args, size_t bytes, unsigned grid_x, unsigned block_x,
             unsigned dyn_lds, double timeout_s, bool args_on_device) {
  aql_dispatch(q, k, args, bytes, grid_x, block_x, dyn_lds, timeout_s, args_on_device);
  aql_wait(q);
}

namespace {
struct Prepared {
  AqlQueue* q;
  AqlKernel k;
  void* args;  // device memory, written once (HIP's kernarg placement)
  size_t bytes;
  unsigned grid, block, lds;
  double timeout_s;
  hipStream_t stream;
};
std::mutex g_prep_mu;
std::vector<Prepared> g_prep;
std::map<std::pair<int, std::string>, AqlKernel> g_kernels;

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

int aql_prepare(const void* host_fn, const char* name_part, const void* args, size_t bytes, unsigned grid_x,
                unsigned block_x, unsigned dyn_lds, double timeout_s, hipStream_t stream) {
  int dev = 0;
  hip_ok(hipGetDevice(&dev), "aql_prepare: hipGetDevice");
  std::string why;
  AqlQueue* q = aql_queue(dev, &why);
  if (q == nullptr) throw std::runtime_error("aql_prepare: no AQL queue: " + why);
  std::lock_guard<std::mutex> lock(g_prep_mu);
  auto key = std::make_pair(dev, std::string(name_part));
  auto it = g_kernels.find(key);
  if (it == g_kernels.end()) it = g_kernels.emplace(key, aql_kernel(q, host_fn, name_part)).first;
  if (it->second.kernarg_bytes != bytes)
    throw std::runtime_error("aql_prepare: " + it->second.name + " has a kernarg segment of " +
                             std::to_string(it->second.kernarg_bytes) + " bytes, the parameter block " +
                             std::to_string(bytes));
  void* dargs = nullptr;  // (one small block per prepared launch shape, kept for the process)
  hip_ok(hipMalloc(&dargs, bytes), "aql_prepare: hipMalloc");
  hip_ok(hipMemcpy(dargs, args, bytes, hipMemcpyHostToDevice), "aql_prepare: hipMemcpy");
  g_prep.push_back(Prepared{q, it->second, dargs, bytes, grid_x, block_x, dyn_lds, timeout_s, stream});
  return (int)g_prep.size() - 1;
}

void aql_prepared_launch(int handle) {
  Prepared d;
  {
    std::lock_guard<std::mutex> lock(g_prep_mu);
    if (handle < 0 || handle >= (int)g_prep.size()) throw std::runtime_error("aql_prepared_run: bad handle");
    d = g_prep[handle];
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  hip_ok(hipStreamIsCapturing(d.stream, &cap), "aql_prepared_run: hipStreamIsCapturing");
  if (cap != hipStreamCaptureStatusNone) throw std::runtime_error("aql_prepared_run: a direct dispatch cannot be captured");
  // the stream's earlier work (the previous window, epoch_begin, copies) must be done: the AQL
  // queue is not ordered after it (usually idle already: one query)
  if (hipStreamQuery(d.stream) != hipSuccess) hip_ok(hipStreamSynchronize(d.stream), "aql_prepared_run: sync");
  aql_dispatch(d.q, d.k, d.args, d.bytes, d.grid, d.block, d.lds, d.timeout_s, true);
}

void aql_prepared_wait(int handle) {
  AqlQueue* q = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_prep_mu);
    if (handle < 0 || handle >= (int)g_prep.size()) throw std::runtime_error("aql_prepared_wait: bad handle");
    q = g_prep[handle].q;
  }
  aql_wait(q);
}

void aql_prepared_run(int handle) {
  aql_prepared_launch(handle);
  aql_prepared_wait(handle);
}

double aql_last_us(AqlQueue* q, bool whole) { return q == nullptr ? 0.0 : (whole ? q->last_whole_us : q->last_wait_us); }

}  // namespace dnn

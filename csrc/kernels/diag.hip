// Diagnostics that are kernels themselves.
//
// lds_poison: fill the LDS of every CU with one 32-bit pattern.  LDS is not cleared between
// kernels - a workgroup sees what the previous workgroup on its CU left there - so a kernel
// that reads LDS it did not write in this launch (a pad it assumes zero, a DMA it did not wait
// for) usually reads its OWN previous launch's identical bytes and passes; after a poison pass
// it reads the pattern instead, every time (tests/test_lds_hygiene_gpu.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "runtime/aql_dispatch.h"

namespace dnn {

constexpr int POISON_THREADS = 256;
constexpr int POISON_LDS = 163840;  // the whole 160 KB of a CU: one workgroup per CU at a time

__global__ void __launch_bounds__(POISON_THREADS) lds_poison_kernel(unsigned pattern) {
  extern __shared__ unsigned lds[];
  for (int i = threadIdx.x; i < POISON_LDS / 4; i += POISON_THREADS) lds[i] = pattern;
  __syncthreads();
}

void lds_poison(unsigned pattern, hipStream_t stream) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    throw std::runtime_error("lds_poison: device query failed");
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(lds_poison_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          POISON_LDS) != hipSuccess)
    throw std::runtime_error("lds_poison: 160 KB of dynamic LDS refused");
  // several waves of workgroups, so every CU runs at least one whatever the dispatcher's order
  hipLaunchKernelGGL(lds_poison_kernel, dim3(8 * cus), dim3(POISON_THREADS), POISON_LDS, stream, pattern);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("lds_poison: ") + hipGetErrorString(e));
}

// lds_squat: workgroups of one wave that each hold `bytes` of LDS filled with their own pattern,
// stay resident for spin_us (wall clock) and then count the words of their LDS that changed into
// *bad (vector atomics).  Launched ahead of an engine's kernels on another stream, they share CUs
// with them: a kernel whose LDS writes land outside its own allocation (an LDS-DMA base taken as
// absolute, say) shows up as changed words here or as different results there.
__global__ void __launch_bounds__(64) lds_squat_kernel(int bytes, long long spin_ticks, unsigned* bad) {
  extern __shared__ unsigned lds[];
  const unsigned pat = 0xC0DE0000u ^ (blockIdx.x * 2654435761u);
  const int n = bytes / 4;
  for (int i = threadIdx.x; i < n; i += 64) lds[i] = pat + (unsigned)i;
  __syncthreads();
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(64);
  unsigned changed = 0;
  for (int i = threadIdx.x; i < n; i += 64) changed += lds[i] != pat + (unsigned)i;
  if (changed) atomicAdd(bad, changed);
}

void lds_squat(int bytes, double spin_us, int blocks, uintptr_t bad, hipStream_t stream) {
  if (bytes < 4 || bytes > 65536 || blocks < 1 || blocks > 65536) throw std::runtime_error("lds_squat: bad shape");
  hipLaunchKernelGGL(lds_squat_kernel, dim3(blocks), dim3(64), bytes, stream, bytes, (long long)(spin_us * 100.0),
                     reinterpret_cast<unsigned*>(bad));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("lds_squat: ") + hipGetErrorString(e));
}

// aql_selftest: the direct AQL dispatch path (runtime/aql_dispatch.h) end to end on a trivial
// kernel - the queue, the loader lookup of a HIP-loaded kernel, host kernel arguments, dynamic
// LDS, the completion signal - with a short bound, before an engine trusts it with a launch.
__global__ void __launch_bounds__(256) aql_probe_kernel(int* out, int base) {
  extern __shared__ int probe_lds[];
  probe_lds[threadIdx.x] = base + (int)blockIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = probe_lds[255 - threadIdx.x] + 1;
}

bool aql_selftest(std::string* why) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    *why = "hipGetDevice failed";
    return false;
  }
  AqlQueue* q = aql_queue(dev, why);
  if (q == nullptr) return false;
  constexpr int BLOCKS = 300;  // more workgroups than CUs
  int* out = nullptr;
  if (hipMalloc(&out, BLOCKS * sizeof(int)) != hipSuccess || hipMemset(out, 0, BLOCKS * sizeof(int)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    *why = "probe buffer allocation failed";
    return false;
  }
  bool ok = true;
  try {
    const AqlKernel k = aql_kernel(q, reinterpret_cast<const void*>(aql_probe_kernel), "aql_probe_kernel");
    // the explicit parameter block: the pointer, then the int - 12 bytes (no tail padding, unlike
    // a struct of the two)
    unsigned char args[sizeof(int*) + sizeof(int)];
    const int base = 1000;
    std::memcpy(args, &out, sizeof(int*));
    std::memcpy(args + sizeof(int*), &base, sizeof(int));
    aql_run(q, k, args, sizeof(args), BLOCKS, 256, 256 * sizeof(int), 5.0);  // host kernarg path
    int host[BLOCKS];
    if (hipMemcpy(host, out, sizeof(host), hipMemcpyDeviceToHost) != hipSuccess) throw std::runtime_error("copy back");
    for (int b = 0; b < BLOCKS; ++b)
      if (host[b] != 1000 + b + 1) throw std::runtime_error("block " + std::to_string(b) + " wrote " + std::to_string(host[b]));
  } catch (const std::exception& e) {
    *why = std::string("aql_selftest: ") + e.what();
    ok = false;
  }
  hipFree(out);
  return ok;
}

}  // namespace dnn

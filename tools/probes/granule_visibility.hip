// Probe: how soon does a consumer workgroup see a {value, tag} granule that a producer
// workgroup stores (system-scope atomic) while both kernels/blocks are still running?
//  A: one launch, block 0 produces at t0 + 10 us then keeps running to t0 + 60 us, block 1 polls
//  B: producer and consumer in two kernels on two streams (concurrent), same timing
// for plain hipMalloc memory and uncached (fine-grained) memory.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__device__ __forceinline__ long long rt() { return (long long)__builtin_amdgcn_s_memrealtime(); }

__device__ void produce(unsigned long long* g, unsigned tag, long long* out) {
  const long long t0 = rt();
  while (rt() - t0 < 1000) __builtin_amdgcn_s_sleep(2);  // 10 us
  out[0] = rt();
  for (int i = 0; i < 64; ++i)
    __hip_atomic_store(g + i * 64 + threadIdx.x, ((unsigned long long)tag << 32) | 7u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  while (rt() - t0 < 6000) __builtin_amdgcn_s_sleep(2);  // keep running to 60 us
  out[1] = rt();
}
__device__ void consume(const unsigned long long* g, unsigned tag, long long* out) {
  const long long t0 = rt();
  for (int i = 0; i < 64; ++i) {
    while ((unsigned)(__hip_atomic_load(g + i * 64 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> 32) != tag) {
      __builtin_amdgcn_s_sleep(1);
      if (rt() - t0 > 100000000ll) { out[3] = 1; return; }
    }
  }
  out[2] = rt();
}
__global__ void both(unsigned long long* g, unsigned tag, long long* out) {
  if (blockIdx.x == 0) { if (threadIdx.x == 0) {} produce(g, tag, out); }
  else consume(g, tag, out);
}
__global__ void prod_k(unsigned long long* g, unsigned tag, long long* out) { produce(g, tag, out); }
__global__ void cons_k(unsigned long long* g, unsigned tag, long long* out) { consume(g, tag, out); }

int main() {
  long long* out;
  CK(hipMalloc(&out, 64));
  for (int kind = 0; kind < 2; ++kind) {
    unsigned long long* g;
    if (kind == 0) CK(hipMalloc(&g, 64 * 64 * 8));
    else CK(hipExtMallocWithFlags((void**)&g, 64 * 64 * 8, hipDeviceMallocUncached));
    CK(hipMemset(g, 0, 64 * 64 * 8));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    for (int mode = 0; mode < 2; ++mode)
      for (int rep = 0; rep < 3; ++rep) {
        const unsigned tag = 1 + 100 * kind + 10 * mode + rep;
        CK(hipMemset(out, 0, 64));
        CK(hipDeviceSynchronize());
        if (mode == 0) {
          hipLaunchKernelGGL(both, dim3(2), dim3(64), 0, s0, g, tag, out);
        } else {
          hipLaunchKernelGGL(cons_k, dim3(1), dim3(64), 0, s1, g, tag, out);
          hipLaunchKernelGGL(prod_k, dim3(1), dim3(64), 0, s0, g, tag, out);
        }
        CK(hipDeviceSynchronize());
        long long h[4];
        CK(hipMemcpy(h, out, 32, hipMemcpyDeviceToHost));
        printf("%s memory, %s: consumer saw the granules %.2f us after the producer stored them "
               "(producer ran on to +%.2f us)%s\n", kind ? "uncached" : "hipMalloc", mode ? "two kernels" : "one launch",
               (h[2] - h[0]) * 0.01, (h[1] - h[0]) * 0.01, h[3] ? " [TIMEOUT]" : "");
      }
    CK(hipFree(g));
  }
  return 0;
}

// Probe: do the two branches of a captured hipGraph (fork on a side stream, join back) run
// CONCURRENTLY on gfx950?  A consumer kernel on one branch spins (bounded, 2 s) on a flag
// that a producer kernel on the other branch sets after ~20 us of its own work.  If the
// runtime serialised the branches with the consumer first, the consumer's wait would hit its
// bound; concurrent branches give a wait of ~the producer's delay.  Both capture orders.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ long long rt() { return (long long)__builtin_amdgcn_s_memrealtime(); }

__global__ void consumer(unsigned* flag, unsigned want, long long* out) {
  if (threadIdx.x != 0) return;
  const long long t0 = rt();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
    __builtin_amdgcn_s_sleep(2);
    if (rt() - t0 > 200000000ll) { out[1] = 1; break; }  // 2 s bound
  }
  out[0] = rt() - t0;
}

__global__ void producer(unsigned* flag, unsigned want) {
  if (threadIdx.x != 0) return;
  const long long t0 = rt();
  while (rt() - t0 < 2000) __builtin_amdgcn_s_sleep(2);  // ~20 us
  __hip_atomic_store(flag, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
  unsigned* flag;
  long long* out;
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&out, 16));
  CK(hipMemset(flag, 0, 4));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  for (int order = 0; order < 2; ++order) {
    for (int rep = 0; rep < 3; ++rep) {
      const unsigned want = 1 + order * 10 + rep;
      CK(hipMemset(out, 0, 16));
      CK(hipDeviceSynchronize());
      hipGraph_t g;
      CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
      CK(hipEventRecord(fork, s0));
      CK(hipStreamWaitEvent(s1, fork, 0));
      if (order == 0) {  // consumer captured first (on the side stream), producer second
        hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, s1, flag, want, out);
        hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, s0, flag, want);
      } else {
        hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, s0, flag, want);
        hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, s1, flag, want, out);
      }
      CK(hipEventRecord(join, s1));
      CK(hipStreamWaitEvent(s0, join, 0));
      CK(hipStreamEndCapture(s0, &g));
      hipGraphExec_t ge;
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(ge, s0));
      CK(hipStreamSynchronize(s0));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      long long h[2];
      CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
      printf("order %d rep %d: consumer waited %.1f us (bound hit: %lld), graph wall %.3f ms\n", order, rep,
             h[0] * 0.01, h[1], ms);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}

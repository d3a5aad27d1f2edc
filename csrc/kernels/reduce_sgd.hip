// Batch reduction of weight gradients + momentum SGD (gfx950).
//
// Capability parity:
//  * the fc/conv weight-gradient reductions over the batch that ATen performs
//    inside convolution_backward / mm / sum(dim 0),
//  * torch.optim.SGD(lr, momentum, dampening=0) as used at
//    data_parallelism_train.py:187,199 (30 per-tensor ATen ops -> one launch over
//    the flat arena; "momentum buffer initialised to grad on the first step" is
//    reproduced by zeroing the buffer: m*0 + g == g),
//  * the per-step `loss.item()` accumulation of data_parallelism_train.py:202-203,
//    done on device (no host sync per step).
//
// Every gradient element is owned by one thread that sums the batch in a fixed
// order, so results are bitwise reproducible run to run (no float atomics).
#include "launchers.h"

namespace dnn {

constexpr int RT = 256;



__device__ __forceinline__ float dot_batch(const float* __restrict__ z, int zld, int o,
                                           const float* __restrict__ x, int xld, int i, int batch) {
  float s = 0.f;
  for (int b = 0; b < batch; ++b) s += z[(size_t)b * zld + o] * x[(size_t)b * xld + i];
  return s;
}

__device__ __forceinline__ float sum_batch(const float* __restrict__ z, int zld, int o, int batch) {
  float s = 0.f;
  for (int b = 0; b < batch; ++b) s += z[(size_t)b * zld + o];
  return s;
}

__device__ __forceinline__ void sgd_update(int e, float g, const ReduceArgs& a) {
  g *= a.grad_scale;
  if (a.fuse_sgd) {
    const float m = a.momentum * a.mom[e] + g;
    const float p = a.master[e] - a.lr * m;
    a.mom[e] = m;
    a.master[e] = p;
    a.shadow[e] = (bf16)p;
  } else {
    a.grad[e] = g;
  }
}

__global__ void __launch_bounds__(RT) grad_reduce_kernel(ReduceArgs a) {
  const int nblk = gridDim.x - a.bookkeeping;
  if ((int)blockIdx.x == nblk) {
    // bookkeeping block: epoch statistics + cursor advance (one wave, fixed order)
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      float ls = 0.f;
      int cs = 0;
      for (int b = lane; b < a.batch; b += 64) { ls += a.loss[b]; cs += a.correct[b]; }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) { ls += __shfl_down(ls, off); cs += __shfl_down(cs, off); }
      if (lane == 0) {
        const int bv = a.state[ST_BVALID];
        if (bv > 0) {
          a.stats[STAT_LOSS] += (double)ls / (double)bv;
          a.stats[STAT_BATCHES] += 1.0;
          a.stats[STAT_CORRECT] += (double)cs;
          a.stats[STAT_SAMPLES] += (double)bv;
        }
        a.state[ST_CURSOR] += 1;
      }
    }
    return;
  }
  for (int e = a.lo + blockIdx.x * RT + threadIdx.x; e < a.hi; e += nblk * RT) {
    float g = 0.f;
    bool real = true;
    if (e >= OFF_F1W && e < OFF_F1W + 48000) {
      const int r = e - OFF_F1W;
      g = dot_batch(a.z1, Z1_LD, r / 400, a.a0, A0_LD, r % 400, a.batch);
    } else if (e >= OFF_F1B && e < OFF_F1B + 120) {
      g = sum_batch(a.z1, Z1_LD, e - OFF_F1B, a.batch);
    } else if (e >= OFF_F2W && e < OFF_F2W + 10080) {
      const int r = e - OFF_F2W;
      g = dot_batch(a.z2, Z2_LD, r / 120, a.h1, H1_LD, r % 120, a.batch);
    } else if (e >= OFF_F2B && e < OFF_F2B + 84) {
      g = sum_batch(a.z2, Z2_LD, e - OFF_F2B, a.batch);
    } else if (e >= OFF_F3W && e < OFF_F3W + 840) {
      const int r = e - OFF_F3W;
      g = dot_batch(a.z3, Z3_LD, r / 84, a.h2, H2_LD, r % 84, a.batch);
    } else if (e >= OFF_F3B && e < OFF_F3B + 10) {
      g = sum_batch(a.z3, Z3_LD, e - OFF_F3B, a.batch);
    } else if (e >= OFF_C1W && e < OFF_C1W + 450) {
      g = sum_batch(a.slab, SLAB, SLAB_C1W + (e - OFF_C1W), a.batch);
    } else if (e >= OFF_C1B && e < OFF_C1B + 6) {
      g = sum_batch(a.slab, SLAB, SLAB_C1B + (e - OFF_C1B), a.batch);
    } else if (e >= OFF_C2W && e < OFF_C2W + 2400) {
      g = sum_batch(a.slab, SLAB, SLAB_C2W + (e - OFF_C2W), a.batch);
    } else if (e >= OFF_C2B && e < OFF_C2B + 16) {
      g = sum_batch(a.slab, SLAB, SLAB_C2B + (e - OFF_C2B), a.batch);
    } else {
      real = false;  // arena padding
    }
    if (real) sgd_update(e, g, a);
  }
}

// grads -> momentum SGD on the flat arena (+ bf16 shadow refresh).  Used after the
// per-step gradient all-reduce, and (lr = 0, momentum = 0, pack_only) to refresh the
// shadow after the arena was overwritten (checkpoint load, epoch averaging).
__global__ void __launch_bounds__(RT) sgd_apply_kernel(float* __restrict__ master, const float* __restrict__ grad,
                                                       float* __restrict__ mom, bf16* __restrict__ shadow, int n,
                                                       float lr, float momentum, float grad_scale, int pack_only) {
  for (int e = blockIdx.x * RT + threadIdx.x; e < n; e += gridDim.x * RT) {
    float p = master[e];
    if (!pack_only) {
      const float m = momentum * mom[e] + grad[e] * grad_scale;
      p -= lr * m;
      mom[e] = m;
      master[e] = p;
    }
    shadow[e] = (bf16)p;
  }
}

// ---- host launchers ---------------------------------------------------------------------
void launch_grad_reduce(const ReduceArgs& args, hipStream_t stream) {
  // ~one element per thread, at most one block per CU; +1 block for the bookkeeping
  int nblk = (args.hi - args.lo + RT - 1) / RT;
  if (nblk > 240) nblk = 240;
  if (nblk < 1) nblk = 1;
  hipLaunchKernelGGL(grad_reduce_kernel, dim3(nblk + (args.bookkeeping ? 1 : 0)), dim3(RT), 0, stream, args);
  HIP_CHECK(hipGetLastError());
}

void launch_sgd_apply(float* master, const float* grad, float* mom, bf16* shadow, int n, float lr, float momentum,
                      float grad_scale, int pack_only, hipStream_t stream) {
  const int nblk = (n + RT - 1) / RT;
  hipLaunchKernelGGL(sgd_apply_kernel, dim3(nblk), dim3(RT), 0, stream, master, grad, mom, shadow, n, lr, momentum,
                     grad_scale, pack_only);
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

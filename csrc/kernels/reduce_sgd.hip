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
#include "reduce_common.h"

namespace dnn {

constexpr int RT = 256;
static_assert(RT % SPLIT == 0, "split column lanes stay inside a wave");



__device__ __forceinline__ void grad_reduce_body(const ReduceArgs& a) {
  // block roles: [MLP tile blocks][MLP bias block][conv element blocks][bookkeeping]
  const bool mlp = a.hi > OFF_F1W;
  const bool conv = a.lo < OFF_F1W;
  int blk = blockIdx.x;
  if (mlp) {
    if (blk < TILE_BLOCKS) {
      const int t = blk * 4 + (threadIdx.x >> 6);
      if (t < FC_T0) fc_tile<0, false>(t, a);
      else if (t < FC_T0 + FC_T1) fc_tile<1, false>(t - FC_T0, a);
      else if (t < FC_TILES) fc_tile<2, false>(t - FC_T0 - FC_T1, a);
      return;
    }
    blk -= TILE_BLOCKS;
    constexpr int FB = (FCB_SLOTS + RT - 1) / RT;
    if (blk < FB) {
      fcb_task<false>(blk * RT + threadIdx.x, a);
      return;
    }
    blk -= FB;
  }
  if (conv) {
    constexpr int CB = (CONV_SLOTS + RT - 1) / RT;
    if (blk < CB) { conv_task<false>(blk * RT + threadIdx.x, a); return; }
    blk -= CB;
  }
  if (a.bookkeeping && blk == 0 && threadIdx.x < 64) bookkeeping<false>(a, threadIdx.x);
}

// diagnostic per-block timeline (tools/reduce_trace.py): [2 * block] start, [2 * block + 1]
// end of the block's work (after its stores drained)
__device__ __forceinline__ void reduce_stamp(const ReduceArgs& a, int k) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    if (k) __builtin_amdgcn_s_waitcnt(0);
    a.stamps[2 * blockIdx.x + k] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

__global__ void __launch_bounds__(RT) __attribute__((amdgpu_waves_per_eu(1, 2))) grad_reduce_kernel(ReduceArgs a) {
  reduce_stamp(a, 0);
  if (a.xg_region != nullptr) {  // gradients -> the shared slot of the coming xGMI step
    const unsigned step = a.xg_ctr[0] + 1u;
    a.grad = reinterpret_cast<float*>(a.xg_region + a.xg_flag_bytes + (step & 1u) * a.xg_slot_bytes);
  }
  grad_reduce_body(a);
  if (a.stamps != nullptr) __syncthreads();
  reduce_stamp(a, 1);
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
    write_shadow(shadow, e, p);
  }
}

// Epoch start on the compute stream in ONE launch: the epoch's sample order (uploaded ahead
// of time into a staging buffer on a side stream) -> the order the bookkeeping reads, the
// first step's sample ids, cursor 0 and the first batch's valid count.
__global__ void __launch_bounds__(RT) epoch_begin_kernel(const int32_t* __restrict__ staged, int32_t* __restrict__ order,
                                                         int n, int32_t* __restrict__ state,
                                                         int32_t* __restrict__ batch_ids, int batch) {
  for (int i = blockIdx.x * RT + threadIdx.x; i < n; i += gridDim.x * RT) {
    const int32_t v = staged[i];
    order[i] = v;
    if (i < batch) batch_ids[i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    state[ST_CURSOR] = 0;
    state[ST_BVALID] = min(batch, n);
  }
}

// ---- host launchers ---------------------------------------------------------------------
void launch_epoch_begin(const int32_t* staged, int32_t* order, int n, int32_t* state, int32_t* batch_ids, int batch,
                        hipStream_t stream) {
  const int nblk = max(1, min((n + RT - 1) / RT, 256));
  hipLaunchKernelGGL(epoch_begin_kernel, dim3(nblk), dim3(RT), 0, stream, staged, order, n, state, batch_ids, batch);
  HIP_CHECK(hipGetLastError());
}

void launch_grad_reduce(const ReduceArgs& args, hipStream_t stream) {
  const bool mlp = args.hi > OFF_F1W;
  const bool conv = args.lo < OFF_F1W;
  int nblk = 0;
  if (mlp) nblk += TILE_BLOCKS + (FCB_SLOTS + RT - 1) / RT;
  if (conv) nblk += (CONV_SLOTS + RT - 1) / RT;
  if (args.bookkeeping) nblk += 1;
  if (nblk == 0) return;
  hipLaunchKernelGGL(grad_reduce_kernel, dim3(nblk), dim3(RT), 0, stream, args);
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

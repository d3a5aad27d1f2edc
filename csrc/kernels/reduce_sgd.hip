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
#include "reduce_device.h"

namespace dnn {

int grad_reduce_blocks() { return GRAD_REDUCE_BLOCKS; }

// diagnostic per-block timeline (tools/reduce_trace.py): [2 * block] start, [2 * block + 1]
// end of the block's work (after its stores drained)
__device__ __forceinline__ void reduce_stamp(const ReduceArgs& a, int k) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    if (k) __builtin_amdgcn_s_waitcnt(0);
    a.stamps[2 * blockIdx.x + k] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

template <int NR, bool PK = false>
__global__ void __launch_bounds__(RT) __attribute__((amdgpu_waves_per_eu(1, 2))) grad_reduce_kernel(const ReduceArgs a) {
  reduce_stamp(a, 0);
  reduce_block<NR, PK>(a, blockIdx.x, threadIdx.x);
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
      float m;
      sgd_update(grad[e] * grad_scale, p, mom[e], lr, momentum, p, m);
      mom[e] = m;
      master[e] = p;
    }
    write_shadow(shadow, e, p);
  }
}

// Epoch start on the compute stream in ONE launch: the epoch's sample order (uploaded ahead
// of time into a staging buffer on a side stream) -> the order the bookkeeping reads, the
// first step's sample ids, cursor 0 and the first batch's valid count.
// With image staging (stage != nullptr): also the ids of step 1 (next_ids) and step 0's images
// + labels in the stage buffer, which the fused kernel reads instead of chasing its batch id.
__global__ void __launch_bounds__(RT) epoch_begin_kernel(const int32_t* __restrict__ staged, int32_t* __restrict__ order,
                                                         int n, int32_t* __restrict__ state,
                                                         int32_t* __restrict__ batch_ids, int batch,
                                                         const uint8_t* __restrict__ images,
                                                         const int32_t* __restrict__ labels,
                                                         int32_t* __restrict__ next_ids,
                                                         unsigned char* __restrict__ stage) {
  for (int i = blockIdx.x * RT + threadIdx.x; i < n; i += gridDim.x * RT) {
    const int32_t v = staged[i];
    order[i] = v;
    if (i < batch) batch_ids[i] = v;
  }
  if (stage != nullptr) {
    constexpr int V = IMG / 16;  // 16-B vectors per image
    for (int i = blockIdx.x * RT + threadIdx.x; i < batch * V; i += gridDim.x * RT) {
      const int b = i / V, k = i - b * V;
      if (b < n) {
        const int s = staged[b];
        reinterpret_cast<uint4*>(stage)[i] = reinterpret_cast<const uint4*>(images + (size_t)s * IMG)[k];
        if (k == 0) reinterpret_cast<int32_t*>(stage + (size_t)batch * IMG)[b] = labels[s];
      }
    }
  }
  if (next_ids != nullptr)  // (the staged step, and the fp32 persistent launch: step 1's ids)
    for (int b = blockIdx.x * RT + threadIdx.x; b < batch; b += gridDim.x * RT)
      next_ids[b] = batch + b < n ? staged[batch + b] : -1;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    state[ST_CURSOR] = 0;
    state[ST_BVALID] = min(batch, n);
  }
}

// ---- host launchers ---------------------------------------------------------------------
void launch_epoch_begin(const int32_t* staged, int32_t* order, int n, int32_t* state, int32_t* batch_ids, int batch,
                        const uint8_t* images, const int32_t* labels, int32_t* next_ids, unsigned char* stage,
                        hipStream_t stream) {
  if (stage != nullptr && (images == nullptr || labels == nullptr || next_ids == nullptr))
    throw std::runtime_error("epoch_begin: staging needs the images, labels and next_ids");
  const int nblk = max(1, min((max(n, batch * (IMG / 16)) + RT - 1) / RT, 256));
  hipLaunchKernelGGL(epoch_begin_kernel, dim3(nblk), dim3(RT), 0, stream, staged, order, n, state, batch_ids, batch,
                     images, labels, next_ids, stage);
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
  // the exchange waits on the same elements of every peer, which the same block reduces there:
  // every block must be resident at once (<= XP_MAX_BLOCKS blocks of RT threads, at most one
  // per CU of the 256) and the launch must take the whole arena
  if (args.xp_nranks > 0 && (nblk > XP_MAX_BLOCKS || !(mlp && conv && args.lo == 0 && args.hi >= ARENA)))
    throw std::runtime_error("grad_reduce exchange needs the whole-arena grid");
  const int nr = args.xp_nranks;
  if (nr > XG_MAX_RANKS) throw std::runtime_error("grad_reduce exchange: at most 8 ranks");
  const bool pk = (args.xp_mode & 4) != 0;
  auto* kern = nr == 0 ? &grad_reduce_kernel<1>
               : pk ? (nr <= 2 ? &grad_reduce_kernel<2, true>
                               : (nr <= 4 ? &grad_reduce_kernel<4, true> : &grad_reduce_kernel<8, true>))
                    : (nr <= 2 ? &grad_reduce_kernel<2> : (nr <= 4 ? &grad_reduce_kernel<4> : &grad_reduce_kernel<8>));
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(RT), 0, stream, args);
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

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



// One launch's blocks: [MLP tile blocks][MLP bias blocks][conv element blocks][bookkeeping].
// Returns true (block-uniform) when this block reduced arena elements.
template <class Sink>
__device__ __forceinline__ bool grad_reduce_body(const ReduceArgs& a, Sink& sk) {
  const bool mlp = a.hi > OFF_F1W;
  const bool conv = a.lo < OFF_F1W;
  int blk = blockIdx.x;
  if (mlp) {
    if (blk < TILE_BLOCKS) {
      const int t = blk * 4 + (threadIdx.x >> 6);
      if (t < FC_T0) fc_tile<0, false>(t, a, sk);
      else if (t < FC_T0 + FC_T1) fc_tile<1, false>(t - FC_T0, a, sk);
      else if (t < FC_TILES) fc_tile<2, false>(t - FC_T0 - FC_T1, a, sk);
      return true;
    }
    blk -= TILE_BLOCKS;
    constexpr int FB = (FCB_SLOTS + RT - 1) / RT;
    if (blk < FB) {
      fcb_task<false>(blk * RT + threadIdx.x, a, sk);
      return true;
    }
    blk -= FB;
  }
  if (conv) {
    constexpr int CB = (CONV_SLOTS + RT - 1) / RT;
    if (blk < CB) { conv_task<false>(blk * RT + threadIdx.x, a, sk); return true; }
    blk -= CB;
  }
  if (a.bookkeeping && blk == 0 && threadIdx.x < 64) bookkeeping<false>(a, threadIdx.x);
  return false;
}

constexpr int GRAD_REDUCE_BLOCKS =
    TILE_BLOCKS + (FCB_SLOTS + RT - 1) / RT + (CONV_SLOTS + RT - 1) / RT + 1;
static_assert(GRAD_REDUCE_BLOCKS <= XP_MAX_BLOCKS, "exchange flag table B has a column per reduce block");
int grad_reduce_blocks() { return GRAD_REDUCE_BLOCKS; }

__device__ __forceinline__ unsigned xp_ld(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The one-launch all-reduce exchange of ONE block (same protocol as xgmi_allreduce_kernel,
// per reduce block instead of per 1024-element slice):
//   publish - the block's gradients are already in the own slot (XpSink::put, system-
//             coherent stores); drain them, then push this block's step flag into EVERY
//             peer's flag table B (remote stores; the peer polls locally);
//   wait    - lanes 0..N-1 poll the N flags of this block (bounded: timeout / abort word ->
//             sticky error word, never a hang);
//   reduce  - every lane reads its elements from all N slots (7 links at once), sums in RANK
//             ORDER (bit-identical replicas), scales by 1/N, applies momentum SGD + images.
// Double buffering by step parity is safe for the same reason as in the slice kernel: block b
// overwrites its elements of slot (s & 1) at step s + 2 only after every peer's block b
// published step s + 1, which each does after finishing its step s reads of those elements.
__device__ __forceinline__ void xp_exchange(const ReduceArgs& a, const XpSink& sk, unsigned step, bool failed) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int par = step & 1u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own slot stores acknowledged
  __syncthreads();
  if (tid < 64) {
    if (a.xp_fences & 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid < a.xp_nranks && tid != a.xp_rank) {
      unsigned* flags = reinterpret_cast<unsigned*>(a.xp_region[tid] + a.xp_flag_off);
      __hip_atomic_store(flags + a.xp_rank * XP_MAX_BLOCKS + b, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (tid < a.xp_nranks && tid != a.xp_rank && !failed) {
    const unsigned* f = reinterpret_cast<const unsigned*>(a.xp_region[a.xp_rank] + a.xp_flag_off) +
                        tid * XP_MAX_BLOCKS + b;
    const long long t0 = wall_clock64();
    int spins = 0;
    while ((int)(xp_ld(f) - step) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 255) == 0) {
        if (wall_clock64() - t0 > a.xp_timeout_ticks || xp_ld(a.xp_abort) != 0u) {
          __hip_atomic_store(a.xp_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
  }
  if (tid < 64 && (a.xp_fences & 2)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // every peer load in flight before the first use (invalid lanes read element 0: harmless)
  float v[XG_MAX_RANKS][4];
#pragma unroll
  for (int r = 0; r < XG_MAX_RANKS; ++r) {
    if (r < a.xp_nranks) {
      const unsigned* src = reinterpret_cast<const unsigned*>(a.xp_region[r] + a.xp_flag_bytes + par * a.xp_slot_bytes);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[r][j] = r == a.xp_rank ? sk.g[j] : __uint_as_float(xp_ld(src + sk.e[j]));
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!sk.v[j]) continue;
    float s = v[0][j];
#pragma unroll
    for (int r = 1; r < XG_MAX_RANKS; ++r)
      if (r < a.xp_nranks) s += v[r][j];
    const float gr = s * a.xp_scale;
    float p, m;
    sgd_update(gr, sk.p[j], sk.m[j], a.lr, a.momentum, p, m);
    a.mom[sk.e[j]] = m;
    a.master[sk.e[j]] = p;
    write_shadow(a.shadow, sk.e[j], p);
  }
  __syncthreads();
  if (tid == 0) a.xp_ctr[b] = step;
}

// diagnostic per-block timeline (tools/reduce_trace.py): [2 * block] start, [2 * block + 1]
// end of the block's work (after its stores drained)
__device__ __forceinline__ void reduce_stamp(const ReduceArgs& a, int k) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    if (k) __builtin_amdgcn_s_waitcnt(0);
    a.stamps[2 * blockIdx.x + k] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

__global__ void __launch_bounds__(RT) __attribute__((amdgpu_waves_per_eu(1, 2))) grad_reduce_kernel(const ReduceArgs a) {
  reduce_stamp(a, 0);
  if (a.xp_nranks > 0) {  // one-launch all-reduce: reduce -> exchange -> SGD, per block
    // (the arguments are only read on this path: the per-lane region index then reads the
    //  kernel-argument segment directly instead of a private copy of the whole struct)
    const unsigned step = a.xp_ctr[blockIdx.x] + 1u;
    const bool failed = *a.xp_err != 0u;
    XpSink sk;
    sk.own = reinterpret_cast<unsigned*>(a.xp_region[a.xp_rank] + a.xp_flag_bytes + (step & 1u) * a.xp_slot_bytes);
    if (grad_reduce_body(a, sk)) xp_exchange(a, sk, step, failed);
  } else {
    ReduceArgs d_args = a;
    if (a.xg_region != nullptr) {  // gradients -> the shared slot of the coming xGMI step
      const unsigned step = a.xg_ctr[0] + 1u;
      d_args.grad = reinterpret_cast<float*>(a.xg_region + a.xg_flag_bytes + (step & 1u) * a.xg_slot_bytes);
    }
    DirectSink d;
    grad_reduce_body(d_args, d);
  }
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
    for (int b = blockIdx.x * RT + threadIdx.x; b < batch; b += gridDim.x * RT)
      next_ids[b] = batch + b < n ? staged[batch + b] : -1;
  }
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
  // the exchange waits on the same block of every peer: every block must be resident at once
  // (<= XP_MAX_BLOCKS blocks of RT threads, one per CU of the 256) and take the whole arena
  if (args.xp_nranks > 0 && (nblk > XP_MAX_BLOCKS || !mlp || !conv))
    throw std::runtime_error("grad_reduce exchange needs the whole-arena grid");
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

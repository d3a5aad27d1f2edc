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
      if (t < FC_T0) fc_tile<0>(t, a, sk);
      else if (t < FC_T0 + FC_T1) fc_tile<1>(t - FC_T0, a, sk);
      else if (t < FC_TILES) fc_tile<2>(t - FC_T0 - FC_T1, a, sk);
      return true;
    }
    blk -= TILE_BLOCKS;
    constexpr int FB = (FCB_SLOTS + RT - 1) / RT;
    if (blk < FB) {
      fcb_task(blk * RT + threadIdx.x, a, sk);
      return true;
    }
    blk -= FB;
  }
  if (conv) {
    constexpr int CB = (CONV_SLOTS + RT - 1) / RT;
    if (blk < CB) { conv_task(blk * RT + threadIdx.x, a, sk); return true; }
    blk -= CB;
  }
  if (a.bookkeeping && blk == 0 && threadIdx.x < 64) bookkeeping(a, threadIdx.x);
  return false;
}

constexpr int GRAD_REDUCE_BLOCKS =
    TILE_BLOCKS + (FCB_SLOTS + RT - 1) / RT + (CONV_SLOTS + RT - 1) / RT + 1;
static_assert(GRAD_REDUCE_BLOCKS <= XP_MAX_BLOCKS, "one exchange step counter per reduce block");
int grad_reduce_blocks() { return GRAD_REDUCE_BLOCKS; }

__device__ __forceinline__ unsigned long long xp_ld(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Exchange-wait accounting (ReduceArgs::xp_wait, optional): every wave stores the longest wait
// of its lanes for this step (s_memrealtime ticks, 100 MHz) into its own word of the ring entry
// [step % XP_WAIT_RING][block][wave] as {step << 32 | ticks} - a plain store per wave, no
// atomics; the host takes the max over blocks and waves (parallel/xgmi.py wait_stats).
__device__ __forceinline__ void record_wait(const ReduceArgs& a, unsigned step, long long ticks) {
  if (a.xp_wait == nullptr) return;
  unsigned t = (unsigned)min(ticks, 0xffffffffll);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t = max(t, (unsigned)__shfl_xor((int)t, off));
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    a.xp_wait[((size_t)(step % XP_WAIT_RING) * XP_MAX_BLOCKS + blockIdx.x) * (RT / 64) + w] =
        ((unsigned long long)step << 32) | t;
  }
}

// Poll the granules in `pending` (bit 4 r + j: element j of source r) until each tag shows
// `step`; the values land in v[r][j].  Every load of a round is in flight before the first
// check.  Bounded: timeout / abort word -> sticky error word, never a hang.  Returns the wait.
template <int NR>
__device__ __forceinline__ long long poll_granules(const ReduceArgs& a, const unsigned long long* const (&src)[NR],
                                                   const int (&e)[4], unsigned pending, unsigned step, bool failed,
                                                   float (&v)[NR][4]) {
  const long long t0 = wall_clock64();
  while (pending != 0u) {
    unsigned long long x[NR][4];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (pending & (1u << (4 * r + j))) x[r][j] = xp_ld(src[r] + e[j]);
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((pending & (1u << (4 * r + j))) && (unsigned)(x[r][j] >> 32) == step) {
          v[r][j] = __uint_as_float((unsigned)x[r][j]);
          pending &= ~(1u << (4 * r + j));
        }
    if (pending == 0u || failed) break;
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > a.xp_timeout_ticks ||
        __hip_atomic_load(a.xp_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
      __hip_atomic_store(a.xp_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
  return wall_clock64() - t0;
}

template <bool PK>
__device__ __forceinline__ void apply_update(const ReduceArgs& a, const XpSinkT<PK>& sk, const float (&s)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!sk.v[j]) continue;
    const float gr = s[j] * a.xp_scale;
    float p, m;
    sgd_update(gr, sk.p[j], sk.m[j], a.lr, a.momentum, p, m);
    a.mom[sk.e[j]] = m;
    a.master[sk.e[j]] = p;
    write_shadow(a.shadow, sk.e[j], p);
  }
}

// bf16 granules (PK): round the pairs (0, 1) and (2, 3) of x to bf16 IN PLACE - a lane's own
// contribution included, so every rank sums the same numbers - and, if dst, publish each pair
// as one granule {lo | hi << 16, step} at the index of its first element (unique: an element
// has one owner lane)
template <bool PK>
__device__ __forceinline__ void pack_pairs(float (&x)[4], const bool (&valid)[4], const int (&e)[4],
                                           unsigned long long* dst, unsigned long long tag) {
  if constexpr (PK) {
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      if (!valid[k]) continue;
      const unsigned lo = bf16_bits(x[k]), hi = valid[k + 1] ? bf16_bits(x[k + 1]) : 0u;
      x[k] = bf16_lo(lo);
      x[k + 1] = bf16_lo(hi);
      if (dst != nullptr)
        __hip_atomic_store(dst + e[k], tag | (unsigned long long)(lo | (hi << 16)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// which of a lane's elements are polled as granules: all valid ones, or (PK) each pair's first
template <bool PK>
__device__ __forceinline__ bool polled(const bool (&valid)[4], int j) { return valid[j] && (!PK || (j & 1) == 0); }

// PK: a polled pair's raw word (in x[k]) -> its two values
template <bool PK>
__device__ __forceinline__ void unpack_pairs(float (&x)[4], const bool (&valid)[4]) {
  if constexpr (PK) {
#pragma unroll
    for (int k = 0; k < 4; k += 2)
      if (valid[k]) {
        const unsigned w = __float_as_uint(x[k]);
        x[k] = bf16_lo(w);
        x[k + 1] = bf16_hi(w);
      }
  }
}

// The one-launch all-reduce exchange of ONE lane's (<= 4) reduced elements.  Each element
// was stored as a granule {value, step} (XpSink::put); the lane reads the same element's
// granule from every peer's slot over xGMI (7 links at once) until each tag shows this step,
// sums the N values in RANK ORDER (bit-identical replicas), scales by 1/N and applies momentum
// SGD + the bf16 images.  The value and its tag are one 8-byte atomic word, so no flag, fence or
// barrier orders anything: a tag match IS the data.
// Double buffering by step parity: the owner overwrites its element e of slot (s & 1) at step
// s + 2 only after it read every peer's step s + 1 granule of e, which each peer wrote only
// after it had read the owner's step s granule of e.
// NR: group-size bucket (2, 4 or 8 >= xp_nranks) - sizes the register arrays, so a 2-rank
// group does not pay for 8 ranks' loads in flight.  PK: bf16 granules (half the link bytes;
// the sum stays fp32 in rank order).
template <int NR, bool PK>
__device__ __forceinline__ void xp_exchange(const ReduceArgs& a, XpSinkT<PK>& sk, unsigned step, bool failed) {
  const int par = step & 1u;
  pack_pairs<PK>(sk.g, sk.v, sk.e, sk.own, sk.tag);
  float v[NR][4];
  unsigned pending = 0;
  const unsigned long long* src[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    src[r] = reinterpret_cast<const unsigned long long*>(a.xp_region[r] + a.xp_gslot_off + par * a.xp_gslot_bytes);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[r][j] = sk.g[j];
      if (r < a.xp_nranks && r != a.xp_rank && polled<PK>(sk.v, j)) pending |= 1u << (4 * r + j);
    }
  }
  record_wait(a, step, poll_granules<NR>(a, src, sk.e, pending, step, failed, v));
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (r < a.xp_nranks && r != a.xp_rank) unpack_pairs<PK>(v[r], sk.v);
  float s[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s[j] = v[0][j];
#pragma unroll
    for (int r = 1; r < NR; ++r)
      if (r < a.xp_nranks) s[j] += v[r][j];
  }
  apply_update(a, sk, s);
}

// The two-hop pull form (xp_mode bit 2): reduce-scatter + all-gather where every rank writes
// only its OWN region.  Block k's elements belong to rank k % N.  A non-owner lane has stored
// its granules into its own pull slot (XpSink::put); the owner lane reads them from the N - 1
// peers' pull slots, sums the N values in RANK ORDER (the same fp32 additions as xp_exchange,
// so both forms give bit-identical parameters), stores {sum, step} into its own ag slot and
// applies SGD; the other ranks read that slot.  2 E / N granules per link instead of E, one
// more dependent remote read.  PK: the sum is all-gathered as bf16 too (every rank, the owner
// included, applies the rounded sum).
template <int NR, bool PK>
__device__ __forceinline__ void xp_exchange_rsag(const ReduceArgs& a, XpSinkT<PK>& sk, unsigned step, bool failed) {
  const int par = step & 1u;
  const int owner = blockIdx.x % a.xp_nranks;
  pack_pairs<PK>(sk.g, sk.v, sk.e, sk.own, sk.tag);  // (null own on the owner: rounding only)
  float s[4];
  long long waited;
  if (owner == a.xp_rank) {
    float v[NR][4];
    unsigned pending = 0;
    const unsigned long long* src[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      src[r] = reinterpret_cast<const unsigned long long*>(a.xp_region[r] + a.xp_gslot_off + par * a.xp_gslot_bytes);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[r][j] = sk.g[j];
        if (r < a.xp_nranks && r != a.xp_rank && polled<PK>(sk.v, j)) pending |= 1u << (4 * r + j);
      }
    }
    waited = poll_granules<NR>(a, src, sk.e, pending, step, failed, v);
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (r < a.xp_nranks && r != a.xp_rank) unpack_pairs<PK>(v[r], sk.v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = v[0][j];
#pragma unroll
      for (int r = 1; r < NR; ++r)
        if (r < a.xp_nranks) s[j] += v[r][j];
    }
    const unsigned long long tag = (unsigned long long)step << 32;
    unsigned long long* dst =
        reinterpret_cast<unsigned long long*>(a.xp_region[a.xp_rank] + a.xp_ag_off + par * a.xp_gslot_bytes);
    if constexpr (PK) {
      pack_pairs<PK>(s, sk.v, sk.e, dst, tag);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (sk.v[j])
          __hip_atomic_store(dst + sk.e[j], tag | __float_as_uint(s[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  } else {
    const unsigned long long* src[1] = {
        reinterpret_cast<const unsigned long long*>(a.xp_region[owner] + a.xp_ag_off + par * a.xp_gslot_bytes)};
    float v[1][4];
    unsigned pending = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[0][j] = 0.f;
      if (polled<PK>(sk.v, j)) pending |= 1u << j;
    }
    waited = poll_granules<1>(a, src, sk.e, pending, step, failed, v);
    unpack_pairs<PK>(v[0], sk.v);
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = v[0][j];
  }
  record_wait(a, step, waited);
  apply_update(a, sk, s);
}

// diagnostic per-block timeline (tools/reduce_trace.py): [2 * block] start, [2 * block + 1]
// end of the block's work (after its stores drained)
__device__ __forceinline__ void reduce_stamp(const ReduceArgs& a, int k) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    if (k) __builtin_amdgcn_s_waitcnt(0);
    a.stamps[2 * blockIdx.x + k] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

// NR = 1: local reduction (+ SGD, or gradients out); NR = 2 / 4 / 8: the one-launch
// exchange for groups of up to NR ranks (separate instances keep the local step's registers
// at its own need).
template <int NR, bool PK = false>
__global__ void __launch_bounds__(RT) __attribute__((amdgpu_waves_per_eu(1, 2))) grad_reduce_kernel(const ReduceArgs a) {
  reduce_stamp(a, 0);
  if constexpr (NR > 1) {  // one-launch all-reduce: reduce -> exchange -> SGD, per lane
    const unsigned step = a.xp_ctr[blockIdx.x] + 1u;
    const bool failed = *a.xp_err != 0u;
    XpSinkT<PK> sk;
    sk.tag = (unsigned long long)step << 32;
    // pull: every lane's granules go to this rank's slot; two-hop: only non-owners' (the owner
    // publishes the SUM in its ag slot instead)
    const bool publish = (a.xp_mode & 2) == 0 || (int)(blockIdx.x % a.xp_nranks) != a.xp_rank;
    sk.own = publish ? reinterpret_cast<unsigned long long*>(a.xp_region[a.xp_rank] + a.xp_gslot_off +
                                                             (step & 1u) * a.xp_gslot_bytes)
                     : nullptr;
    if (grad_reduce_body(a, sk)) {
      if ((a.xp_mode & 2) == 0) xp_exchange<NR, PK>(a, sk, step, failed);
      else xp_exchange_rsag<NR, PK>(a, sk, step, failed);
    }
    __syncthreads();  // every thread read this block's counter before it advances
    if (threadIdx.x == 0) a.xp_ctr[blockIdx.x] = step;
  } else {
    DirectSink d;
    grad_reduce_body(a, d);
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
  // the exchange waits on the same elements of every peer, which the same block reduces there:
  // every block must be resident at once (<= XP_MAX_BLOCKS blocks of RT threads, at most one
  // per CU of the 256) and the launch must take the whole arena
  if (args.xp_nranks > 0 && (nblk > XP_MAX_BLOCKS || !mlp || !conv))
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

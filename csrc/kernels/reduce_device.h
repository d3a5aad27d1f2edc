// Device code of the batch reduction + momentum SGD + one-launch xGMI exchange, shared by the
// grad_reduce kernel (reduce_sgd.hip) and the pipelined / persistent launches' reduction
// workgroups (lenet_fused.hip, lenet_f32.hip).  See reduce_sgd.hip for the parity notes.
#pragma once
#include "reduce_common.h"

namespace dnn {

constexpr int RT = 256;
static_assert(RT % SPLIT == 0, "split column lanes stay inside a wave");



// One launch's blocks: [MLP tile blocks][MLP bias blocks][conv element blocks][bookkeeping].
// Returns true (block-uniform) when this block reduced arena elements.
// rblk / rtid: the reduction block and its thread (grad_reduce_kernel: blockIdx / threadIdx;
// the pipelined / persistent launches: two 256-thread reduction blocks per workgroup).
// SC / rp: fc_tile's (the persistent launch).
template <class Sink, bool SC = false>
__device__ __forceinline__ bool grad_reduce_body(const ReduceArgs& a, Sink& sk, int rblk, int rtid, int rp = 0) {
  const bool mlp = a.hi > OFF_F1W;
  const bool conv = a.lo < OFF_F1W;
  int blk = rblk;
  if (mlp) {
    if (blk < TILE_BLOCKS) {
      const int t = blk * 4 + (rtid >> 6);
      if (t < FC_T0) fc_tile<0, Sink, SC>(t, a, sk, rp);
      else if (t < FC_T0 + FC_T1) fc_tile<1, Sink, SC>(t - FC_T0, a, sk, rp);
      else if (t < FC_TILES) fc_tile<2, Sink, SC>(t - FC_T0 - FC_T1, a, sk, rp);
      return true;
    }
    blk -= TILE_BLOCKS;
    constexpr int FB = (FCB_SLOTS + RT - 1) / RT;
    if (blk < FB) {
      fcb_task<Sink, SC>(blk * RT + rtid, a, sk, rp);
      return true;
    }
    blk -= FB;
  }
  if (conv) {
    constexpr int CB = (CONV_SLOTS + RT - 1) / RT;
    if (blk < CB) { conv_task<Sink, SC>(blk * RT + rtid, a, sk, rp); return true; }
    blk -= CB;
  }
  if (a.bookkeeping && blk == 0 && rtid < 64) bookkeeping(a, rtid);
  return false;
}

constexpr int GRAD_REDUCE_BLOCKS =
    TILE_BLOCKS + (FCB_SLOTS + RT - 1) / RT + (CONV_SLOTS + RT - 1) / RT + 1;
static_assert(GRAD_REDUCE_BLOCKS <= XP_MAX_BLOCKS, "one exchange step counter per reduce block");

__device__ __forceinline__ unsigned long long xp_ld(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Exchange-wait accounting (ReduceArgs::xp_wait, optional): every wave stores the longest wait
// of its lanes for this step (s_memrealtime ticks, 100 MHz) into its own word of the ring entry
// [step % XP_WAIT_RING][block][wave] as {step << 32 | ticks} - a plain store per wave, no
// atomics; the host takes the max over blocks and waves (parallel/xgmi.py wait_stats).
__device__ __forceinline__ void record_wait(const ReduceArgs& a, unsigned step, long long ticks, int rblk, int rtid) {
  if (a.xp_wait == nullptr) return;
  unsigned t = (unsigned)min(ticks, 0xffffffffll);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t = max(t, (unsigned)__shfl_xor((int)t, off));
  if ((rtid & 63) == 0) {
    const int w = rtid >> 6;
    a.xp_wait[((size_t)(step % XP_WAIT_RING) * XP_MAX_BLOCKS + rblk) * (RT / 64) + w] =
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

// WT (the persistent launch): write-through stores of everything the samples of the same launch
// read - an fc1 / fc2 tile through wt_tile_update (the same SGD arithmetic: grad_scale is 1 there,
// so acc * grad_scale is s * xp_scale bit for bit), any other element as sgd_finish<true>.
// F32 (the fp32 persistent launch): every parameter write-through to the fp32 master, the
// momentum and the bf16 shadow plain - the serial exchange's arithmetic, element by element.
template <class Sink>
__device__ __forceinline__ void apply_update(const ReduceArgs& a, const Sink& sk, const float (&s)[4]) {
  constexpr bool WT = Sink::kWT;
  if constexpr (Sink::kF32) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!sk.v[j]) continue;
      float p, m;
      sgd_update(s[j] * a.xp_scale, sk.pv(j), sk.mv(j), a.lr, a.momentum, p, m);
      st_wt(a.master + sk.e[j], p);
      a.mom[sk.e[j]] = m;
      write_shadow(a.shadow, sk.e[j], p);
    }
    return;
  }
  if constexpr (WT) {
    if (sk.tl == 0 || sk.tl == 1) {  // (wave-uniform: one tile per wave)
      f32x4 acc;
      float pv[4], mv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] = s[j] * a.xp_scale;
        pv[j] = sk.v[j] ? sk.pv(j) : 0.f;
        mv[j] = sk.v[j] ? sk.mv(j) : 0.f;
      }
      const int lane = threadIdx.x & 63;
      if (sk.tl == 0) wt_tile_update<0>(acc, pv, mv, sk.e, sk.to0, sk.ti0, lane, a);
      else wt_tile_update<1>(acc, pv, mv, sk.e, sk.to0, sk.ti0, lane, a);
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!sk.v[j]) continue;
    const float gr = s[j] * a.xp_scale;
    float p, m;
    sgd_update(gr, sk.pv(j), sk.mv(j), a.lr, a.momentum, p, m);
    a.mom[sk.e[j]] = m;
    if constexpr (WT) {
      if (is_bias(sk.e[j])) st_wt(a.master + sk.e[j], p);
      else a.master[sk.e[j]] = p;
      write_shadow_wt(a.shadow, sk.e[j], p);
    } else {
      a.master[sk.e[j]] = p;
      write_shadow(a.shadow, sk.e[j], p);
    }
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

// Read every peer rank's granules of this lane's elements (own: this rank's values, kept for
// r == xp_rank) and fold the N values into s in RANK ORDER (s = v0 + v1 + ... in fp32).  RC ranks
// per polling round: the register arrays hold RC ranks' 64-bit loads in flight; RC < NR spends one
// more remote round per chunk to fit a tighter register budget (the fp32 persistent launch runs at
// 128 VGPRs).  Chunks go in ascending rank order, so the additions are exactly one round's.
// Returns the total wait.
template <int NR, int RC, bool PK>
__device__ __forceinline__ long long gather_rank_sum(const ReduceArgs& a, const int (&e)[4], const bool (&vld)[4],
                                                     const float (&own)[4], unsigned step, bool failed, int par,
                                                     float (&s)[4]) {
  static_assert(NR % RC == 0, "whole chunks");
  long long waited = 0;
#pragma unroll
  for (int r0 = 0; r0 < NR; r0 += RC) {
    float v[RC][4];
    unsigned pending = 0;
    const unsigned long long* src[RC];
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int r = r0 + k;
      src[k] = reinterpret_cast<const unsigned long long*>(a.xp_region[r] + a.xp_gslot_off + par * a.xp_gslot_bytes);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[k][j] = own[j];
        if (r < a.xp_nranks && r != a.xp_rank && polled<PK>(vld, j)) pending |= 1u << (4 * k + j);
      }
    }
    waited += poll_granules<RC>(a, src, e, pending, step, failed, v);
#pragma unroll
    for (int k = 0; k < RC; ++k)
      if (r0 + k < a.xp_nranks && r0 + k != a.xp_rank) unpack_pairs<PK>(v[k], vld);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < RC; ++k) {
        const int r = r0 + k;
        if (r == 0) s[j] = v[k][j];
        else if (r < a.xp_nranks) s[j] += v[k][j];
      }
  }
  return waited;
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
template <int NR, class Sink>
__device__ __forceinline__ void xp_exchange(const ReduceArgs& a, Sink& sk, unsigned step, bool failed, int rblk,
                                            int rtid) {
  constexpr bool PK = Sink::kPK;
  constexpr int RC = NR < Sink::kRC ? NR : Sink::kRC;
  const int par = step & 1u;
  pack_pairs<PK>(sk.g, sk.v, sk.e, sk.own, sk.tag);
  float s[4];
  record_wait(a, step, gather_rank_sum<NR, RC, PK>(a, sk.e, sk.v, sk.g, step, failed, par, s), rblk, rtid);
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
template <int NR, class Sink>
__device__ __forceinline__ void xp_exchange_rsag(const ReduceArgs& a, Sink& sk, unsigned step, bool failed, int rblk,
                                                 int rtid) {
  constexpr bool PK = Sink::kPK;
  const int par = step & 1u;
  const int owner = rblk % a.xp_nranks;
  pack_pairs<PK>(sk.g, sk.v, sk.e, sk.own, sk.tag);  // (null own on the owner: rounding only)
  float s[4];
  long long waited;
  if (owner == a.xp_rank) {
    constexpr int RC = NR < Sink::kRC ? NR : Sink::kRC;
    waited = gather_rank_sum<NR, RC, PK>(a, sk.e, sk.v, sk.g, step, failed, par, s);
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
  record_wait(a, step, waited, rblk, rtid);
  apply_update(a, sk, s);
}


// One reduction block's work (rblk, rtid as grad_reduce_body's).  NR = 1: local reduction
// (+ SGD, or gradients out); NR = 2 / 4 / 8: the one-launch exchange for groups of up to NR
// ranks (separate instances keep the local step's registers at its own need).
// Every thread of the workgroup calls it once (it has a workgroup barrier).
template <int NR, bool PK>
__device__ __forceinline__ void reduce_block(const ReduceArgs& a, int rblk, int rtid) {
  if constexpr (NR > 1) {  // one-launch all-reduce: reduce -> exchange -> SGD, per lane
    const int gb = rblk;
    const unsigned step = a.xp_ctr[gb] + 1u;
    const bool failed = *a.xp_err != 0u;
    XpSinkT<PK> sk;
    sk.tag = (unsigned long long)step << 32;
    // pull: every lane's granules go to this rank's slot; two-hop: only non-owners' (the owner
    // publishes the SUM in its ag slot instead)
    const bool publish = (a.xp_mode & 2) == 0 || gb % a.xp_nranks != a.xp_rank;
    sk.own = publish ? reinterpret_cast<unsigned long long*>(a.xp_region[a.xp_rank] + a.xp_gslot_off +
                                                             (step & 1u) * a.xp_gslot_bytes)
                     : nullptr;
    if (grad_reduce_body(a, sk, rblk, rtid)) {
      if ((a.xp_mode & 2) == 0) xp_exchange<NR>(a, sk, step, failed, rblk, rtid);
      else xp_exchange_rsag<NR>(a, sk, step, failed, rblk, rtid);
    }
    __syncthreads();  // every thread read this block's counters before they advance
    if (rtid == 0) a.xp_ctr[gb] = step;
  } else {
    DirectSink d;
    grad_reduce_body(a, d, rblk, rtid);
  }
}


}  // namespace dnn

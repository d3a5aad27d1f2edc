// Device helpers of the persistent launch shared by the bf16 (lenet_fused.hip) and fp32
// (lenet_f32.hip) training kernels: the reduction's block map, the control block layout, the
// generation-relative step tags, the reduction workgroups' row wait and the in-launch bookkeeping.
#pragma once
#include "reduce_device.h"

namespace dnn {

// The whole grad_reduce of one step, block by block (reduce_device.h grad_reduce_body's map).
constexpr int PIPE_MLP_BLOCKS = TILE_BLOCKS + (FCB_SLOTS + RT - 1) / RT;
constexpr int PIPE_CONV_BLOCKS = (CONV_SLOTS + RT - 1) / RT;
constexpr int PIPE_C1_BLOCKS = (SLAB_C2W * SPLIT + RT - 1) / RT;  // conv1 W + b: slab [0, SLAB_C2W)
constexpr int PIPE_C2_BLOCKS = PIPE_CONV_BLOCKS - PIPE_C1_BLOCKS;
constexpr int PIPE_BLOCKS = PIPE_MLP_BLOCKS + PIPE_CONV_BLOCKS + 1;

constexpr int PERS_AROW = 256;  // arrival words per reduction workgroup (max batch)
constexpr int PERS_RROW = 64;   // ready words per sample (one per reduction workgroup)
// control memory: [256 generation words], [batch][PERS_RROW] ready rows, [reduction workgroups]
// [PERS_AROW] arrival words
constexpr int PERS_MAX_GRID = 256;
constexpr long PERS_FLG_OFF = PERS_MAX_GRID * 4;
__host__ __device__ constexpr long pers_arrive_off(int batch) { return (PERS_FLG_OFF + 4L * batch * PERS_RROW + 1023) / 1024 * 1024; }

__device__ __forceinline__ unsigned ld_tag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_tag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool tag_ge(unsigned v, unsigned tgt) { return (int)(v - tgt) >= 0; }  // wrap-safe
__device__ __forceinline__ int ld_sc1(const int32_t* p) {
  return (int)__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt_i(int32_t* p, int v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), (unsigned)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave of a reduction workgroup waits until every sample's arrival word reached tgt
// (bounded: the sticky error word, then no more waits anywhere - never a hang).
__device__ __forceinline__ void pers_wait_rows(const PipeCtl& pc, const unsigned* row, int batch, unsigned tgt,
                                               int lane) {
  if (ld_tag(pc.err) != 0u) return;
  const long long t0 = wall_clock64();
  while (true) {
    bool ok = true;
    for (int b = lane; b < batch; b += 64) ok &= tag_ge(ld_tag(row + b), tgt);
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > pc.timeout_ticks) {
      __hip_atomic_store(pc.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// The bookkeeping of the persistent launch, the same sequence of publications as a PIPE chunk
// of nsteps launches + its closing grad_reduce (engine.py _launch_steps_pipe):
//   t = -1 (launch start, no statistics): cursor + 1, publish slot 1 (step 1's bvalid, step 2's ids);
//   t = 0 .. n - 2 (step t reduced): statistics of step t (bvalid from slot t & 1), cursor + 1,
//     publish slot t & 1 (step t + 2's);
//   t = n - 1: statistics of step n - 1, cursor unchanged, publish slot 0 (the next launch's).
// Loads of anything written inside the launch are sc1 and every store the samples read is
// written through.  batch_ids (the serial layout's "this step's ids") is written at t = n - 1
// only: the fp32 persistent launch's samples read their step-0 ids from it at their start, and a
// launch-start write of step 1's ids there raced with late-starting samples (one in three
// back-to-back launch sequences under load trained on wrong ids: tools/race_hunt.py,
// profiles/r5/fp32_pers_race).  One wave.
__device__ __forceinline__ void bookkeeping_pers(const ReduceArgs& a, const PipeCtl& pc, int lane, int t) {
  const int n = pc.nsteps;
  const bool stats = t >= 0;
  const int adv = t == n - 1 ? 0 : 1;
  const int sin = t < 0 ? 1 : (t & 1);
  const int sout = t < 0 ? 1 : (t == n - 1 ? 0 : (t & 1));
  const int bv = ld_sc1(pc.bv_slot[sin]);  // (before anything is published: sin may be sout)
  float ls = 0.f;
  int cs = 0;
  if (stats) {
    const long r = (long)(t & 1) * a.batch;
    for (int b = lane; b < a.batch; b += 64) {
      ls += ldrow<true>(a.loss + r + b);
      cs += ld_sc1(a.correct + r + b);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) { ls += __shfl_down(ls, off); cs += __shfl_down(cs, off); }
  const int next = ld_sc1(a.state + ST_CURSOR) + adv;
  if (lane == 0 && bv > 0 && stats) {
    a.stats[STAT_LOSS] += (double)ls / (double)bv;
    a.stats[STAT_BATCHES] += 1.0;
    a.stats[STAT_CORRECT] += (double)cs;
    a.stats[STAT_SAMPLES] += (double)bv;
  }
  const long base = (long)next * a.batch;
  for (int b = lane; b < a.batch; b += 64) {
    const long g = base + b;
    if (t == n - 1) a.batch_ids[b] = g < a.order_len ? a.order[g] : 0;
    const long g2 = base + a.batch + b;
    st_wt_i(pc.nid_slot[sout] + b, g2 < a.order_len ? a.order[g2] : -1);
  }
  const long rem = (long)a.order_len - base;
  const int nbv = rem < a.batch ? (rem > 0 ? (int)rem : 0) : a.batch;
  if (lane == 0) {
    st_wt_i(a.state + ST_CURSOR, next);
    st_wt_i(pc.bv_slot[sout], nbv);
  }
}

}  // namespace dnn

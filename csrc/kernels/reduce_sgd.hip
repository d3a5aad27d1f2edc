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



// SGD epilogue with the master/momentum values already in registers (prefetched
// together with the gradient operands, so the update costs no extra memory latency).
__device__ __forceinline__ void sgd_finish(int e, float g, float p_old, float m_old, const ReduceArgs a) {
  g *= a.grad_scale;
  if (a.fuse_sgd) {
    const float m = a.momentum * m_old + g;
    const float p = p_old - a.lr * m;
    a.mom[e] = m;
    a.master[e] = p;
    write_shadow(a.shadow, e, p);
  } else {
    a.grad[e] = g;
  }
}

// fc weight-gradient tiles: dW[o][i] = sum_b z[b][o] * x[b][i]  (K = batch), one 16x16
// output tile per wave on v_mfma_f32_16x16x4_f32 (exact fp32 fma chain, fixed order).
template <int LAYER> struct Fc;
template <> struct Fc<0> { static constexpr int O = 120, I = 400, IT = 25, OFF = OFF_F1W, ZLD = Z1_LD, XLD = A0_LD; };
template <> struct Fc<1> { static constexpr int O = 84, I = 120, IT = 8, OFF = OFF_F2W, ZLD = Z2_LD, XLD = H1_LD; };
template <> struct Fc<2> { static constexpr int O = 10, I = 84, IT = 6, OFF = OFF_F3W, ZLD = Z3_LD, XLD = H2_LD; };
constexpr int FC_T0 = 8 * 25, FC_T1 = 6 * 8, FC_T2 = 1 * 6;
constexpr int FC_TILES = FC_T0 + FC_T1 + FC_T2;   // 254 wave-tiles
constexpr int TILE_BLOCKS = (FC_TILES + 3) / 4;  // 4 waves per block

template <int LAYER>
__device__ __forceinline__ void fc_tile(int t, const ReduceArgs a) {
  using L = Fc<LAYER>;
  const float* z = LAYER == 0 ? a.z1 : (LAYER == 1 ? a.z2 : a.z3);
  const float* x = LAYER == 0 ? a.a0 : (LAYER == 1 ? a.h1 : a.h2);
  const int lane = threadIdx.x & 63;
  const int col = lane & 15, kq = lane >> 4;
  const int o0 = (t / L::IT) * 16, i0 = (t % L::IT) * 16;
  const int om = o0 + col, in = i0 + col;
  const bool ov = om < L::O, iv = in < L::I;
  // this lane's 4 output elements: rows o0 + 4kq + j, column in
  int e[4];
  float pv[4], mv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = min(o0 + 4 * kq + j, L::O - 1);
    e[j] = L::OFF + o * L::I + (iv ? in : 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) { pv[j] = a.master[e[j]]; mv[j] = a.mom[e[j]]; }  // (unused if !fuse_sgd)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int omc = ov ? om : 0, inc = iv ? in : 0;
  for (int b0 = 0; b0 < a.batch; b0 += 64) {
    // every operand load is unconditional (clamped address) and issued before the first
    // MFMA; out-of-range operands are zeroed by a select afterwards
    float av[16], bv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int b = min(b0 + 4 * s + kq, a.batch - 1);
      av[s] = z[(size_t)b * L::ZLD + omc];
      bv[s] = x[(size_t)b * L::XLD + inc];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool bvld = b0 + 4 * s + kq < a.batch;
      av[s] = (bvld && ov) ? av[s] : 0.f;
      bv[s] = (bvld && iv) ? bv[s] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = o0 + 4 * kq + j;
    if (o < L::O && iv) sgd_finish(e[j], acc[j], pv[j], mv[j], a);
  }
}

// element tasks: fc biases (sum_b z[b][o]) and conv slab columns (sum_b slab[b][j]);
// all 64 rows of a chunk are loaded before the (fixed-order) sum
constexpr int FCB_ELEMS = 120 + 84 + 10;
constexpr int CONV_ELEMS = SLAB;
__device__ __forceinline__ void elem_task(int e, bool mlp_part, const ReduceArgs a) {
  const float* src;
  int ld, col, dst;
  if (mlp_part) {
    if (e >= FCB_ELEMS) return;
    if (e < 120) { src = a.z1; ld = Z1_LD; col = e; dst = OFF_F1B + e; }
    else if (e < 204) { src = a.z2; ld = Z2_LD; col = e - 120; dst = OFF_F2B + e - 120; }
    else { src = a.z3; ld = Z3_LD; col = e - 204; dst = OFF_F3B + e - 204; }
  } else {
    if (e >= CONV_ELEMS) return;
    src = a.slab; ld = SLAB; col = e;
    if (e < SLAB_C1B) dst = OFF_C1W + e;
    else if (e < SLAB_C2W) dst = OFF_C1B + (e - SLAB_C1B);
    else if (e < SLAB_C2B) dst = OFF_C2W + (e - SLAB_C2W);
    else dst = OFF_C2B + (e - SLAB_C2B);
  }
  const float pv = a.master[dst], mv = a.mom[dst];  // (unused if !fuse_sgd)
  float g = 0.f;
  for (int b0 = 0; b0 < a.batch; b0 += 64) {
    float v[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] = src[(size_t)min(b0 + k, a.batch - 1) * ld + col];
#pragma unroll
    for (int k = 0; k < 64; ++k) g += (b0 + k < a.batch) ? v[k] : 0.f;
  }
  sgd_finish(dst, g, pv, mv, a);
}

__global__ void __launch_bounds__(RT) __attribute__((amdgpu_waves_per_eu(1, 2))) grad_reduce_kernel(ReduceArgs a) {
  // block roles: [MLP tile blocks][MLP bias block][conv element blocks][bookkeeping]
  const bool mlp = a.hi > OFF_F1W;
  const bool conv = a.lo < OFF_F1W;
  int blk = blockIdx.x;
  if (mlp) {
    if (blk < TILE_BLOCKS) {
      const int t = blk * 4 + (threadIdx.x >> 6);
      if (t < FC_T0) fc_tile<0>(t, a);
      else if (t < FC_T0 + FC_T1) fc_tile<1>(t - FC_T0, a);
      else if (t < FC_TILES) fc_tile<2>(t - FC_T0 - FC_T1, a);
      return;
    }
    blk -= TILE_BLOCKS;
    if (blk < 1) { elem_task(threadIdx.x, true, a); return; }
    blk -= 1;
  }
  if (conv) {
    constexpr int CB = (CONV_ELEMS + RT - 1) / RT;
    if (blk < CB) { elem_task(blk * RT + threadIdx.x, false, a); return; }
    blk -= CB;
  }
  if (a.bookkeeping && blk == 0 && threadIdx.x < 64) {
    // (1) epoch statistics of the step that just ran (one wave, fixed order)
    const int lane = threadIdx.x;
    float ls = 0.f;
    int cs = 0;
    for (int b = lane; b < a.batch; b += 64) { ls += a.loss[b]; cs += a.correct[b]; }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) { ls += __shfl_down(ls, off); cs += __shfl_down(cs, off); }
    const int bv = a.state[ST_BVALID];
    const int next = a.state[ST_CURSOR] + 1;
    if (lane == 0 && bv > 0) {
      a.stats[STAT_LOSS] += (double)ls / (double)bv;
      a.stats[STAT_BATCHES] += 1.0;
      a.stats[STAT_CORRECT] += (double)cs;
      a.stats[STAT_SAMPLES] += (double)bv;
    }
    // (2) publish the NEXT step: cursor, valid count and its sample ids, so the next
    //     fused kernel reads its sample id directly (no cursor -> order dependency)
    const long base = (long)next * a.batch;
    for (int b = lane; b < a.batch; b += 64) {
      const long g = base + b;
      a.batch_ids[b] = g < a.order_len ? a.order[g] : 0;
    }
    const long rem = (long)a.order_len - base;
    const int nbv = rem < a.batch ? (rem > 0 ? (int)rem : 0) : a.batch;
    if (lane == 0) {
      a.state[ST_CURSOR] = next;
      a.state[ST_BVALID] = nbv;
    }
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
    write_shadow(shadow, e, p);
  }
}

// ---- host launchers ---------------------------------------------------------------------
void launch_grad_reduce(const ReduceArgs& args, hipStream_t stream) {
  const bool mlp = args.hi > OFF_F1W;
  const bool conv = args.lo < OFF_F1W;
  int nblk = 0;
  if (mlp) nblk += TILE_BLOCKS + 1;
  if (conv) nblk += (CONV_ELEMS + RT - 1) / RT;
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

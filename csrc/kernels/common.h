// Shared definitions for the gfx950 (CDNA4) kernels of the LeNet/CIFAR-10 engine.
//
// Layout contract with python (distributed_neural_network_amd/models/network.py,
// ArenaLayout): every parameter lives in one flat fp32 arena, each tensor on a
// 64-element (256 B) boundary, in reference state_dict order
// (reference models/model.py:13-18).  ops/native.py asserts these constants
// against ArenaLayout at import time.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace dnn {

// ---- arena offsets (fp32 elements) -------------------------------------------------
constexpr int OFF_C1W = 0;      // [6][3][5][5]   450
constexpr int OFF_C1B = 512;    // [6]
constexpr int OFF_C2W = 576;    // [16][6][5][5] 2400
constexpr int OFF_C2B = 3008;   // [16]
constexpr int OFF_F1W = 3072;   // [120][400]   48000
constexpr int OFF_F1B = 51072;  // [120]
constexpr int OFF_F2W = 51200;  // [84][120]    10080
constexpr int OFF_F2B = 61312;  // [84]
constexpr int OFF_F3W = 61440;  // [10][84]       840
constexpr int OFF_F3B = 62336;  // [10]
constexpr int ARENA = 62400;    // padded length
constexpr int NUM_PARAMS = 62006;

// ---- per-sample conv weight-gradient slab (fp32) -----------------------------------
// [dW1 450][db1 6][dW2 2400][db2 16]
constexpr int SLAB_C1W = 0;
constexpr int SLAB_C1B = 450;
constexpr int SLAB_C2W = 456;
constexpr int SLAB_C2B = 2856;
constexpr int SLAB = 2872;

// ---- per-sample activation rows written by the fused kernel --------------------------
constexpr int A0_LD = 400;  // pooled conv2 output (fc1 input)
constexpr int H1_LD = 120;  // relu(fc1)
constexpr int H2_LD = 84;   // relu(fc2)
constexpr int Z1_LD = 120;  // dL/d(fc1 pre-activation)
constexpr int Z2_LD = 84;   // dL/d(fc2 pre-activation)
constexpr int Z3_LD = 16;   // dL/dlogits (10 used)
constexpr int IMG = 3 * 32 * 32;

// ---- bf16 shadow buffer: [plain copy of the arena | kernel-ready weight images] -------
// Written by the optimizer kernels right after each update (one owner thread per
// parameter writes its bf16 value to every position it occupies), so the fused kernel
// loads MFMA fragments with one 16-B load each instead of re-arranging weights per sample.
constexpr int SH_W1F = ARENA;               // conv1 fwd B frags  [16 pairs (c,ky)][16 n' = 2 o + s][8 j]: W[o][c][ky][j - s]
constexpr int SH_W2F = SH_W1F + 16 * 16 * 8;  // conv2 fwd B frags  [32 pairs (c,ky)][16 n][8 kx]
constexpr int SH_WF = SH_W2F + 32 * 16 * 8;   // conv2 dgrad B frags (flipped) [80 (ky',o)][16 c][8 kx']
constexpr int SH_W2T = SH_WF + 80 * 16 * 8;   // fc2 transposed [120 i][96 o]
constexpr int SH_W3T = SH_W2T + 120 * 96;     // fc3 transposed [84 i][16 o]
constexpr int SH_TOTAL = SH_W3T + 84 * 16 + 64;  // + slack so padded fragment reads stay in bounds

// bf16 gradient granules (the xGMI exchanges' bf16 option): round-to-nearest-even bits, and
// a pair {lo | hi << 16} back to the two floats
__device__ __forceinline__ unsigned bf16_bits(float f) {
  const unsigned u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_lo(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(unsigned w) { return __uint_as_float(w & 0xffff0000u); }

__device__ __forceinline__ void write_shadow(bf16* __restrict__ sh, int e, float p) {
  const bf16 v = (bf16)p;
  sh[e] = v;
  if (e >= OFF_C1W && e < OFF_C1W + 450) {
    const int r = e - OFF_C1W, n = r / 75, rem = r - 75 * n, c = rem / 25, ky = (rem % 25) / 5, kx = rem % 5;
    sh[SH_W1F + ((c * 5 + ky) * 16 + 2 * n) * 8 + kx] = v;  // shift 0 (lenet_fused.hip phase B: pixel pairs)
    sh[SH_W1F + ((c * 5 + ky) * 16 + 2 * n + 1) * 8 + kx + 1] = v;  // shift 1
  } else if (e >= OFF_C2W && e < OFF_C2W + 2400) {
    const int r = e - OFF_C2W, n = r / 150, rem = r - 150 * n, c = rem / 25, ky = (rem % 25) / 5, kx = rem % 5;
    sh[SH_W2F + ((c * 5 + ky) * 16 + n) * 8 + kx] = v;
    sh[SH_WF + (((4 - ky) * 16 + n) * 16 + c) * 8 + (4 - kx)] = v;  // K pairs kyp-major: p = 16 kyp + o
  } else if (e >= OFF_F2W && e < OFF_F2W + 10080) {
    const int r = e - OFF_F2W, o = r / 120, i = r - 120 * o;
    sh[SH_W2T + i * 96 + o] = v;
  } else if (e >= OFF_F3W && e < OFF_F3W + 840) {
    const int r = e - OFF_F3W, o = r / 84, i = r - 84 * o;
    sh[SH_W3T + i * 16 + o] = v;
  }
}

// momentum SGD (torch.optim.SGD, dampening 0): m <- momentum * m + g; p <- p - lr * m.
// Both steps are explicit fmas, so every kernel that applies the update (batch reduction,
// xGMI all-reduce, one-launch exchange) rounds identically and replicas stay bit-identical
// whichever path produced them.
__device__ __forceinline__ void sgd_update(float g, float p_old, float m_old, float lr, float momentum, float& p,
                                           float& m) {
  m = __builtin_fmaf(momentum, m_old, g);
  p = __builtin_fmaf(-lr, m, p_old);
}

// ---- device step state (int32 words) -------------------------------------------------
// [0] cursor: step index within the epoch (advanced by the reduce kernel)
// [1] bvalid: valid samples of the current batch (written by the fused kernel)
constexpr int ST_CURSOR = 0;
constexpr int ST_BVALID = 1;
// device stats (fp64): [0] sum of batch-mean losses, [1] batches, [2] correct, [3] samples
constexpr int STAT_LOSS = 0, STAT_BATCHES = 1, STAT_CORRECT = 2, STAT_SAMPLES = 3;

// Cross-lane reductions on DPP (VALU lane permutes, a few cycles) instead of __shfl_xor (a
// ds_bpermute through the LDS unit, ~100+ cycles of latency per dependent step).  Pairings:
// quad_perm [1,0,3,2] = xor 1, [2,3,0,1] = xor 2, row_half_mirror (i <-> 7 - i in each 8) and
// row_mirror (i <-> 15 - i in each 16).  After the quad steps every lane of a quad holds the
// bit-identical quad total, so pairing by mirror instead of xor 4 / xor 8 gives bit-identical
// sums (fp32 + is commutative), and every lane of the group ends with the same value.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
constexpr int DPP_XOR1 = 0xb1, DPP_XOR2 = 0x4e, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
__device__ __forceinline__ float sum4(float v) {
  v += dppf<DPP_XOR1>(v);
  return v + dppf<DPP_XOR2>(v);
}
__device__ __forceinline__ float sum8(float v) {
  v = sum4(v);
  return v + dppf<DPP_HALF_MIRROR>(v);
}
__device__ __forceinline__ float sum16(float v) {
  v = sum8(v);
  return v + dppf<DPP_MIRROR>(v);
}
__device__ __forceinline__ float max16(float v) {
  v = fmaxf(v, dppf<DPP_XOR1>(v));
  v = fmaxf(v, dppf<DPP_XOR2>(v));
  v = fmaxf(v, dppf<DPP_HALF_MIRROR>(v));
  return fmaxf(v, dppf<DPP_MIRROR>(v));
}
__device__ __forceinline__ int min16(int v) {
  v = min(v, dppi<DPP_XOR1>(v));
  v = min(v, dppi<DPP_XOR2>(v));
  v = min(v, dppi<DPP_HALF_MIRROR>(v));
  return min(v, dppi<DPP_MIRROR>(v));
}

}  // namespace dnn

#define HIP_CHECK(x)                                                                      \
  do {                                                                                    \
    hipError_t err__ = (x);                                                               \
    if (err__ != hipSuccess) {                                                            \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(err__) +    \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));       \
    }                                                                                     \
  } while (0)

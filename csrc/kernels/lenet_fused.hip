// Fused per-sample forward + data-backward + conv weight-gradient kernel (gfx950).
//
// Capability parity: one workgroup runs, for ONE CIFAR image, everything the
// reference's hot loop does per sample in
//   data_parallelism_train.py:195-198  (forward, CrossEntropy, backward)
// i.e. ATen conv/relu/maxpool/addmm/log_softmax/nll + their backward ops
// (SURVEY.md §2.5 K0..K18), plus the ToTensor/Normalize ingest
// (data_parallelism_train.py:24-27).  Weight gradients that need a reduction over
// the batch are NOT finished here: conv weight grads are written as a per-sample
// fp32 slab and fc weight grads as per-sample (activation, delta) rows; the
// grad_reduce kernel sums them in a fixed order (bitwise deterministic, no atomics).
//
// MI355X design:
//  * one workgroup = one sample = 8 waves (512 threads); every intermediate stays
//    in LDS (160 KB budget laid out below), HBM sees the u8 image, the bf16 weights
//    and the small per-sample output rows only.
//  * conv fwd, conv wgrad and conv dgrad run on MFMA (v_mfma_f32_16x16x32_bf16 /
//    16x16x16bf16_1k, f32 accumulate).  The im2col gather is removed by "window
//    records": rec[c][y][x] = X[c][y][x..x+7] (16 B, bf16).  Ordering K as
//    (c, ky, kx<8) makes every A/B fragment ONE aligned ds_read_b128, for the
//    forward (8 kx per lane) AND for the weight gradient (8 consecutive pixels per
//    lane).
//  * ReLU + 2x2 maxpool are fused into the MFMA epilogue: each 16-row M-tile is 4
//    pooling windows x 4 pixels, so a lane's 4 accumulator rows ARE one window.
//    The argmax is kept as a 2-bit code (4 = no gradient, i.e. max <= 0), which
//    replaces both max_pool2d_with_indices and threshold_backward.
//  * conv2 dgrad is an MFMA col2im (dCols = dY2^T W2) followed by a deterministic
//    gather-sum, not float atomics.
#include "launchers.h"

namespace dnn {

constexpr int NT = 512;

// ---- LDS map (bytes) ----------------------------------------------------------------
constexpr int L_REGA = 0;          // fc1 bf16 [120][400] | dCols/DY2/DY2T/DP1 | dY1
constexpr int L_REGA_SZ = 96256;
constexpr int L_REGB = L_REGA + L_REGA_SZ;  // R1 records [3][32][29] | R2 records [6][14][13]
constexpr int L_REGB_SZ = 44544;
constexpr int L_P1 = L_REGB + L_REGB_SZ;    // f32 [6][14][20] (cols 14..19 zero)
constexpr int L_CODE1 = L_P1 + 6720;        // u8 [6][196]
constexpr int L_A0 = L_CODE1 + 1184;        // f32 [400]
constexpr int L_CODE2 = L_A0 + 1600;        // u8 [400]
constexpr int L_H1 = L_CODE2 + 400;         // f32 [128]
constexpr int L_H2 = L_H1 + 512;            // f32 [96]
constexpr int L_LOG = L_H2 + 384;           // f32 [16]
constexpr int L_DZ3 = L_LOG + 64;           // f32 [16]
constexpr int L_DZ2 = L_DZ3 + 64;           // f32 [96]
constexpr int L_DZ1 = L_DZ2 + 384;          // f32 [128]
constexpr int L_DA0 = L_DZ1 + 512;          // f32 [400]
constexpr int L_W1S = L_DA0 + 1600;         // bf16 [6][75] (+pad)
constexpr int L_W2S = L_W1S + 912;          // bf16 [16][150]
constexpr int L_IMG = L_W2S + 4800;         // u8 [3][32][32] raw image (re-used by phase F)
constexpr int L_MISC = L_IMG + 3072;        // scalars
constexpr int LDS_TOTAL = L_MISC + 64;      // 163,072 B
static_assert(LDS_TOTAL <= 163840, "LDS budget");

// REGA sub-layout during the conv backward
constexpr int DCOLS_LD = 164;               // f32 row stride of dCols [112][164]
constexpr int A_DCOLS = 0;                  // 73,472
constexpr int A_DY2 = 73472;                // bf16 [16][10][16]   5,120
constexpr int A_DY2T = A_DY2 + 5120;        // bf16 [112][16]      3,584
constexpr int A_DP1 = A_DY2T + 3584;        // f32 [6][196]        4,704
constexpr int A_DY1 = 0;                    // bf16 [6][28][32]   10,752 (after dCols is dead)
static_assert(A_DP1 + 4704 <= L_REGA_SZ, "REGA sub-layout");

__device__ __forceinline__ float u8norm(uint32_t u) {
  // ToTensor (x/255) then Normalize(mean .5, std .5): same op order as torchvision.
  return ((float)u / 255.0f - 0.5f) / 0.5f;
}

// Barrier for LDS hand-offs only: waits for this wave's LDS ops, not for vmcnt, so an
// in-flight LDS-DMA (global_load_lds) keeps streaming across it.  __syncthreads()
// would emit s_waitcnt vmcnt(0) and drain the DMA.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One LDS-DMA wave-instruction: 64 lanes x 16 B from per-lane global addresses into
// LDS [lds_base, lds_base + 1 KB).  Inline asm on purpose: hipcc's waitcnt pass does
// not see it, so it neither drains it at unrelated ds_reads (it cannot disprove LDS
// aliasing inside the single dynamic LDS array) nor at later plain-load uses.  The
// caller owns completion: s_waitcnt vmcnt(0) + a barrier before reading the bytes,
// and every plain global load issued before a DMA is consumed before the DMA.
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
}

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ short bf16_bits(float f) {
  bf16 h = (bf16)f;
  return __builtin_bit_cast(short, h);
}

// Build the 29 window records of one input row (c, y) from the u8 image staged in LDS.
__device__ __forceinline__ void build_r1_row(const uint8_t* img, bf16x8* R1, int row) {
  const uint4* src = reinterpret_cast<const uint4*>(img + row * 32);
  uint4 lo = src[0], hi = src[1];
  uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  float v[40];
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k] = u8norm((w[k >> 2] >> (8 * (k & 3))) & 0xffu);
#pragma unroll
  for (int k = 32; k < 40; ++k) v[k] = 0.f;
#pragma unroll
  for (int x = 0; x < 29; ++x) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)v[x + j];
    R1[row * 29 + x] = r;
  }
}

template <bool TRAIN>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 2))) lenet_fused_kernel(
    const uint8_t* __restrict__ images,   // [N][3][32][32] u8 (CIFAR binary order)
    const int32_t* __restrict__ labels,   // [N]
    const int32_t* __restrict__ order,    // [order_len] sample ids (nullptr: identity)
    int order_len, int batch, int base_index,
    int32_t* __restrict__ state,          // TRAIN: cursor/bvalid words
    const float* __restrict__ master,     // fp32 arena (biases)
    const bf16* __restrict__ shadow,      // bf16 arena (weights)
    float* __restrict__ a0_out, float* __restrict__ h1_out, float* __restrict__ h2_out,
    float* __restrict__ z1_out, float* __restrict__ z2_out, float* __restrict__ z3_out,
    float* __restrict__ slab_out, float* __restrict__ loss_out, int32_t* __restrict__ correct_out,
    long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // diagnostic phase timeline (block 0, thread 0): s_memrealtime ticks (100 MHz)
  const bool stamp = stamps != nullptr && blockIdx.x == 0 && threadIdx.x == 0;
#define STAMP(i) do { if (stamp) stamps[i] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
  STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int b = blockIdx.x;

  long gidx;
  int bvalid = 1;
  if (TRAIN) {
    const int cursor = state[ST_CURSOR];
    gidx = (long)cursor * batch + b;
    long rem = (long)order_len - (long)cursor * batch;
    bvalid = rem < batch ? (rem > 0 ? (int)rem : 0) : batch;
    if (b == 0 && tid == 0) state[ST_BVALID] = bvalid;
  } else {
    gidx = (long)base_index + b;
  }
  const bool valid = gidx < order_len;
  if (!valid) {
    if (TRAIN) {
      for (int i = tid; i < A0_LD; i += NT) a0_out[(size_t)b * A0_LD + i] = 0.f;
      for (int i = tid; i < H1_LD; i += NT) { h1_out[(size_t)b * H1_LD + i] = 0.f; z1_out[(size_t)b * Z1_LD + i] = 0.f; }
      for (int i = tid; i < H2_LD; i += NT) { h2_out[(size_t)b * H2_LD + i] = 0.f; z2_out[(size_t)b * Z2_LD + i] = 0.f; }
      for (int i = tid; i < Z3_LD; i += NT) z3_out[(size_t)b * Z3_LD + i] = 0.f;
      for (int i = tid; i < SLAB; i += NT) slab_out[(size_t)b * SLAB + i] = 0.f;
      if (tid == 0) { loss_out[b] = 0.f; correct_out[b] = 0; }
    }
    return;
  }
  const int sample = order ? order[gidx] : (int)gidx;
  const int label = labels[sample];
  const uint8_t* img = images + (size_t)sample * IMG;

  bf16* fc1s = reinterpret_cast<bf16*>(smem + L_REGA);
  bf16x8* R1 = reinterpret_cast<bf16x8*>(smem + L_REGB);
  bf16x8* R2 = reinterpret_cast<bf16x8*>(smem + L_REGB);
  float* P1 = reinterpret_cast<float*>(smem + L_P1);
  uint8_t* CODE1 = smem + L_CODE1;
  float* A0 = reinterpret_cast<float*>(smem + L_A0);
  uint8_t* CODE2 = smem + L_CODE2;
  float* H1 = reinterpret_cast<float*>(smem + L_H1);
  float* H2 = reinterpret_cast<float*>(smem + L_H2);
  float* LOG = reinterpret_cast<float*>(smem + L_LOG);
  float* DZ3 = reinterpret_cast<float*>(smem + L_DZ3);
  float* DZ2 = reinterpret_cast<float*>(smem + L_DZ2);
  float* DZ1 = reinterpret_cast<float*>(smem + L_DZ1);
  float* DA0 = reinterpret_cast<float*>(smem + L_DA0);
  bf16* W1S = reinterpret_cast<bf16*>(smem + L_W1S);
  bf16* W2S = reinterpret_cast<bf16*>(smem + L_W2S);

  // ============ phase A: ingest + weight staging ======================================
  // Loads are issued before any is consumed, in order of use: image + conv weights and
  // biases (needed now), then fc1 (96 KB) by LDS-DMA straight into its LDS region; the
  // DMA stays in flight through both convolutions (phases B-C synchronise with
  // LDS-only barriers, which do not drain vmcnt) and is waited for before phase D.
  uint8_t* IMGS = smem + L_IMG;
  const uint4 im = reinterpret_cast<const uint4*>(img)[min(tid, 191)];
  const uint4 w1v = reinterpret_cast<const uint4*>(shadow + OFF_C1W)[min(tid, 56)];  // 450 bf16 + zero pad
  const uint4 w2v = reinterpret_cast<const uint4*>(shadow + OFF_C2W)[max(tid - 212, 0)];
  const float bias_c1 = master[OFF_C1B + min(lane & 15, 5)];
  const float bias_c2 = master[OFF_C2B + (lane & 15)];
  for (int i = tid; i < 6 * 14 * 20; i += NT) P1[i] = 0.f;
  if (tid < 192) reinterpret_cast<uint4*>(IMGS)[tid] = im;
  if (tid < 57) reinterpret_cast<uint4*>(smem + L_W1S)[tid] = w1v;
  if (tid >= 212) reinterpret_cast<uint4*>(smem + L_W2S)[tid - 212] = w2v;
  // (hipcc waits vmcnt(0) for a plain load consumed while an LDS-DMA is in flight, so the
  //  loads above are consumed first and the DMA is issued after them)
  float bc1 = bias_c1, bc2 = bias_c2;
  asm volatile("" : "+v"(bc1), "+v"(bc2));  // consume (wait for) the bias loads before the DMA
  {
    // 94 wave-instructions x 1 KB = 96,256 B (fc1 + the head of fc1.bias, all in-arena).
    // 12 per wave with the index clamped: a duplicate copies identical bytes.
    const uint4* f1src = reinterpret_cast<const uint4*>(shadow + OFF_F1W);
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem + L_REGA));
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const int i = min(wave + 8 * k, 93);
      dma16(f1src + i * 64 + lane, base + (uint32_t)__builtin_amdgcn_readfirstlane(i) * 1024u);
    }
  }
  lds_barrier();
  if (tid < 96) build_r1_row(IMGS, R1, tid);
  lds_barrier();
  STAMP(1);

  const int fr = lane & 15;   // MFMA fragment row/col within the 16-tile
  const int fg = lane >> 4;   // MFMA k-group (0..3)

  // ============ phase B: conv1 (3->6, 5x5) + bias + ReLU + maxpool, MFMA ================
  {
    bf16x8 bw[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int pr = 4 * s + fg;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        bw[s][j] = (fr < 6 && pr < 15 && j < 5) ? W1S[fr * 75 + pr * 5 + j] : (bf16)0.f;
    }
    const float bias = fr < 6 ? bc1 : 0.f;
    const int wi = fr >> 2, pi = fr & 3;  // A-operand row -> (window, pixel)
    for (int t = wave; t < 49; t += 8) {
      const int q = 4 * t + wi;
      const int y = 2 * (q / 14) + (pi >> 1), x = 2 * (q % 14) + (pi & 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int pr = 4 * s + fg;
        bf16x8 a;
        if (pr < 15) {
          const int c = pr / 5, ky = pr % 5;
          a = R1[(c * 32 + y + ky) * 29 + x];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = (bf16)0.f;
        }
        acc = mfma32(a, bw[s], acc);
      }
      if (fr < 6) {  // lane holds window fg of tile t for channel fr
        const int qo = 4 * t + fg;
        float best = acc[0] + bias;
        int arg = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i) {
          const float v = acc[i] + bias;
          if (v > best) { best = v; arg = i; }
        }
        P1[(fr * 14 + qo / 14) * 20 + qo % 14] = fmaxf(best, 0.f);
        CODE1[fr * 196 + qo] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
      }
    }
  }
  lds_barrier();

  STAMP(2);
  // ============ phase C: conv2 (6->16, 5x5) + bias + ReLU + maxpool, MFMA ===============
  // MLP operands each lane needs in phase D, loaded now so conv2 hides their latency.
  const int mo = tid >> 2, mp = tid & 3;   // MLP lane roles: output (or input) index, quarter
  bf16x8 w2f[4];                           // fc2 forward: row mo, chunks mp + 4k
#pragma unroll
  for (int k = 0; k < 4; ++k)
    w2f[k] = reinterpret_cast<const bf16x8*>(shadow + OFF_F2W + min(mo, 83) * 120)[min(mp + 4 * k, 14)];
  bf16x4 w3f[6];                           // fc3 forward: row mo, chunks mp + 4k
#pragma unroll
  for (int k = 0; k < 6; ++k)
    w3f[k] = reinterpret_cast<const bf16x4*>(shadow + OFF_F3W + min(mo, 9) * 84)[min(mp + 4 * k, 20)];
  bf16 w3d[10];                            // fc3 dgrad: column tid
#pragma unroll
  for (int o = 0; o < 10; ++o) w3d[o] = shadow[OFF_F3W + o * 84 + min(tid, 83)];
  bf16 w2d[21];                            // fc2 dgrad: column mo, rows mp*21 + k
#pragma unroll
  for (int k = 0; k < 21; ++k) w2d[k] = shadow[OFF_F2W + (mp * 21 + k) * 120 + min(mo, 119)];
  const float bias_f1 = master[OFF_F1B + min(mo, 119)];
  const float bias_f2 = master[OFF_F2B + min(mo, 83)];
  const float bias_f3 = master[OFF_F3B + min(mo, 9)];
  if (tid < 84) {  // window records of P1 rows (overwrite R1: dead until phase F)
    const int row = tid;  // c*14 + y
    float v[20];
#pragma unroll
    for (int k = 0; k < 20; ++k) v[k] = P1[row * 20 + k];
#pragma unroll
    for (int x = 0; x < 13; ++x) {
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = (bf16)v[x + j];
      R2[row * 13 + x] = r;
    }
  }
  lds_barrier();
  if (wave < 7) {
    const int t = wave;
    const int wi = fr >> 2, pi = fr & 3;
    int q = 4 * t + wi;
    if (q > 24) q = 24;  // padding windows of the last tile: computed, discarded
    const int y = 2 * (q / 5) + (pi >> 1), x = 2 * (q % 5) + (pi & 1);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int pr = 4 * s + fg;
      bf16x8 a, bw;
      if (pr < 30) {
        const int c = pr / 5, ky = pr % 5;
        a = R2[(c * 14 + y + ky) * 13 + x];
#pragma unroll
        for (int j = 0; j < 8; ++j) bw[j] = j < 5 ? W2S[fr * 150 + pr * 5 + j] : (bf16)0.f;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = (bf16)0.f; bw[j] = (bf16)0.f; }
      }
      acc = mfma32(a, bw, acc);
    }
    const int qo = 4 * t + fg;
    if (qo < 25) {
      const float bias = bc2;
      float best = acc[0] + bias;
      int arg = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        const float v = acc[i] + bias;
        if (v > best) { best = v; arg = i; }
      }
      A0[fr * 25 + qo] = fmaxf(best, 0.f);  // torch.flatten order [16][5][5]
      CODE2[fr * 25 + qo] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // fc1 LDS-DMA (and MLP prefetch) landed
  __syncthreads();

  STAMP(3);
  // ============ phase D: MLP forward, cross-entropy, MLP data-backward ==================
  {  // fc1: 120 x 400, 4 lanes per output
    const int o = tid >> 2, p = tid & 3;
    float acc = 0.f;
    if (o < 120) {
      const bf16x8* wrow = reinterpret_cast<const bf16x8*>(fc1s + o * 400);
      for (int c8 = p; c8 < 50; c8 += 4) {
        const bf16x8 w = wrow[c8];
        const float4 xa = reinterpret_cast<const float4*>(A0)[2 * c8];
        const float4 xb = reinterpret_cast<const float4*>(A0)[2 * c8 + 1];
        acc += (float)w[0] * xa.x + (float)w[1] * xa.y + (float)w[2] * xa.z + (float)w[3] * xa.w +
               (float)w[4] * xb.x + (float)w[5] * xb.y + (float)w[6] * xb.z + (float)w[7] * xb.w;
      }
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (o < 120 && p == 0) H1[o] = fmaxf(acc + bias_f1, 0.f);
  }
  __syncthreads();
  {  // fc2: 84 x 120 (prefetched fragments)
    float acc = 0.f;
    if (mo < 84) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c8 = mp + 4 * k;
        if (c8 < 15) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += (float)w2f[k][j] * H1[c8 * 8 + j];
        }
      }
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (mo < 84 && mp == 0) H2[mo] = fmaxf(acc + bias_f2, 0.f);
  }
  __syncthreads();
  {  // fc3: 10 x 84 (prefetched fragments)
    float acc = 0.f;
    if (mo < 10) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int c4 = mp + 4 * k;
        if (c4 < 21) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc += (float)w3f[k][j] * H2[c4 * 4 + j];
        }
      }
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (mo < 10 && mp == 0) LOG[mo] = acc + bias_f3;
  }
  __syncthreads();
  if (tid == 0) {  // CrossEntropy (mean over the valid batch) + accuracy
    float mx = LOG[0];
    int pred = 0;
#pragma unroll
    for (int o = 1; o < 10; ++o) if (LOG[o] > mx) { mx = LOG[o]; pred = o; }
    float e[10], sum = 0.f;
#pragma unroll
    for (int o = 0; o < 10; ++o) { e[o] = expf(LOG[o] - mx); sum += e[o]; }
    const float lse = mx + logf(sum);
    loss_out[b] = lse - LOG[label];
    correct_out[b] = pred == label ? 1 : 0;
    if (TRAIN) {
      const float inv = 1.0f / (float)bvalid;
      const float rs = 1.0f / sum;
#pragma unroll
      for (int o = 0; o < 16; ++o) DZ3[o] = o < 10 ? (e[o] * rs - (o == label ? 1.f : 0.f)) * inv : 0.f;
    }
  }
  if (!TRAIN) return;
  __syncthreads();
  STAMP(4);
  if (tid < 84) {  // fc3 dgrad + ReLU mask (prefetched column)
    float acc = 0.f;
#pragma unroll
    for (int o = 0; o < 10; ++o) acc += DZ3[o] * (float)w3d[o];
    DZ2[tid] = H2[tid] > 0.f ? acc : 0.f;
  }
  __syncthreads();
  {  // fc2 dgrad + ReLU mask: 4 lanes per input, 21 prefetched rows each
    float acc = 0.f;
    if (mo < 120) {
#pragma unroll
      for (int k = 0; k < 21; ++k) acc += DZ2[mp * 21 + k] * (float)w2d[k];
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (mo < 120 && mp == 0) DZ1[mo] = H1[mo] > 0.f ? acc : 0.f;
  }
  __syncthreads();
  if (tid < 400) {  // fc1 dgrad (mask applied through CODE2 below)
    float acc = 0.f;
#pragma unroll 8
    for (int o = 0; o < 120; ++o) acc += DZ1[o] * (float)fc1s[o * 400 + tid];
    DA0[tid] = acc;
  }
  // per-sample rows for the batch-reduced fc weight gradients
  for (int i = tid; i < A0_LD; i += NT) a0_out[(size_t)b * A0_LD + i] = A0[i];
  if (tid < H1_LD) { h1_out[(size_t)b * H1_LD + tid] = H1[tid]; z1_out[(size_t)b * Z1_LD + tid] = DZ1[tid]; }
  if (tid < H2_LD) { h2_out[(size_t)b * H2_LD + tid] = H2[tid]; z2_out[(size_t)b * Z2_LD + tid] = DZ2[tid]; }
  if (tid < Z3_LD) z3_out[(size_t)b * Z3_LD + tid] = DZ3[tid];
  __syncthreads();

  STAMP(5);
  // ============ phase E: conv2 backward =================================================
  float* slab = slab_out + (size_t)b * SLAB;
  bf16* DY2 = reinterpret_cast<bf16*>(smem + L_REGA + A_DY2);     // [16][10][16]
  bf16* DY2T = reinterpret_cast<bf16*>(smem + L_REGA + A_DY2T);   // [112][16]
  float* DCOLS = reinterpret_cast<float*>(smem + L_REGA + A_DCOLS);
  float* DP1 = reinterpret_cast<float*>(smem + L_REGA + A_DP1);
  // unpool + ReLU mask -> dY2 (two layouts); wave w owns channels w and w+8 and
  // reduces their bias gradient with shuffles (fixed order: deterministic)
  for (int o = wave; o < 16; o += 8) {
    float bsum = 0.f;
    for (int r = lane; r < 160; r += 64) {
      const int y = r >> 4, x = r & 15;
      float v = 0.f;
      if (x < 10) {
        const int q = (y >> 1) * 5 + (x >> 1), i = ((y & 1) << 1) | (x & 1);
        if (CODE2[o * 25 + q] == i) v = DA0[o * 25 + q];
        DY2T[(y * 10 + x) * 16 + o] = (bf16)v;
      }
      DY2[o * 160 + r] = (bf16)v;
      bsum += v;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) bsum += __shfl_xor(bsum, off);
    if (lane == 0) slab[SLAB_C2B + o] = bsum;
  }
  for (int e = tid; e < 12 * 16; e += NT) DY2T[100 * 16 + e] = (bf16)0.f;
  __syncthreads();
  // conv2 wgrad: dW2[o][(c,ky,kx)] = sum_pix dY2[o][pix] * P1[c][y+ky][x+kx]
  for (int nt = wave; nt < 10; nt += 8) {
    const int n = nt * 16 + fr;
    const int c = n / 25, ky = (n % 25) / 5, kx = n % 5;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int y = 2 * s + (fg >> 1), x0 = 8 * (fg & 1);
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(DY2 + (fr * 10 + y) * 16 + x0);
      bf16x8 bb;
      if (n < 150) {
        bb = R2[(c * 14 + y + ky) * 13 + x0 + kx];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = (bf16)0.f;
      }
      acc = mfma32(a, bb, acc);
    }
    if (n < 150) {
#pragma unroll
      for (int i = 0; i < 4; ++i) slab[SLAB_C2W + (4 * fg + i) * 150 + n] = acc[i];
    }
  }
  // conv2 dgrad, col2im form: dCols[pix][(c,ky,kx)] = sum_o dY2[pix][o] * W2[o][(c,ky,kx)]
  for (int p = wave; p < 70; p += 8) {
    const int mt = p / 10, nt = p % 10;
    const s16x4 a = *reinterpret_cast<const s16x4*>(DY2T + (mt * 16 + fr) * 16 + 4 * fg);
    const int n = nt * 16 + fr;
    s16x4 bb;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bb[j] = n < 150 ? __builtin_bit_cast(short, W2S[(4 * fg + j) * 150 + n]) : (short)0;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bb, acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) DCOLS[(mt * 16 + 4 * fg + i) * DCOLS_LD + n] = acc[i];
  }
  __syncthreads();
  for (int e = tid; e < 6 * 196; e += NT) {  // deterministic col2im gather
    const int c = e / 196, r = e % 196, y = r / 14, x = r % 14;
    float s = 0.f;
#pragma unroll
    for (int ky = 0; ky < 5; ++ky) {
      const int y2 = y - ky;
      if (y2 < 0 || y2 >= 10) continue;
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
        const int x2 = x - kx;
        if (x2 < 0 || x2 >= 10) continue;
        s += DCOLS[(y2 * 10 + x2) * DCOLS_LD + c * 25 + ky * 5 + kx];
      }
    }
    DP1[e] = s;
  }
  __syncthreads();

  STAMP(6);
  // ============ phase F: conv1 weight gradient ==========================================
  bf16* DY1 = reinterpret_cast<bf16*>(smem + L_REGA + A_DY1);  // [6][28][32]
  if (wave < 6) {  // wave c: unpool + ReLU mask -> dY1[c], and the conv1 bias gradient
    const int c = wave;
    float bsum = 0.f;
#pragma unroll 2
    for (int r = lane; r < 896; r += 64) {
      const int y = r >> 5, x = r & 31;
      float v = 0.f;
      if (x < 28) {
        const int q = (y >> 1) * 14 + (x >> 1), i = ((y & 1) << 1) | (x & 1);
        if (CODE1[c * 196 + q] == i) v = DP1[c * 196 + q];
      }
      DY1[c * 896 + r] = (bf16)v;
      bsum += v;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) bsum += __shfl_xor(bsum, off);
    if (lane == 0) slab[SLAB_C1B + c] = bsum;
  } else if (tid - 384 < 96) {
    build_r1_row(IMGS, R1, tid - 384);  // R2 is dead: rebuild R1
  }
  __syncthreads();
  if (wave < 5) {  // dW1[o][(c,ky,kx)] = sum_pix dY1[o][pix] * X[c][y+ky][x+kx]
    const int nt = wave;
    const int n = nt * 16 + fr;
    const int c = n / 25, ky = (n % 25) / 5, kx = n % 5;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < 28; ++s) {  // one K-step = one 32-pixel output row
      bf16x8 a, bb;
      if (fr < 6) {
        a = *reinterpret_cast<const bf16x8*>(DY1 + (fr * 28 + s) * 32 + 8 * fg);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = (bf16)0.f;
      }
      if (n < 75) {
        bb = R1[(c * 32 + s + ky) * 29 + 8 * fg + kx];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = (bf16)0.f;
      }
      acc = mfma32(a, bb, acc);
    }
    if (n < 75) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 4 * fg + i;
        if (o < 6) slab[SLAB_C1W + o * 75 + n] = acc[i];
      }
    }
  }
  if (stamp) {
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(7);
  }
#undef STAMP
}

}  // namespace dnn

// ---- host launchers ---------------------------------------------------------------------
namespace dnn {

void init_kernels() {
  static bool done = false;
  if (done) return;
  HIP_CHECK(hipFuncSetAttribute((const void*)lenet_fused_kernel<true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL));
  HIP_CHECK(hipFuncSetAttribute((const void*)lenet_fused_kernel<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL));
  done = true;
}

void launch_fused_train(const uint8_t* images, const int32_t* labels, const int32_t* order, int order_len,
                        int batch, int32_t* state, const float* master, const bf16* shadow, float* a0,
                        float* h1, float* h2, float* z1, float* z2, float* z3, float* slab, float* loss,
                        int32_t* correct, long long* stamps, hipStream_t stream) {
  init_kernels();
  hipLaunchKernelGGL(lenet_fused_kernel<true>, dim3(batch), dim3(NT), LDS_TOTAL, stream, images, labels,
                     order, order_len, batch, 0, state, master, shadow, a0, h1, h2, z1, z2, z3, slab, loss,
                     correct, stamps);
  HIP_CHECK(hipGetLastError());
}

void launch_fused_eval(const uint8_t* images, const int32_t* labels, const int32_t* order, int n, int base,
                       int count, const float* master, const bf16* shadow, float* loss, int32_t* correct,
                       hipStream_t stream) {
  init_kernels();
  if (count <= 0) return;
  hipLaunchKernelGGL(lenet_fused_kernel<false>, dim3(count), dim3(NT), LDS_TOTAL, stream, images, labels,
                     order, n, count, base, nullptr, master, shadow, nullptr, nullptr, nullptr, nullptr,
                     nullptr, nullptr, nullptr, loss, correct, nullptr);
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

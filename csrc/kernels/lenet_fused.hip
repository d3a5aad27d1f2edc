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
//  * one workgroup = one sample = 8 waves (512 threads); every intermediate stays in
//    LDS (159 KB map below); HBM/L2 see the u8 image, bf16 weights and the small
//    per-sample output rows only.
//  * EVERY matmul-shaped op runs on MFMA v_mfma_f32_16x16x32_bf16 (fp32 accumulate):
//    conv fwd, conv wgrad, conv dgrad and all six MLP GEMVs (M = 1 row of a 16-row
//    tile: latency, not FLOPs, is the budget at this size).
//  * The im2col gather is replaced by "window records": rec[c][y][x] = X[c][y][x..x+7]
//    (16 B, bf16).  Ordering K as (c, ky, kx<8) makes every conv A/B fragment ONE
//    aligned ds_read_b128 - for the forward (8 kx per lane), the weight gradients
//    (8 consecutive pixels per lane) and the data gradient (records of zero-padded
//    dY2 against the flipped kernel).
//  * ReLU + 2x2 maxpool are fused into the conv epilogues: each 16-row M-tile is 4
//    pooling windows x 4 pixels, so a lane's 4 accumulator rows ARE one window.  The
//    argmax is a 2-bit code (4 = no gradient: max <= 0), replacing both
//    max_pool2d_with_indices and threshold_backward.
//  * Weights arrive pre-packed: the optimizer kernels keep MFMA-fragment images of
//    the conv kernels (incl. the flipped dgrad kernel) and transposed fc2/fc3 copies
//    in the bf16 shadow (common.h SH_*), so every B fragment is one 16-B load.
//  * fc1 (96 KB) streams into LDS by LDS-DMA (inline-asm global_load_lds) during the
//    convolutions, the flipped conv2 kernel during the MLP; both cross LDS-only
//    barriers (s_waitcnt lgkmcnt(0); s_barrier) that leave vmcnt alone.
//  * Every MFMA loop issues all of a tile's operand loads before its MFMA chain
//    (sched_barrier), so LDS latency is paid once per batch, not once per K-step.
#include <algorithm>
#include <cstddef>
#include <string>

#include "pers_common.h"
#include "runtime/aql_dispatch.h"

namespace dnn {

constexpr int NT = 512;
constexpr int CODES_PER_SAMPLE = 6 * 196 + 400;  // CODE1 [6][196] | CODE2 [16][25]: 2-bit argmax, 4 = no gradient

// ---- LDS map (bytes) ----------------------------------------------------------------
constexpr int L_REGA = 0;          // fc1 bf16 [120][400] (A-D) | conv2-bwd scratch (E) | dY1 (F)
constexpr int L_REGA_SZ = 96256;
constexpr int L_REGB = L_REGA + L_REGA_SZ;  // R1 records [3][32][29] (A-B, F) | R2 + WF (C-E)
constexpr int L_REGB_SZ = 44544;
constexpr int B_WF = 17472;                 // REGB: flipped conv2 kernel fragments after R2 (20,480 B)
constexpr int L_P1 = L_REGB + L_REGB_SZ;    // bf16 [6][14][20] (cols 14..19 zero; R2 holds bf16 anyway)
constexpr int L_CODE1 = L_P1 + 3360;        // u8 [6][196]
constexpr int L_A0 = L_CODE1 + 1184;        // f32 [400]  pooled conv2 output
constexpr int L_A0B = L_A0 + 1600;          // bf16 [416] (MFMA operand, zero padded)
constexpr int L_CODE2 = L_A0B + 832;        // u8 [400]
constexpr int L_H1 = L_CODE2 + 400;         // f32 [128]
constexpr int L_H1B = L_H1 + 512;           // bf16 [128]
constexpr int L_H2 = L_H1B + 256;           // f32 [96]
constexpr int L_H2B = L_H2 + 384;           // bf16 [96]
constexpr int L_LOG = L_H2B + 192;          // f32 [16]
constexpr int L_DZ3 = L_LOG + 64;           // f32 [16]
constexpr int L_DZ3B = L_DZ3 + 64;          // bf16 [32]
constexpr int L_DZ2 = L_DZ3B + 64;          // f32 [96]
constexpr int L_DZ2B = L_DZ2 + 384;         // bf16 [96]
constexpr int L_DZ1 = L_DZ2B + 192;         // f32 [128]
constexpr int L_DZ1B = L_DZ1 + 512;         // bf16 [128]
constexpr int L_DA0 = L_DZ1B + 256;         // f32 [400]
constexpr int L_IMG = L_DA0 + 1600;         // u8 [3][32][32] raw image (re-used by phase F)
constexpr int L_MISC = L_IMG + 3072;
constexpr int L_F1C = L_MISC + 64;          // u8 [80] phase F's conv1-wgrad column table (kF1Col)
constexpr int LDS_TOTAL = L_F1C + 128;      // 156,432 B
static_assert(LDS_TOTAL <= 163840, "LDS budget");
static_assert(B_WF + 20480 <= L_REGB_SZ, "REGB sub-layout");

// REGA sub-layout during the conv backward (fc1 weights are dead after the MLP dgrad)
constexpr int A_R3 = 0;                     // bf16x8 records [16][18][16 (14 used)] of padded dY2 73,728
constexpr int A_DY2 = 73728;                // bf16 [16][10][16], channel stride DY2_CS          5,632
constexpr int DY2_CS = 176;                 //   (elements = 22 x 16 B: the conv2-wgrad A reads are conflict-free,
                                            //   4 LDS cycles per read instead of 8 at 160 - tools/lds_banks.py)
constexpr int A_DP1 = A_DY2 + 16 * DY2_CS * 2;  // f32 [6][196]                                  4,704
constexpr int A_RS = A_DP1 + 4704;          // f32 [16][10] dY2 row sums (conv2 bias grad)         640
constexpr int A_DY1 = 0;                    // bf16 [6] x 1824 B (28 rows x 64 B + 32 B pad)    10,944
constexpr int DY1_CH = 1824;                //   channel stride 456 dwords (= 8 mod 64): conv1-wgrad A reads conflict-free
constexpr int A_RS1 = A_DY1 + 6 * DY1_CH;   // f32 [6][28] dY1 row sums (conv1 bias grad)          672
static_assert(A_RS + 1152 <= L_REGA_SZ, "REGA sub-layout");
static_assert(A_RS1 + 672 <= A_DP1, "phase F scratch must not overlap dP1");

// bf16 of the normalised value by ONE fma: fmaf(u, 2/255, -1) rounds to the same bf16 as
// the exact ToTensor+Normalize value for every u in 0..255 (checked exhaustively in
// tests/test_oracle_cpu.py), so no lookup table is needed.
__device__ __forceinline__ bf16 u8norm_bf16(uint32_t u) {
  return (bf16)__builtin_fmaf((float)u, (float)(2.0 / 255.0), -1.0f);
}

// Barrier for LDS hand-offs only: waits for this wave's LDS ops, not for vmcnt, so an
// in-flight LDS-DMA (global_load_lds) keeps streaming across it.  __syncthreads()
// would emit s_waitcnt vmcnt(0) and drain the DMA (and every outstanding store).
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

// Make hipcc treat a register as defined here: it waits for the load that produced it
// now (not at some later use where an asm DMA may be in flight behind it).
template <typename T>
__device__ __forceinline__ void consume(T& v) {
  asm volatile("" : "+v"(v));
}

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  return z;
}

// A operand of an M = 1 product: row 0 of the 16-row tile (lanes with fr == 0) holds
// x[k0 .. k0+7]; every other row is zero.
__device__ __forceinline__ bf16x8 row0(const bf16* x, int k0, int fr) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + k0);
  return fr == 0 ? v : zero8();
}

// Transposed B fragment of a [K rows][N cols] row-major bf16 LDS matrix (row stride
// `ld` elements): lane (fr, fg) gets B[k0 + 8fg + j][n0 + fr], j = 0..7, from two
// ds_read_b64_tr_b16 (4 rows x 16 columns each).  Rows are clamped to kmax - 1 (the
// clamped rows meet zero A entries).  EXEC must be all ones.
__device__ __forceinline__ bf16x8 tr_frag(const bf16* m, int ld, int k0, int n0, int kmax, int lane) {
  typedef __attribute__((address_space(3))) bf16x4* lp;
  const int l16 = lane & 15, q = l16 >> 2, p = l16 & 3, fg = lane >> 4;
  const int r0 = min(k0 + 8 * fg + q, kmax - 1), r1 = min(k0 + 8 * fg + 4 + q, kmax - 1);
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp)(m + r0 * ld + n0 + 4 * p));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp)(m + r1 * ld + n0 + 4 * p));
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
  return v;
}

// Build window records x = 8q .. 8q+7 (x < 29) of input row (c, y) = `row` from the u8
// image staged in LDS (normalised by u8norm_bf16, no table lookups); 4 threads per row.
__device__ __forceinline__ void build_r1_part(const uint8_t* img, bf16x8* R1, int row, int q) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(img + row * 32);
  uint32_t w[4];  // elements 8q .. 8q+15 (zero past the row end)
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = src[min(2 * q + k, 7)];
  bf16 v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t u = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    const bf16 t = u8norm_bf16(u);
    v[k] = (8 * q + k < 32) ? t : (bf16)0.f;
  }
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    if (8 * q + x < 29) {
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = v[x + j];
      R1[row * 29 + 8 * q + x] = r;
    }
  }
}

// Half of build_r1_part: records x = 4h .. 4h+3 (x < 29) of input row `row` (bit-identical
// records).  Phase F's R1 rebuild runs on these finer tasks so it balances over all 512 threads
// next to the dY1 rows.  Task u -> row (u & 7) + 8 (u >> 6), h = (u >> 3) & 7: the 8 lanes of a
// ds_write_b128 group take 8 consecutive rows of the same h (record stride 29 = 5 mod 8: 8
// distinct 4-dword slots).
__device__ __forceinline__ void build_r1_half(const uint8_t* img, bf16x8* R1, int u) {
  const int row = (u & 7) + 8 * (u >> 6), h = (u >> 3) & 7;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(img + row * 32);
  uint32_t w[3];  // pixels 4h .. 4h+11 (zero past the row end)
#pragma unroll
  for (int k = 0; k < 3; ++k) w[k] = src[min(h + k, 7)];
  bf16 v[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    const uint32_t px = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    const bf16 t = u8norm_bf16(px);
    v[k] = (4 * h + k < 32) ? t : (bf16)0.f;
  }
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    if (4 * h + x < 29) {
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = v[x + j];
      R1[row * 29 + 4 * h + x] = r;
    }
  }
}

// R1 builder thread -> (row, quarter): the 8 lanes of a ds_write_b128 group take 8
// different rows (row stride 29 records = 116 dwords -> 8 distinct 4-dword bank slots),
// conflict-free; the natural (row = t / 4) map put 4 lanes on one slot (tools/lds_banks.py).
__device__ __forceinline__ int r1_row(int t) { return (t & 7) + 8 * (t >> 5); }
__device__ __forceinline__ int r1_q(int t) { return (t >> 3) & 3; }

// R3 record (o, yy, x), x < 14: 16-record rows, x XOR-swizzled by yy & 7.  The conv2
// dgrad K order is kyp-major (p = 16 kyp + o, o = 4 (kk % 4) + fg), so the four K-groups of
// a K-step read the SAME yy of four channels: one XOR for all of them, 16 distinct 4-dword
// bank slots per read group; the builder's write groups (8 consecutive yy) hit 8 slots.
__device__ __forceinline__ int r3_index(int o, int yy, int x) { return (o * 18 + yy) * 16 + (x ^ (yy & 7)); }

// conv2 data gradient of output row Y0 (and Y0 + 8 when TWO) against the flipped kernel:
// K-step kk = (kyp, o-group) reads R3 row Y + kyp, and only rows 4..13 hold dY2, so the
// K-steps of the y-padding rows are dropped at compile time (row Y0 <= 7 needs
// kyp >= 4 - Y0, row Y0 + 8 needs kyp <= 5 - Y0).  Loads are batched per half.
template <int Y0, bool TWO>
__device__ __forceinline__ void dgrad_rows(const unsigned char* r3b, const bf16x8* wfl, int fg, int x,
                                           f32x4& acc0, f32x4& acc1) {
  constexpr int Y1 = TWO ? Y0 + 8 : Y0;
  const unsigned char* base0[5];
  const unsigned char* base1[5];
#pragma unroll
  for (int kyp = 0; kyp < 5; ++kyp) {
    base0[kyp] = r3b + 16 * r3_index(fg, Y0 + kyp, x);
    base1[kyp] = r3b + 16 * r3_index(fg, Y1 + kyp, x);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bf16x8 a0[10], a1[10], bv[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int kk = 10 * h + k, kyp = kk / 4, orow = 4 * (kk % 4) * 18 * 16 * 16;  // o offset, bytes
      bv[k] = wfl[kk * 64];
      if (Y0 + kyp >= 4) a0[k] = *reinterpret_cast<const bf16x8*>(base0[kyp] + orow);
      if (TWO && Y1 + kyp <= 13) a1[k] = *reinterpret_cast<const bf16x8*>(base1[kyp] + orow);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int kyp = (10 * h + k) / 4;
      if (Y0 + kyp >= 4) acc0 = mfma32(a0[k], bv[k], acc0);
      if (TWO && Y1 + kyp <= 13) acc1 = mfma32(a1[k], bv[k], acc1);
    }
  }
}

// ---- the pipelined step (PIPE) ----------------------------------------------------------
// Launch i of a pipelined chunk runs step i - 1's batch reduction + momentum SGD in its first
// workgroups and step i's samples in the rest, so the reduction hides under the samples' phase
// A (ingest) instead of sitting between two kernel boundaries.  Step i - 1's rows are in the
// other parity's buffers (written by launch i - 1: visible across the kernel boundary).  The
// new weights are a hand-off INSIDE the launch (MI355X guide §6 G16, R1): the reduction stores
// master biases / bf16 images write-through (sc1), every storing wave drains (vmcnt(0)), a
// workgroup barrier, then one lane per reduction block adds 1 to its group's counter; the block
// whose returning add completes the group stores a ready flag for every sample workgroup; the
// samples poll their own flag from one lane and load every weight byte with sc1 loads (buffer
// loads / LDS-DMA with sc1) - no acquire fence.
// Three ready groups, in the order the samples need them (reduction blocks start in this order):
//   PG_C1  conv1 weights + bias (phase B; with the head of conv2's - the group's last block is
//          shared), waited for by thread 0 after phase A's record build;
//   PG_C2  the rest of conv2 (phase C forward, phase E dgrad image), waited for by each wave
//          after phase B's first MFMA round - its fragments load behind the second;
//   PG_MLP fc weights + biases (phase C: the fc1 LDS stream; phase D fragments): checked in the
//          same poll round - a wave streams its part of fc1 mid-phase B if the group is
//          already complete, else after phase B once it is.
constexpr int PG_C1 = 0, PG_C2 = 1, PG_MLP = 2, PIPE_GROUPS = 3;
constexpr int PIPE_CTR_STRIDE = 32;  // counters and flags 128 B apart, each on a line of its own
static_assert(PIPE_BLOCKS == GRAD_REDUCE_BLOCKS, "the pipelined launch runs the whole grad_reduce");
static_assert(PIPE_C2_BLOCKS > 0, "conv2 keeps blocks of its own");
int pipe_reduce_blocks() { return PIPE_BLOCKS; }
int pipe_groups() { return PIPE_GROUPS; }

__device__ __forceinline__ int pipe_group_blocks(int grp) {
  return grp == PG_C1 ? PIPE_C1_BLOCKS : grp == PG_C2 ? PIPE_C2_BLOCKS : PIPE_MLP_BLOCKS;
}
// ready counters [parity][group]; broadcast flags [parity][group][sample]
__device__ __forceinline__ long pipe_ctr_index(int par, int grp) { return (long)(PIPE_GROUPS * par + grp) * PIPE_CTR_STRIDE; }
__device__ __forceinline__ long pipe_flag_index(int par, int grp, int b, int batch) {
  return ((long)(PIPE_GROUPS * par + grp) * batch + b) * PIPE_CTR_STRIDE;
}

// Reduction workgroup `wg` of a PIPE launch: two 256-thread reduction blocks.
__device__ __forceinline__ void pipe_reduce(const ReduceArgs& a, const PipeCtl& pc, int wg, long long* stamps) {
  const int half = threadIdx.x >> 8, m = 2 * wg + half, rtid = threadIdx.x & 255;
  if (wg == 0) {  // the next launch's counters and flags start from zero (kernel boundary)
    if (threadIdx.x < PIPE_GROUPS) pc.ctr[pipe_ctr_index(pc.par ^ 1, threadIdx.x)] = 0u;
    for (int i = threadIdx.x; i < PIPE_GROUPS * a.batch; i += blockDim.x)
      pc.flg[pipe_flag_index(pc.par ^ 1, i / a.batch, i % a.batch, a.batch)] = 0u;
  }
  int grp = -1;  // ready group this block signals (-1: none, the bookkeeping block)
  if (m < pc.nred) {
    int rblk = 0;  // (nred == 1: the bookkeeping alone - the launch range holds no elements)
    if (pc.nred > 1) {
      if (m < PIPE_CONV_BLOCKS) { rblk = PIPE_MLP_BLOCKS + m; grp = m < PIPE_C1_BLOCKS ? PG_C1 : PG_C2; }
      else if (m == PIPE_CONV_BLOCKS) rblk = PIPE_MLP_BLOCKS + PIPE_CONV_BLOCKS;
      else { rblk = m - PIPE_CONV_BLOCKS - 1; grp = PG_MLP; }
    }
    WtSink sk;
    grad_reduce_body(a, sk, rblk, rtid);
  }
  if (stamps != nullptr && threadIdx.x == 0) stamps[16 + 4 * wg + 1] = (long long)__builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its write-through stores
  __syncthreads();
  // the LAST block of a group (its returning add saw every other block's add, each made after
  // that block drained its stores) stores one flag per sample workgroup, each on a line of its
  // own: 64 pollers of ONE counter word serialize at its memory channel (a poll took 1-2 us
  // there: profiles/r4/pipe_v5, pipe_v6), their own flags return every ~0.3 us (pipe_v7)
  if ((rtid >> 6) == 0 && grp >= 0) {  // wave 0 of the block
    unsigned old = 0;
    if (rtid == 0)
      old = __hip_atomic_fetch_add(pc.ctr + pipe_ctr_index(pc.par, grp), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (stamps != nullptr && rtid == 0 && half == 0) stamps[16 + 4 * wg + 3] = (long long)__builtin_amdgcn_s_memrealtime();
    if (old == (unsigned)pipe_group_blocks(grp) - 1u)
      for (int b = rtid; b < a.batch; b += 64)
        __hip_atomic_store(pc.flg + pipe_flag_index(pc.par, grp, b, a.batch), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One lane waits until this sample workgroup's flag of group `grp` is set (uncached sc1 loads
// ~0.3 us apart).  also >= 0: each poll round also loads that group's flag (in flight with the
// first), its value at the round that ended the wait returned in *also_set - no extra round trip.
// Bounded: past the timeout it sets the sticky error word and returns (the step then runs on
// stale weights and the host raises at the next check) - never a hang.
// tgt: the tag the flag must reach (PIPE: 1; PERS: the step whose weights are awaited).
__device__ __forceinline__ void pipe_wait(const PipeCtl& pc, int grp, int b, int batch, long long* diag = nullptr,
                                          int also = -1, bool* also_set = nullptr, unsigned tgt = 1u) {
  const unsigned* f = pc.flg + pipe_flag_index(pc.par, grp, b, batch);
  const unsigned* g = pc.flg + pipe_flag_index(pc.par, also < 0 ? grp : also, b, batch);
  if (__hip_atomic_load(pc.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;  // failed before: no wait
  const long long t0 = wall_clock64();
  if (diag != nullptr) diag[0] = t0;
  long long polls = 0;
  while (true) {
    const unsigned v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned w = also >= 0 ? __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    if (diag != nullptr && polls < 12) {  // (t, value) of each poll's return: stamps[4096 + 2 k]
      diag[4082 + 2 * polls] = (long long)__builtin_amdgcn_s_memrealtime();
      diag[4083 + 2 * polls] = v;
    }
    if (v >= tgt) {
      if (also_set != nullptr) *also_set = w >= tgt;
      break;
    }
    ++polls;
    if (diag != nullptr) diag[1] = polls;
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > pc.timeout_ticks) {
      __hip_atomic_store(pc.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// ---- the persistent launch (PERS) -------------------------------------------------------------
// ONE launch runs pc.nsteps steps: the PIPE grid (reduction workgroups first, then one workgroup
// per sample), every workgroup looping over the steps.  Sample step s waits for the ready flags
// of the reduction of step s - 1 exactly as a PIPE launch waits for its own reduction (tags s
// instead of 1); the reduction of step t waits for its rows: every sample stores an arrival tag
// t + 1 into one word per reduction workgroup of the kind that reads its rows - MLP (after phase
// D': the MLP reduction overlaps the conv backward) and conv (after phase F) - written through,
// after its row / slab stores drained (the PIPE weight hand-off, run the other way).  Each word
// has one writer and one poller (a wave of the workgroup polls its batch of words in one load
// per 64 samples): no counter shared by many pollers.  Rows alternate between two parities; a
// sample writes parity s & 1 only after the waits of step s, which imply that every reduction
// block finished step s - 2 (blocks run their steps in order; each one is in a ready group).
// No kernel boundary, launch ramp or tail sits between two steps.
constexpr int PERS_WG = (PIPE_BLOCKS + 1) / 2;                // reduction workgroups
constexpr int PERS_CONV_WG = (PIPE_CONV_BLOCKS + 1 + 1) / 2;  // conv blocks + the bookkeeping block
constexpr int PERS_C1_WG = PIPE_C1_BLOCKS / 2;                // ready groups = workgroup ranges:
                                                              //   C1 [0, 4), C2 + bookkeeping [4, 23), MLP [23, 57)
static_assert((PIPE_CONV_BLOCKS + 1) % 2 == 0, "conv + bookkeeping blocks fill whole workgroups");
static_assert(PIPE_C1_BLOCKS % 2 == 0, "the conv1 group is whole workgroups");
static_assert(PERS_WG <= PERS_RROW, "one ready word per reduction workgroup in a sample's row");
// Step tags are generation-relative: every workgroup keeps its own generation word (the steps run
// by earlier launches; all equal, as every launch adds its nsteps to each), reads it at its start
// and adds nsteps at its end.  Tags of this launch are gen + t + 1 and compare wrap-safe, so no
// control word is ever reset: no exit counter, no reset pass before the kernel can retire.
// Ready hand-off: every reduction workgroup stores its step tag into ONE word of every sample's
// ready row [batch][PERS_RROW] (no counter, no atomic round trip, no last-block broadcast); a
// sample polls its whole row with one wave-wide load (lane = workgroup) and checks the lanes of
// the group it waits for.
// control memory: [256 generation words], [batch][PERS_RROW] ready rows, [PERS_WG][PERS_AROW]
// arrival words
int persist_ctl_bytes(int batch) { return (int)(pers_arrive_off(batch) + (long)PERS_WG * PERS_AROW * 4); }

// A sample's arrival at step tag - 1: kind 0 = the conv workgroups (slab, loss / correct read by
// the bookkeeping), 1 = the MLP workgroups.  One store per lane (lane = workgroup), by ONE wave,
// after every wave of the sample drained its stores and met a barrier.
__device__ __forceinline__ void pers_arrive(const PipeCtl& pc, int kind, int b, unsigned tag, int lane) {
  const int w0 = kind ? PERS_CONV_WG : 0, nw = kind ? PERS_WG - PERS_CONV_WG : PERS_CONV_WG;
  if (lane < nw) st_tag(pc.arrive + (long)(w0 + lane) * PERS_AROW + b, tag);
}

// A sample's wave waits until the ready words of workgroups [lo, hi) in its row reach tgt (every
// lane loads one word: lane = workgroup).  also_lo < also_hi: the same round also reports whether
// workgroups [also_lo, also_hi) are ready (*also_set, wave-uniform).  Bounded like pipe_wait.
// has_pre: the error word and this lane's ready word were loaded by the caller earlier (pre_err,
// pre_v: their round trip overlapped with other work); otherwise both are loaded here in ONE
// round trip.
struct PersPoll {
  unsigned err, v;
};
__device__ __forceinline__ const unsigned* pers_ready_word(const PipeCtl& pc, int b, int lane) {
  return pc.flg + (long)b * PERS_RROW + min(lane, PERS_WG - 1);
}
__device__ __forceinline__ PersPoll pers_poll_issue(const PipeCtl& pc, int b, int lane) {
  return PersPoll{ld_tag(pc.err), ld_tag(pers_ready_word(pc, b, lane))};
}
__device__ __forceinline__ void pers_wait_ready(const PipeCtl& pc, int b, int lo, int hi, unsigned tgt, int lane,
                                                int also_lo = 0, int also_hi = 0, bool* also_set = nullptr,
                                                long long* diag = nullptr, bool has_pre = false, unsigned pre_err = 0u,
                                                unsigned pre_v = 0u) {
  const unsigned* row = pers_ready_word(pc, b, lane);
  unsigned ferr = pre_err, v = pre_v;
  if (!has_pre) {
    const PersPoll first = pers_poll_issue(pc, b, lane);
    ferr = first.err;
    v = first.v;
  }
  if (ferr != 0u) return;
  const long long t0 = wall_clock64();
  if (diag != nullptr && lane == 0) diag[0] = t0;
  long long polls = 0;
  while (true) {
    if (__all((lane < lo || lane >= hi) || tag_ge(v, tgt))) {
      if (also_set != nullptr) *also_set = __all((lane < also_lo || lane >= also_hi) || tag_ge(v, tgt));
      break;
    }
    ++polls;
    if (diag != nullptr && lane == 0) diag[1] = polls;
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > pc.timeout_ticks) {
      if (lane == 0) __hip_atomic_store(pc.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    v = ld_tag(row);
  }
}

// Wave 0 at a persistent step's start: wait for the conv1 group's ready words (as pers_wait_ready).
// If the MLP group's words show ready first - the MLP reduction overlaps the previous step's conv
// backward, so it usually is - the wave streams the whole fc1 image into LDS meanwhile (every
// chunk: the other waves are at the barrier), in the idle time before conv1's weights instead of
// mid-phase B on every wave.  Returns whether it did (the caller skips the mid-phase-B stream).
template <class F>
__device__ __forceinline__ bool pers_wait_c1_early_fc1(const PipeCtl& pc, int b, unsigned tgt, int lane,
                                                       F&& stream_all) {
  const unsigned* row = pers_ready_word(pc, b, lane);
  const PersPoll first = pers_poll_issue(pc, b, lane);
  if (first.err != 0u) return false;
  const long long t0 = wall_clock64();
  bool streamed = false;
  unsigned v = first.v;
  while (true) {
    if (__all(lane >= PERS_C1_WG || tag_ge(v, tgt))) break;
    if (!streamed && __all(lane < PERS_CONV_WG || tag_ge(v, tgt))) {
      stream_all();
      streamed = true;
    }
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > pc.timeout_ticks) {
      if (lane == 0) __hip_atomic_store(pc.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    v = ld_tag(row);
  }
  return streamed;
}

// Reduction workgroup `wg` of a persistent launch: blocks 2 wg, 2 wg + 1 (pipe_reduce's map),
// every step in order: wait for the rows, reduce + SGD (write-through), signal the ready group.
// The bookkeeping block is in the conv2 group (samples read its slots after that wait).  Nothing
// is reset between launches: every ready / arrival tag is relative to the workgroup's generation
// word (all of them start at 0 and each launch advances every one by nsteps, as this one does last).
// XNR > 1 (the per-step all-reduce inside the persistent launch, up to XNR ranks): each block
// reduces its elements as above, then exchanges them over xGMI exactly as the serial one-launch
// exchange does (reduce_device.h xp_exchange / xp_exchange_rsag: the same per-lane granule
// protocol, block -> counter map, two-hop owner map and rank-order sum, so the parameters are
// bit-identical to it), and applies SGD with write-through stores before the workgroup signals
// its ready group.  The step tag of block gb in step t is xp_ctr[gb] + t + 1 (the counter the
// serial exchange keeps); the launch advances every counter by nsteps at its end.
template <int XNR>
__device__ __forceinline__ void pers_reduce(const ReduceArgs& a, const PipeCtl& pc, int wg, long long* stamps) {
  // (block-level indices are wave-uniform: readfirstlane keeps them - and the exchange's step tag
  // and slot pointers derived from them - in scalar registers)
  const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8), m = 2 * wg + half, rtid = threadIdx.x & 255,
            lane = threadIdx.x & 63;
  const bool bk = m == PIPE_CONV_BLOCKS;
  int rblk = 0;
  if (m < PIPE_CONV_BLOCKS) rblk = PIPE_MLP_BLOCKS + m;
  else if (!bk) rblk = m - PIPE_CONV_BLOCKS - 1;
  const unsigned g0 = __builtin_amdgcn_readfirstlane(ld_tag(pc.gen + blockIdx.x));  // this workgroup's generation
  // (XNR) this block's exchange counter: the grad_reduce block index (bookkeeping: the last one)
  const int gb = bk ? PIPE_MLP_BLOCKS + PIPE_CONV_BLOCKS : rblk;
  const unsigned xc0 = XNR > 1 ? __builtin_amdgcn_readfirstlane(a.xp_ctr[gb]) : 0u;
  if (bk && rtid < 64) bookkeeping_pers(a, pc, lane, -1);
  const unsigned* arr = pc.arrive + (long)wg * PERS_AROW;
  for (int t = 0; t < pc.nsteps; ++t) {
    if (threadIdx.x < 64) pers_wait_rows(pc, arr, a.batch, g0 + (unsigned)t + 1u, lane);
    // diagnostic (stamps): the last step's rows seen / body done / ready stored, per workgroup
    const bool st = stamps != nullptr && threadIdx.x == 0 && t == pc.nsteps - 1;
    if (st) stamps[2400 + 4 * wg] = (long long)__builtin_amdgcn_s_memrealtime();
    __syncthreads();
    // the lane's indices are re-derived in every step from an opaque copy of threadIdx.x, so the
    // per-lane address math of the reduction paths stays inside the step instead of being hoisted
    // out of the loop and kept live across it (the sample loop's trick: ~130 VGPRs held otherwise)
    int tid_o = threadIdx.x;
    asm volatile("" : "+v"(tid_o));
    const int rtid_s = tid_o & 255;
    if (bk) {
      if (rtid < 64) bookkeeping_pers(a, pc, lane, t);
    } else if constexpr (XNR > 1) {
      const unsigned step = xc0 + (unsigned)t + 1u;
      const bool failed = __hip_atomic_load(a.xp_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
      XpSinkT<false, true> sk;
      sk.tag = (unsigned long long)step << 32;
      sk.stash = tid_o;  // (8 x NT floats of the otherwise unused LDS)
      sk.stride = NT;
      // pull: every lane's granules go to this rank's slot; two-hop: only non-owners' (the
      // owner publishes the SUM in its ag slot instead)
      const bool publish = (a.xp_mode & 2) == 0 || gb % a.xp_nranks != a.xp_rank;
      sk.own = publish ? reinterpret_cast<unsigned long long*>(a.xp_region[a.xp_rank] + a.xp_gslot_off +
                                                               (step & 1u) * a.xp_gslot_bytes)
                       : nullptr;
      if (grad_reduce_body<XpSinkT<false, true>, true>(a, sk, rblk, rtid_s, t & 1)) {
        if ((a.xp_mode & 2) == 0) xp_exchange<XNR>(a, sk, step, failed, rblk, rtid_s);
        else xp_exchange_rsag<XNR>(a, sk, step, failed, rblk, rtid_s);
      }
    } else {
      WtSink sk;
      grad_reduce_body<WtSink, true>(a, sk, rblk, rtid_s, t & 1);
    }
    if (st) stamps[2401 + 4 * wg] = (long long)__builtin_amdgcn_s_memrealtime();
    // (diagnostic: the last step's per-wave body done / drain done of the conv1 workgroups)
    const bool wst = stamps != nullptr && (threadIdx.x & 63) == 0 && t == pc.nsteps - 1 && wg < PERS_C1_WG;
    if (wst) stamps[2640 + 16 * wg + 2 * (threadIdx.x >> 6)] = (long long)__builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
    if (wst) stamps[2641 + 16 * wg + 2 * (threadIdx.x >> 6)] = (long long)__builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (st) stamps[2402 + 4 * wg] = (long long)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < 64)  // both blocks done: this workgroup's word in every sample's ready row
      for (int b = lane; b < a.batch; b += 64) st_tag(pc.flg + (long)b * PERS_RROW + wg, g0 + (unsigned)t + 1u);
  }
  if (threadIdx.x == 0) st_tag(pc.gen + blockIdx.x, g0 + (unsigned)pc.nsteps);
  if constexpr (XNR > 1) {
    if (rtid == 0) a.xp_ctr[gb] = xc0 + (unsigned)pc.nsteps;  // (the next launch reads it: kernel boundary)
  }
}

// Weight loads: plain, or (WT: the pipelined step) sc1 buffer loads of the write-through bytes
template <bool WT>
struct WeightRd {
  const bf16* sh;
  const float* ms;
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ WeightRd(const bf16* shadow, const float* master) : sh(shadow), ms(master) {
    if constexpr (WT) r = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(shadow), 0, SH_TOTAL * 2, 0x00020000);
  }
  __device__ __forceinline__ bf16x8 w8(int e) const {  // 8 bf16 at element e (16-B aligned)
    if constexpr (WT) return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, e * 2, 0, 16));
    else return *reinterpret_cast<const bf16x8*>(sh + e);
  }
  __device__ __forceinline__ bf16x4 w4(int e) const {  // 4 bf16 at element e (8-B aligned)
    if constexpr (WT) return __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(r, e * 2, 0, 16));
    else return *reinterpret_cast<const bf16x4*>(sh + e);
  }
  __device__ __forceinline__ float f(int i) const {  // fp32 master element (biases)
    if constexpr (WT)
      return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(ms + i), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT));
    else return ms[i];
  }
};

// LDS-DMA with the sc1 cache policy (the pipelined step's weight streams; see dma16)
__device__ __forceinline__ void dma16_sc1(const void* gsrc, uint32_t lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}
template <bool WT>
__device__ __forceinline__ void dma_w(const void* gsrc, uint32_t lds_base) {
  if constexpr (WT) dma16_sc1(gsrc, lds_base);
  else dma16(gsrc, lds_base);
}

// Phase F's conv1 weight gradient: which of the 75 columns (c, ky, kx) lane fr of wave w (< 5)
// computes, kF1Col[16 w + fr] (bit 7: a padding lane - it reads that column, its result is
// discarded).  The B fragments are R1 records at (c * 32 + ky) * 29 + 8 fg + kx: in column order
// the 16 lanes of a ds_read_b128 lane group hit 8 of the 16 bank quads twice (2 LDS cycles per group
// instead of 1, 140 reads per step: tools/lds_banks.py).  This assignment (a search over the
// guide's lane groups) leaves 16 of the 20 (wave, group) pairs conflict-free.
__constant__ unsigned char kF1Col[80] = {73, 39, 201, 19, 35, 65, 56, 42, 30, 27, 59, 33, 38, 3, 25, 62, 74, 20, 17, 0, 57, 23, 72, 36, 13, 53, 10, 4, 22, 202, 18, 34, 54, 182, 67, 41, 68, 28, 2, 71, 31, 11, 55, 15, 40, 6, 9, 58, 49, 51, 37, 177, 43, 44, 12, 63, 21, 26, 24, 14, 60, 61, 48, 64, 50, 7, 70, 47, 46, 69, 45, 1, 8, 16, 32, 5, 66, 29, 178, 52};

// STAGED (TRAIN only): the image + label come from the stage buffer (see `stage` below)
// PIPE (TRAIN + STAGED only): the pipelined step's merged launch (above)
// PERS (PIPE only): the persistent launch - pc.nsteps steps, rows of both parities (above)
// XNR (PERS only): the per-step xGMI all-reduce inside the launch for groups of up to XNR ranks (0: none)
template <bool TRAIN, bool STAGED = false, bool PIPE = false, bool PERS = false, int XNR = 0>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 2))) lenet_fused_kernel(
    const uint8_t* __restrict__ images,   // [N][3][32][32] u8 (CIFAR binary order)
    const int32_t* __restrict__ labels,   // [N]
    const int32_t* __restrict__ order,    // [order_len] sample ids (nullptr: identity)
    int order_len, int batch, int base_index,
    int32_t* __restrict__ state,          // TRAIN: cursor/bvalid words
    const float* __restrict__ master,     // fp32 arena (biases)
    const bf16* __restrict__ shadow,      // bf16 shadow: arena copy + kernel-ready weight images
    float* __restrict__ a0_out, float* __restrict__ h1_out, float* __restrict__ h2_out,
    float* __restrict__ z1_out, float* __restrict__ z2_out, float* __restrict__ z3_out,
    float* __restrict__ slab_out, float* __restrict__ loss_out, int32_t* __restrict__ correct_out,
    long long* __restrict__ stamps,
    uint8_t* __restrict__ codes_out,       // TRAIN, diagnostic (tests): [batch][6*196 + 400] pool argmax codes
    const int32_t* __restrict__ next_ids,  // TRAIN + stage: sample ids of the NEXT step (-1: none)
    unsigned char* __restrict__ stage,     // TRAIN: [batch][IMG] u8 images + [batch] labels of THIS step
    const ReduceArgs ra,                   // PIPE: the previous step's reduction,
    const PipeCtl pc) {                     //   pc its control
  static_assert(!PIPE || (TRAIN && STAGED), "the pipelined step is a staged training launch");
  static_assert(!PERS || PIPE, "the persistent launch is a PIPE grid");
  static_assert(XNR == 0 || PERS, "the in-launch exchange is a persistent-launch feature");
  // stage (optional): block b of step c stores the image + label of step c + 1's sample b
  // there during phase F (next_ids: published two steps ahead by the reduce kernel's
  // bookkeeping; epoch_begin stages step 0); step c + 1 then loads its image from a fixed
  // address - one dependent load level (batch id -> image) off the start of phase A.
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // per-block diagnostic trace (stamps != nullptr): stamps[16 + 4 * block + k], k = 0 start,
  // 1 rows published, 2 end, 3 XCC id (reduction workgroups: start, end)
  const bool btrace = stamps != nullptr && threadIdx.x == 0;
  if (btrace) {
    stamps[16 + 4 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
    stamps[16 + 4 * blockIdx.x + 3] = (long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
  }
  // PIPE: the first workgroups run the previous step's reduction; the samples follow
  const int nrw = PIPE ? (pc.nred + 1) / 2 : 0;
  if constexpr (PIPE) {
    if ((int)blockIdx.x < nrw) {
      if constexpr (PERS) pers_reduce<XNR>(ra, pc, blockIdx.x, XNR > 1 ? nullptr : stamps);  // (XNR: at the register limit)
      else pipe_reduce(ra, pc, blockIdx.x, stamps);
      if (btrace) stamps[16 + 4 * blockIdx.x + 2] = (long long)__builtin_amdgcn_s_memrealtime();
      return;
    }
  }
  const int b = (int)blockIdx.x - nrw;
  const WeightRd<PIPE> wr(shadow, master);
  // PERS: the next step's image + label, loaded by waves 5-7 in phase F (register carry: the
  // same threads store it to LDS in the next step's phase A - no global round trip in-launch)
  uint4 carry_im = make_uint4(0, 0, 0, 0);
  int carry_lab = 0;
  const int nsteps = PERS ? pc.nsteps : 1;
  const unsigned g0 = PERS ? __builtin_amdgcn_readfirstlane(ld_tag(pc.gen + blockIdx.x)) : 0u;  // (PERS) generation
  if (TRAIN && threadIdx.x < 80) smem[L_F1C + threadIdx.x] = kF1Col[threadIdx.x];  // (read in phase F)
  int s = 0;  // (a do-while: without PERS the body is straight-line code, no loop at all)
  do {
  // the lane's indices are re-derived in every step from an opaque copy of threadIdx.x: the
  // per-lane address math of every phase then stays inside the step instead of being hoisted
  // out of the loop and kept live across it (that spilled ~1 KB per lane)
  int tid_opaque = threadIdx.x;
  if constexpr (PERS) asm volatile("" : "+v"(tid_opaque));
  const int tid = tid_opaque;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int fr = lane & 15;   // MFMA fragment row/col within the 16-tile
  const int fg = lane >> 4;   // MFMA k-group (0..3)
  // PERS: this step's rows are parity s & 1 (parity 1 of each row kind follows parity 0)
  const long rsh = PERS ? (long)(s & 1) * batch : 0;
  float* const a0_s = a0_out + rsh * A0_LD;
  float* const h1_s = h1_out + rsh * H1_LD;
  float* const h2_s = h2_out + rsh * H2_LD;
  float* const z1_s = z1_out + rsh * Z1_LD;
  float* const z2_s = z2_out + rsh * Z2_LD;
  float* const z3_s = z3_out + rsh * Z3_LD;
  float* const slab_s = slab_out + rsh * SLAB;
  float* const loss_s = loss_out + rsh;
  int32_t* const correct_s = correct_out + rsh;
  // PERS: waits from step 1 on (step 0's weights are the previous launch's), tag = the step
  const int do_wait = PERS ? (s > 0 ? 1 : 0) : pc.wait;
  const unsigned wtgt = PERS ? g0 + (unsigned)s : 1u;
  // diagnostic phase timeline (sample block 0, thread 0; PERS: the last step): s_memrealtime ticks
  const bool stamp = stamps != nullptr && (int)blockIdx.x == nrw && threadIdx.x == 0 && (!PERS || s == nsteps - 1);
  if (PERS && stamps != nullptr && (int)blockIdx.x == nrw && threadIdx.x == 0 && s < 1024)  // per-step starts
    stamps[2048 + s] = (long long)__builtin_amdgcn_s_memrealtime();
#define STAMP(i) do { if (stamp) stamps[i] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
  // (diagnostic: lane 0 of EVERY wave of the stamped block, stamps[base + wave])
  const bool wstamp = stamps != nullptr && (int)blockIdx.x == nrw && (threadIdx.x & 63) == 0 && (!PERS || s == nsteps - 1);
#define WSTAMP(base) do { if (wstamp) stamps[(base) + (threadIdx.x >> 6)] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
  STAMP(0);

  // TRAIN: the sample ids and valid count of this step were published by the previous
  // step's reduce kernel (begin_epoch for the first step): one dependent load level less
  // than cursor -> order -> sample.
  int bvalid = 1, sample = 0;
  bool valid;
  uint4 st_im = make_uint4(0, 0, 0, 0);
  int st_label = 0;
  uint4* const stage_im = reinterpret_cast<uint4*>(stage);
  int32_t* const stage_lab = reinterpret_cast<int32_t*>(stage + (size_t)batch * IMG);
  constexpr bool staged = TRAIN && STAGED;
  if (TRAIN) {
    if constexpr (staged) {  // issued first: independent of every other load of the kernel
      if (!PERS || s == 0) {
        st_im = stage_im[(size_t)b * (IMG / 16) + min(tid, IMG / 16 - 1)];
        st_label = stage_lab[b];
      }
    } else {
      sample = order[b];  // `order` = the published batch ids [batch]
    }
    // (PIPE: this launch's bookkeeping slot.  PERS: step 0's is the previous launch's; from step
    // 1 on the slot is read after the conv2 wait and checked after phase B - until then valid)
    if constexpr (PERS) bvalid = s == 0 ? *pc.bv_slot[0] : batch;
    else bvalid = PIPE ? *pc.bvalid : state[ST_BVALID];
    valid = b < bvalid;
  } else {
    const long gidx = (long)base_index + b;
    valid = gidx < order_len;
    sample = (int)gidx;
  }
  float my_loss = 0.f;
  int my_correct = 0;
  // a row element: plain, or (PERS) written through - the reduction of the same launch reads it
  auto put_row = [&](float* p, float v) {
    if constexpr (PERS) st_wt(p, v);
    else *p = v;
  };
  // PERS: every wave drained its stores (rows, slab, image stage) -> barrier -> one wave stores
  // this sample's arrival tags for the conv workgroups (kind 0) or the MLP workgroups (kind 1)
  auto pers_arrive_kind = [&](int kind) {
    // fault injection (flags & 256, tests only): sample 0 arrives for the conv workgroups of step 1
    // only 3 wait timeouts late - the reduction's bounded wait then fails, sets the sticky error
    // word, and every later wait returns at once (the host steps down to a slower step form)
    if (PERS && (pc.flags & 256) && b == 0 && s == 1 && kind == 0 && tid == 0) {
      const long long t0 = wall_clock64();
      while (wall_clock64() - t0 < 3 * pc.timeout_ticks) __builtin_amdgcn_s_sleep(64);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave == 0) pers_arrive(pc, kind, b, g0 + (unsigned)s + 1u, lane);
  };
  // an invalid sample (past the batch's valid count): zero rows, and (PERS) both arrivals
  auto invalid_sample = [&]() {
    // (an opaque thread index: these addresses must not be shared with phase D''s row stores -
    // a shared computation stays live across the whole step)
    int ti = threadIdx.x, bo = b;  // (b too: its row offsets were hoisted into the prologue and spilled)
    asm volatile("" : "+v"(ti), "+v"(bo));
    for (int i = ti; i < A0_LD; i += NT) put_row(a0_s + (size_t)bo * A0_LD + i, 0.f);
    for (int i = ti; i < H1_LD; i += NT) {
      put_row(h1_s + (size_t)bo * H1_LD + i, 0.f);
      put_row(z1_s + (size_t)bo * Z1_LD + i, 0.f);
    }
    for (int i = ti; i < H2_LD; i += NT) {
      put_row(h2_s + (size_t)bo * H2_LD + i, 0.f);
      put_row(z2_s + (size_t)bo * Z2_LD + i, 0.f);
    }
    for (int i = ti; i < Z3_LD; i += NT) put_row(z3_s + (size_t)bo * Z3_LD + i, 0.f);
    for (int i = ti; i < SLAB; i += NT) put_row(slab_s + (size_t)bo * SLAB + i, 0.f);
    if (ti == 0) {
      put_row(loss_s + bo, 0.f);
      put_row(reinterpret_cast<float*>(correct_s + bo), 0.f);
    }
    if constexpr (PERS) {
      pers_arrive_kind(1);
      pers_arrive_kind(0);
    }
  };
  if (!valid) {
    if constexpr (PERS) {
      invalid_sample();
      continue;
    } else {
      if (TRAIN) {
        for (int i = tid; i < A0_LD; i += NT) a0_out[(size_t)b * A0_LD + i] = 0.f;
        for (int i = tid; i < H1_LD; i += NT) {
          h1_out[(size_t)b * H1_LD + i] = 0.f;
          z1_out[(size_t)b * Z1_LD + i] = 0.f;
        }
        for (int i = tid; i < H2_LD; i += NT) {
          h2_out[(size_t)b * H2_LD + i] = 0.f;
          z2_out[(size_t)b * Z2_LD + i] = 0.f;
        }
        for (int i = tid; i < Z3_LD; i += NT) z3_out[(size_t)b * Z3_LD + i] = 0.f;
        for (int i = tid; i < SLAB; i += NT) slab_out[(size_t)b * SLAB + i] = 0.f;
        if (tid == 0) { loss_out[b] = 0.f; correct_out[b] = 0; }
      }
      return;
    }
  }
  int label;
  const uint8_t* img = images + (size_t)sample * IMG;
  if constexpr (staged) label = st_label;
  else label = labels[sample];

  bf16* fc1s = reinterpret_cast<bf16*>(smem + L_REGA);
  bf16x8* R1 = reinterpret_cast<bf16x8*>(smem + L_REGB);
  bf16x8* R2 = reinterpret_cast<bf16x8*>(smem + L_REGB);
  bf16x8* WF = reinterpret_cast<bf16x8*>(smem + L_REGB + B_WF);
  bf16* P1 = reinterpret_cast<bf16*>(smem + L_P1);
  uint8_t* CODE1 = smem + L_CODE1;
  float* A0 = reinterpret_cast<float*>(smem + L_A0);
  bf16* A0B = reinterpret_cast<bf16*>(smem + L_A0B);
  uint8_t* CODE2 = smem + L_CODE2;
  float* H1 = reinterpret_cast<float*>(smem + L_H1);
  bf16* H1B = reinterpret_cast<bf16*>(smem + L_H1B);
  float* H2 = reinterpret_cast<float*>(smem + L_H2);
  bf16* H2B = reinterpret_cast<bf16*>(smem + L_H2B);
  float* LOG = reinterpret_cast<float*>(smem + L_LOG);
  float* DZ3 = reinterpret_cast<float*>(smem + L_DZ3);
  bf16* DZ3B = reinterpret_cast<bf16*>(smem + L_DZ3B);
  float* DZ2 = reinterpret_cast<float*>(smem + L_DZ2);
  bf16* DZ2B = reinterpret_cast<bf16*>(smem + L_DZ2B);
  float* DZ1 = reinterpret_cast<float*>(smem + L_DZ1);
  bf16* DZ1B = reinterpret_cast<bf16*>(smem + L_DZ1B);
  float* DA0 = reinterpret_cast<float*>(smem + L_DA0);
  uint8_t* IMGS = smem + L_IMG;

  // ============ phase A: ingest + weight staging ======================================
  // Plain loads first: the image (issued first, so storing it to LDS waits for it alone),
  // then the conv B fragments and biases, whose latency hides behind the R1 record build;
  // they are consumed before the fc1 LDS-DMA is issued (hipcc would otherwise drain the
  // DMA at their first use, or under-count vmcnt for them).
  uint4 im;
  if constexpr (staged) im = st_im;
  else im = reinterpret_cast<const uint4*>(img)[min(tid, 191)];
  bf16x8 bw1[4], bw2[8];  // conv1 / conv2 forward B fragments (optimizer-packed images)
  float bias_c1 = 0.f, bias_c2 = 0.f;
  auto load_conv1_w = [&]() {
#pragma unroll
    for (int sk = 0; sk < 4; ++sk) bw1[sk] = wr.w8(SH_W1F + ((4 * sk + fg) * 16 + fr) * 8);
    bias_c1 = wr.f(OFF_C1B + min(fr >> 1, 5));  // (column fr = 2 o + s: channel o)
  };
  auto load_conv2_w = [&]() {
#pragma unroll
    for (int sk = 0; sk < 8; ++sk) bw2[sk] = wr.w8(SH_W2F + ((4 * sk + fg) * 16 + fr) * 8);
    bias_c2 = wr.f(OFF_C2B + fr);
  };
  auto consume_conv2_w = [&]() {
#pragma unroll
    for (int sk = 0; sk < 8; ++sk) consume(bw2[sk]);
    consume(bias_c2);
  };
  if constexpr (!PIPE) {  // (PIPE: conv1's once its reduction is ready, below; conv2's in phase B)
    load_conv1_w();
    load_conv2_w();
  }
  for (int i = tid; i < 6 * 14 * 20; i += NT) P1[i] = (bf16)0.f;
  if (tid < 16) A0B[400 + tid] = (bf16)0.f;                                   // MLP operand padding
  else if (tid < 24) H1B[120 + tid - 16] = (bf16)0.f;
  else if (tid < 36) H2B[84 + tid - 24] = (bf16)0.f;
  else if (tid < 58) DZ3B[10 + tid - 36] = (bf16)0.f;
  else if (tid < 70) DZ2B[84 + tid - 58] = (bf16)0.f;
  else if (tid < 78) DZ1B[120 + tid - 70] = (bf16)0.f;
  if (PERS && s > 0) {  // the image + label this wave group staged in the previous step's phase F
    if (tid >= 320) reinterpret_cast<uint4*>(IMGS)[tid - 320] = carry_im;
    if (tid == 320) *reinterpret_cast<int*>(smem + L_MISC) = carry_lab;
  } else {
    if (tid < 192) reinterpret_cast<uint4*>(IMGS)[tid] = im;
    if (PERS && tid == 0) *reinterpret_cast<int*>(smem + L_MISC) = label;
  }
  lds_barrier();
  if (PERS) label = *reinterpret_cast<const int*>(smem + L_MISC);  // (one path for every step)
  STAMP(9);
  if (tid < 384) build_r1_part(IMGS, R1, r1_row(tid), r1_q(tid));
  unsigned c2_err = 0u, c2_v = 0u;  // (PERS, below)
  int bv_pre = batch;
  if constexpr (PIPE) {
    // conv1's weights are the previous step's reduction's: one lane waits for its group (the
    // image and its records need none of it, so they are done first); the barrier releases the
    // other waves, then every wave loads its fragments (sc1) - waited for at phase B's first MFMA
    if constexpr (PERS) {
      if (wave == 0) {
        bool early = false;
        if (do_wait && !(pc.flags & 3)) {  // (flags & 2, measurement: no early stream)
          early = pers_wait_c1_early_fc1(pc, b, wtgt, lane, [&]() {  // all 94 fc1 chunks (1 KB each)
            const uint4* f1src = reinterpret_cast<const uint4*>(shadow + OFF_F1W);
            const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem + L_REGA));
            for (int i = 0; i < 94; ++i) dma_w<PIPE>(f1src + i * 64 + lane, base + (uint32_t)i * 1024u);
          });
        } else if (do_wait) {
          pers_wait_ready(pc, b, 0, PERS_C1_WG, wtgt, lane, 0, 0, nullptr, stamp ? stamps + 14 : nullptr);
        }
        if (lane == 0) reinterpret_cast<int*>(smem + L_MISC)[1] = early ? 1 : 0;
      }
    } else {
      if (tid == 0 && do_wait) pipe_wait(pc, PG_C1, b, batch, stamp ? stamps + 14 : nullptr, -1, nullptr, wtgt);
    }
    STAMP(12);
    lds_barrier();
    // PERS: the mid-phase-B poll's first round (error word + ready row) and, from step 2 on, this
    // step's valid count are loaded NOW, just before conv1's fragments - their round trips fly
    // with those loads and under phase B's first MFMA round instead of following it.  (The valid
    // count of step s was published by the bookkeeping of step s - 2, which the conv2-group wait
    // of step s - 1 already ordered before this load; step 1's slot is the launch start's
    // publication, ordered only by this step's conv2-group wait: read after it.)
    if constexpr (PERS) {
      if (do_wait) {
        const PersPoll p = pers_poll_issue(pc, b, lane);
        c2_err = p.err;
        c2_v = p.v;
      }
      if (s > 1) bv_pre = ld_sc1(pc.bv_slot[s & 1]);
    }
    load_conv1_w();
  } else {
#pragma unroll
    for (int sk = 0; sk < 4; ++sk) consume(bw1[sk]);
    consume(bias_c1);
    consume_conv2_w();
  }
  STAMP(11);
  // fc1: 94 wave-instructions x 1 KB = 96,256 B (fc1 + the head of fc1.bias, all in-arena);
  // 12 per wave with the index clamped (a duplicate copies identical bytes).  Issued here, or
  // (PIPE) per wave once the MLP reduction is ready: during or right after phase B
  auto stream_fc1 = [&]() {
    const uint4* f1src = reinterpret_cast<const uint4*>(shadow + OFF_F1W);
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem + L_REGA));
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const int i = min(wave + 8 * k, 93);
      dma_w<PIPE>(f1src + i * 64 + lane, base + (uint32_t)__builtin_amdgcn_readfirstlane(i) * 1024u);
    }
  };
  if constexpr (!PIPE) {
    stream_fc1();
    lds_barrier();
  }
  // PIPE: this wave has issued its part of the fc1 stream (PERS: or wave 0 streamed all of it
  // while waiting for conv1's weights)
  bool fc1_out = !PIPE;
  if constexpr (PERS) fc1_out = reinterpret_cast<const int*>(smem + L_MISC)[1] != 0;
  int bv_late = bv_pre;  // PERS: this step's valid count (from step 1 on)
  STAMP(1);

  // ============ phase B: conv1 (3->6, 5x5) + bias + ReLU + maxpool, MFMA ================
  {
    // conv1 as a GEMM over output PIXEL PAIRS: row = (pool window q, output row dy) of the two
    // horizontally adjacent outputs x, x + 1; column n' = 2 o + s = output channel o at shift s
    // (12 of 16 used); K = (c, ky) pairs x the 8 pixels j of an R1 record, against the B image
    // W1F[(c, ky)][2 o + s][j] = W[o][c][ky][j - s] (common.h write_shadow).  One 8-pixel record
    // feeds both outputs of a pair, so 25 tiles x 4 K-steps instead of 49 x 4 (one pixel per
    // row, 6 of 16 columns): half the MFMAs and half the A-operand LDS reads.
    float bias = 0.f;  // (set after round 0's MFMAs: see there)
    const int wl = fr >> 1, dy = fr & 1;  // A-operand row -> (window of the tile, output row)
    auto a_index = [&](int t, int sk) {  // R1 record of (tile t, K-step sk) for this lane
      const int q = min(8 * t + wl, 195);  // (tile 24's rows past window 195: clamped, discarded)
      const int y = 2 * (q / 14) + dy, x = 2 * (q % 14);
      const int pr = min(4 * sk + fg, 14);  // pair 15 is K padding: real data x zero weights
      return (pr / 5 * 32 + y + pr % 5) * 29 + x;
    };
    auto epilogue = [&](int t, f32x4 acc) {
      // lane (fr = 2 o + s, fg) holds rows 4 fg + i = (window 2 fg + (i >> 1), dy = i & 1) at
      // shift s; its neighbour lane fr ^ 1 (DPP quad swap, every lane) holds the other shift
      float nb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        nb[i] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc[i]), 0xB1, 0xf, 0xf, false));
      if (fr < 12 && dy == 0) {  // (fr even: s = 0) channel o = fr / 2, windows 2 fg, 2 fg + 1
        const int o = fr >> 1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int qo = 8 * t + 2 * fg + h;
          if (qo < 196) {
            // the window's pixels in torch's order (first max wins): (y, x), (y, x + 1), (y + 1, x), (y + 1, x + 1)
            float best = acc[2 * h] + bias;
            int arg = 0;
            const float v1 = nb[2 * h] + bias, v2 = acc[2 * h + 1] + bias, v3 = nb[2 * h + 1] + bias;
            if (v1 > best) { best = v1; arg = 1; }
            if (v2 > best) { best = v2; arg = 2; }
            if (v3 > best) { best = v3; arg = 3; }
            P1[(o * 14 + qo / 14) * 20 + qo % 14] = (bf16)fmaxf(best, 0.f);
            CODE1[o * 196 + qo] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
          }
        }
      }
    };
    // 25 tiles: round 0 = tiles wave, wave + 8; round 1 = tile wave + 16 (+ tile 24 on wave 0)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int t0 = r == 0 ? wave : wave + 16, t1 = r == 0 ? wave + 8 : 24;
      const bool two = r == 0 || wave == 0;  // wave-uniform
      bf16x8 a0[4], a1[4];
#pragma unroll
      for (int sk = 0; sk < 4; ++sk) {
        a0[sk] = R1[a_index(t0, sk)];
        if (two) a1[sk] = R1[a_index(t1, sk)];
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sk = 0; sk < 4; ++sk) {
        acc0 = mfma32(a0[sk], bw1[sk], acc0);
        if (two) acc1 = mfma32(a1[sk], bw1[sk], acc1);
      }
      // the bias is waited for HERE, on every lane (its load came with the B fragments the MFMAs
      // just waited for): first used inside the epilogue's divergent branch, hipcc otherwise keeps
      // it "pending" past that branch and waits again in round 1 with a vmcnt that also drains
      // the fc1 LDS-DMA issued in between (it does not count asm DMA)
      if (r == 0) {
        asm volatile("" : "+v"(bias_c1));
        bias = fr < 12 ? bias_c1 : 0.f;
      }
      epilogue(t0, acc0);
      if (two) epilogue(t1, acc1);
      STAMP(1000 + 3 * r);  // (diagnostic: phase B round r's epilogue issued)
      WSTAMP(1010 + 10 * r);
      if (PIPE && r == 0) {
        // conv2's group: lane 0 of each wave waits (the wave's other lanes with it) - with the MLP
        // flag in the same poll round.  If the MLP group is complete too, the wave's part of the
        // fc1 stream goes out first (the conv2 fragments after it: phase C's first use of them
        // then waits for both, issued a whole round earlier); else the fragments alone, consumed
        // before the stream is issued after phase B (vmcnt counts in issue order)
        int mlp = 0;
        if constexpr (PERS) {  // the whole wave polls its sample's ready row (C2 + bookkeeping, MLP)
          bool m = true;
          // (the pre-issued round's values become "defined" only here, after round 0's MFMAs - hipcc
          // would otherwise hoist the error check to the loads and wait for their round trip there)
          unsigned c2e = c2_err, c2v = c2_v;
          asm volatile("" : "+v"(c2e), "+v"(c2v) : "v"(acc0[0]));
          if (do_wait) pers_wait_ready(pc, b, PERS_C1_WG, PERS_CONV_WG, wtgt, lane, PERS_CONV_WG, PERS_WG, &m, nullptr, true,
                                       c2e, c2v);
          mlp = m && !(pc.flags & 1);
        } else if (lane == 0) {
          bool m = false;
          if (do_wait) pipe_wait(pc, PG_C2, b, batch, nullptr, (pc.flags & 1) ? -1 : PG_MLP, &m, wtgt);
          else m = true;  // (no reduction in this launch: every weight is the previous kernel's)
          mlp = m && !(pc.flags & 1);
        }
        // PERS: this step's valid count (published by the bookkeeping, a conv2-group block),
        // consumed after phase B
        if (PERS && s == 1) bv_late = ld_sc1(pc.bv_slot[s & 1]);
        STAMP(1001);  // (diagnostic: the mid-phase-B wait returned)
        WSTAMP(1040);
        if (!fc1_out && __builtin_amdgcn_readfirstlane(mlp)) {
          stream_fc1();
          fc1_out = true;
        }
        load_conv2_w();
        STAMP(1002);  // (diagnostic: the fc1 stream + conv2 fragment loads issued)
      }
    }
  }
  if constexpr (PIPE) {
    if (!fc1_out) {  // the MLP group was not complete mid-phase B: this wave waits for it here
      if constexpr (PERS) {
        if (do_wait) pers_wait_ready(pc, b, PERS_CONV_WG, PERS_WG, wtgt, lane);
      } else {
        if (lane == 0 && do_wait) pipe_wait(pc, PG_MLP, b, batch, nullptr, -1, nullptr, wtgt);
      }
      consume_conv2_w();
      stream_fc1();
    }
    STAMP(13);
  }
  WSTAMP(1050);  // (diagnostic: each wave at phase B's closing barrier)
  lds_barrier();
  if constexpr (PERS) {
    if (s > 0) {
      bvalid = bv_late;
      valid = b < bvalid;
      if (!valid) {  // (block-uniform) past the epoch's end: no phases C-F for this sample
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fc1 stream has landed before LDS is reused
        invalid_sample();
        continue;
      }
    }
  }

  STAMP(2);
  // ============ phase C: conv2 (6->16, 5x5) + bias + ReLU + maxpool, MFMA ===============
  // The MLP B fragments each lane needs in phase D are loaded now so conv2 hides their
  // latency; lane roles in the MLP: wave w owns output columns 16w + fr.
  const int ncol = 16 * wave + fr;
  if (tid < 168) {  // window records of P1 rows (overwrite R1: dead until phase F); 2 threads per row
    const int row = tid >> 1, h = tid & 1;  // row = c*14 + y; half h builds records 7h .. 7h+6 (< 13)
    bf16 v[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) v[k] = P1[row * 20 + 7 * h + k];
#pragma unroll
    for (int x = 0; x < 7; ++x) {
      if (7 * h + x < 13) {
        bf16x8 r;
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = v[x + j];
        R2[row * 13 + 7 * h + x] = r;
      }
    }
  }
  bf16x8 w2f[4], w2t[3], w3t, w3f[3];
  float bias_f1 = wr.f(OFF_F1B + min(ncol, 119));  // (first: waited for right after the R2 barrier, below)
  // Only the waves that use a fragment load it (fc2, fc3^T: waves 0-5; fc3: wave 0), and fc2^T's
  // (the MLP dgrad's) are loaded in phase D: the CU's vector-memory path is the bound here (a
  // wave stalls at issue while it is backed up, ~25 cycles per 1-KB wave load), and the record
  // builders go first so their LDS work overlaps the other waves' loads
  {
    const int r2 = OFF_F2W + min(ncol, 83) * 120;             // fc2 row (forward)
    if (wave < 6) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) w2f[ks] = wr.w8(r2 + 32 * ks + 8 * fg);
      w3t = wr.w8(SH_W3T + min(ncol, 83) * 16 + 8 * fg);       // fc3^T (dgrad)
    }
    if (wave == 0) {
      const int r3 = OFF_F3W + min(fr, 9) * 84;                // fc3 row (forward; 8-B aligned)
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x4 lo = wr.w4(r3 + 32 * ks + 8 * fg);
        const bf16x4 hi = wr.w4(r3 + 32 * ks + 8 * fg + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { w3f[ks][j] = lo[j]; w3f[ks][4 + j] = hi[j]; }
      }
    }
  }
  float bias_f2 = 0.f, bias_f3 = 0.f;
  if (wave < 6) bias_f2 = wr.f(OFF_F2B + min(ncol, 83));
  if (wave == 0) bias_f3 = wr.f(OFF_F3B + min(fr, 9));
  lds_barrier();
  // Wave 7 has no conv2 tile: it streams the flipped conv2 kernel (20,480 B) for phase E now -
  // LDS-DMA into REGB behind R2 (R1 is dead) - instead of every wave queueing three chunks at
  // phase D's start.  bias_f1 is waited for first on every wave (it is the oldest MLP load, so
  // only it): hipcc does not count the DMA, and a later wait of its own for a value this wave
  // loaded before the stream would drain the stream with it.
  consume(bias_f1);
  if (TRAIN && wave == 7) {
    const uint4* src = reinterpret_cast<const uint4*>(shadow + SH_WF);
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(smem + L_REGB + B_WF));
#pragma unroll
    for (int i = 0; i < 20; ++i) dma_w<PIPE>(src + i * 64 + lane, base + (uint32_t)i * 1024u);
  }
  if (wave < 7) {
    const int t = wave;
    const int wi = fr >> 2, pi = fr & 3;
    int q = 4 * t + wi;
    if (q > 24) q = 24;  // padding windows of the last tile: computed, discarded
    const int y = 2 * (q / 5) + (pi >> 1), x = 2 * (q % 5) + (pi & 1);
    bf16x8 a[8];
#pragma unroll
    for (int sk = 0; sk < 8; ++sk) {
      const int prc = min(4 * sk + fg, 29);  // pairs 30,31: zero weights in the B image
      a[sk] = R2[(prc / 5 * 14 + y + prc % 5) * 13 + x];
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sk = 0; sk < 8; ++sk) acc = mfma32(a[sk], bw2[sk], acc);
    const int qo = 4 * t + fg;
    if (qo < 25) {
      float best = acc[0] + bias_c2;
      int arg = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        const float v = acc[i] + bias_c2;
        if (v > best) { best = v; arg = i; }
      }
      const float r = fmaxf(best, 0.f);
      A0[fr * 25 + qo] = r;  // torch.flatten order [16][5][5]
      A0B[fr * 25 + qo] = (bf16)r;
      CODE2[fr * 25 + qo] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
    }
  }
  // fc1 LDS-DMA and the MLP fragments landed (wave 7: all but its 20 WF chunks, the newest -
  // waited for at phase E's start); each fragment consumed only where it was loaded
  if (TRAIN && wave == 7) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wave < 6) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) consume(w2f[ks]);
    consume(w3t);
    consume(bias_f2);
  }
  if (wave == 0) {
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) consume(w3f[ks]);
    consume(bias_f3);
  }
  lds_barrier();

  STAMP(3);
  // ============ phase D: MLP forward, cross-entropy, MLP data-backward ==================
  {  // fc1: h1 = relu(W1 a0 + b1), 120 x 400; wave w -> output tile w
    const bf16* wrow = fc1s + min(ncol, 119) * 400;
    bf16x8 av[13], bv[13];
#pragma unroll
    for (int ks = 0; ks < 13; ++ks) {
      bv[ks] = *reinterpret_cast<const bf16x8*>(wrow + 32 * ks + 8 * fg);
      av[ks] = row0(A0B, 32 * ks + 8 * fg, fr);
    }
    if (TRAIN) {  // fc2^T fragments (the MLP dgrad's), behind this wave's LDS reads
      const int t2 = SH_W2T + min(ncol, 119) * 96;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) w2t[ks] = wr.w8(t2 + 32 * ks + 8 * fg);
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 13; ++ks) acc = mfma32(av[ks], bv[ks], acc);
    if (fg == 0 && ncol < 120) {
      const float h = fmaxf(acc[0] + bias_f1, 0.f);
      H1[ncol] = h;
      H1B[ncol] = (bf16)h;
    }
  }
  lds_barrier();
  if (wave < 6) {  // fc2: 84 x 120
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) acc = mfma32(row0(H1B, 32 * ks + 8 * fg, fr), w2f[ks], acc);
    if (fg == 0 && ncol < 84) {
      const float h = fmaxf(acc[0] + bias_f2, 0.f);
      H2[ncol] = h;
      H2B[ncol] = (bf16)h;
    }
  }
  lds_barrier();
  if (wave == 0) {  // fc3 (10 x 84) + CrossEntropy (mean over the valid batch) + accuracy
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) acc = mfma32(row0(H2B, 32 * ks + 8 * fg, fr), w3f[ks], acc);
    // row 0 of the tile lives in lanes 0..15 (fg == 0): lane o holds logit o
    const bool act = lane < 10;
    const float lg = act ? acc[0] + bias_f3 : -INFINITY;
    // row reductions on DPP (common.h): bit-identical to xor-shuffle butterflies, without a
    // ds_bpermute round trip per step on the loss's critical path
    const float mx = max16(lg);
    const float e = act ? expf(lg - mx) : 0.f;
    const float sum = sum16(e);
    const int pred = min16((act && lg == mx) ? lane : 64);  // first max wins (torch.argmax)
    const float lse = mx + logf(sum);
    // (= __shfl(lg, label & 15, 16); ds_bpermute on the step's lane index - __shfl derives its own
    // lane id, which the persistent loop kept live across every step)
    const float ll = __int_as_float(__builtin_amdgcn_ds_bpermute(((lane & 48) | (label & 15)) << 2, __float_as_int(lg)));
    if (lane == 0) {
      put_row(loss_s + b, lse - ll);
      put_row(reinterpret_cast<float*>(correct_s + b), __int_as_float(pred == label ? 1 : 0));
      my_loss = lse - ll;  // (thread 0: also the in-launch bookkeeping's granule)
      my_correct = pred == label ? 1 : 0;
    }
    if (TRAIN && lane < 32) {
      const float dz = act ? (e / sum - (lane == label ? 1.f : 0.f)) / (float)bvalid : 0.f;
      DZ3B[lane] = (bf16)dz;
      if (lane < 16) DZ3[lane] = dz;
    }
  }
  if (!TRAIN) return;
  lds_barrier();
  STAMP(4);
  if (wave < 6) {  // fc3 dgrad: dh2 = W3^T dz3 (84 x 10), ReLU mask
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mfma32(row0(DZ3B, 8 * fg, fr), w3t, acc);
    if (fg == 0 && ncol < 84) {
      const float d = H2[ncol] > 0.f ? acc[0] : 0.f;
      DZ2[ncol] = d;
      DZ2B[ncol] = (bf16)d;
    }
  }
  lds_barrier();
  {  // fc2 dgrad: dh1 = W2^T dz2 (120 x 84), ReLU mask
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) acc = mfma32(row0(DZ2B, 32 * ks + 8 * fg, fr), w2t[ks], acc);
    if (fg == 0 && ncol < 120) {
      const float d = H1[ncol] > 0.f ? acc[0] : 0.f;
      DZ1[ncol] = d;
      DZ1B[ncol] = (bf16)d;
    }
  }
  lds_barrier();
  // fc1 dgrad: dA0 = W1^T dz1 (400 x 120), B fragments by transposed LDS reads of fc1.  The 25
  // column tiles of a wave (3, wave 0: 4) run as ONE batch: the A fragments (dz1, the same for
  // every tile) once, every tile's transposed reads in flight together, then the MFMA chains -
  // one LDS round trip per wave instead of one per tile (wave 0's fourth tile was a round of its
  // own on the phase's critical path)
  {
    bf16x8 av[4], bv[4][4];
    const bool four = wave == 0;  // wave-uniform: tile 24
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      av[ks] = row0(DZ1B, 32 * ks + 8 * fg, fr);
#pragma unroll
      for (int u = 0; u < 3; ++u) bv[u][ks] = tr_frag(fc1s, 400, 32 * ks, 16 * (wave + 8 * u), 120, lane);
      if (four) bv[3][ks] = tr_frag(fc1s, 400, 32 * ks, 16 * 24, 120, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
      for (int u = 0; u < 3; ++u) acc[u] = mfma32(av[ks], bv[u][ks], acc[u]);
      if (four) acc[3] = mfma32(av[ks], bv[3][ks], acc[3]);
    }
    if (fg == 0) {  // (the pool2/ReLU mask is applied via CODE2)
#pragma unroll
      for (int u = 0; u < 3; ++u) DA0[16 * (wave + 8 * u) + fr] = acc[u][0];
      if (four) DA0[16 * 24 + fr] = acc[3][0];
    }
  }
  // per-sample rows for the batch-reduced fc weight gradients (the reduction that follows, or
  // in a PERS launch the reduction workgroups of the same launch, reads them)
  for (int i = tid; i < A0_LD; i += NT) put_row(a0_s + (size_t)b * A0_LD + i, A0[i]);
  if (tid < H1_LD) { put_row(h1_s + (size_t)b * H1_LD + tid, H1[tid]); put_row(z1_s + (size_t)b * Z1_LD + tid, DZ1[tid]); }
  if (tid < H2_LD) { put_row(h2_s + (size_t)b * H2_LD + tid, H2[tid]); put_row(z2_s + (size_t)b * Z2_LD + tid, DZ2[tid]); }
  if (tid < Z3_LD) put_row(z3_s + (size_t)b * Z3_LD + tid, DZ3[tid]);
  lds_barrier();

  STAMP(5);
  if (!PERS && btrace) stamps[16 + 4 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
  // ============ phase E: conv2 backward =================================================
  // dY2 = unpool(dA0) masked by ReLU is materialised by rows, branch-free, twice:
  //  * DY2 [16][10][16] (channel stride DY2_CS): A operand of the conv2 weight gradient (8 pixels per lane),
  //  * R3  [16][18][14] window records of dY2 zero-padded by 4 in x (y rows 4..13; the y
  //    padding rows are skipped by the consumer, never stored): A operand of
  //    the conv2 DATA gradient as a direct implicit GEMM, K = (o, ky', kx'<8) against the
  //    flipped kernel WF - no col2im scratch, no gather pass.
  float* slab = slab_s + (size_t)b * SLAB;
#define SLAB_PUT(i, v) put_row(slab + (i), (v))
  bf16x8* R3 = reinterpret_cast<bf16x8*>(smem + L_REGA + A_R3);
  bf16* DY2 = reinterpret_cast<bf16*>(smem + L_REGA + A_DY2);
  float* DP1 = reinterpret_cast<float*>(smem + L_REGA + A_DP1);
  float* RS = reinterpret_cast<float*>(smem + L_REGA + A_RS);
  // 160 dY2 rows (o, y) x 2 record halves; the half is wave-uniform: threads 0-191 (waves
  // 0-2) build records 0-6 and the first DY2 record, threads 192-383 (waves 3-5) records
  // 7-13, the second DY2 record and the row sum.  The zero-padding rows of R3 (yy 0-3 and
  // 14-17) are never written: the data gradient skips the K-steps that would read them.
  {
    const int half = tid >= 192 ? 1 : 0;
    const int r = tid - 192 * half;
    if (tid < 384 && r < 160) {
      const int o = r / 10, y = r - 10 * o, yy = y + 4, yb = (y & 1) << 1;
      int cd[5];
      float da[5];
#pragma unroll
      for (int px = 0; px < 5; ++px) {
        const int q = o * 25 + (y >> 1) * 5 + px;
        cd[px] = CODE2[q];
        da[px] = DA0[q];
      }
      float v[22];  // v[cc] = dY2[o][y][cc - 4]
#pragma unroll
      for (int cc = 0; cc < 22; ++cc) {
        const int x = cc - 4;
        v[cc] = (x >= 0 && x < 10 && cd[x >> 1] == (yb | (x & 1))) ? da[x >> 1] : 0.f;
      }
      bf16x8* drow = reinterpret_cast<bf16x8*>(DY2 + o * DY2_CS + y * 16);
      if (half == 0) {
#pragma unroll
        for (int xr = 0; xr < 7; ++xr) {
          bf16x8 rr;
#pragma unroll
          for (int j = 0; j < 8; ++j) rr[j] = (bf16)v[xr + j];
          R3[r3_index(o, yy, xr)] = rr;
        }
        bf16x8 r0;
#pragma unroll
        for (int j = 0; j < 8; ++j) r0[j] = (bf16)v[4 + j];
        drow[0] = r0;
      } else {
#pragma unroll
        for (int xr = 7; xr < 14; ++xr) {
          bf16x8 rr;
#pragma unroll
          for (int j = 0; j < 8; ++j) rr[j] = (bf16)v[xr + j];
          R3[r3_index(o, yy, xr)] = rr;
        }
        bf16x8 r1;
        float rs = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) r1[j] = (bf16)(j < 2 ? v[12 + j] : 0.f);
#pragma unroll
        for (int x = 0; x < 10; ++x) rs += v[4 + x];
        drow[1] = r1;
        RS[o * 10 + y] = rs;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // WF (wave 7's LDS-DMA, issued in phase C) landed
  lds_barrier();
  STAMP(8);
  // PERS: every wave's row stores (phase D') drained before that barrier: the MLP workgroups go
  if (PERS && wave == 7) pers_arrive(pc, 1, b, g0 + (unsigned)s + 1u, lane);
  if (wave == 3) {  // conv2 bias gradient: 4 lanes per channel over its 10 row sums
    const int o = lane >> 2, part = lane & 3;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) t += (part + 4 * k < 10) ? RS[o * 10 + min(part + 4 * k, 9)] : 0.f;
    t = sum4(t);
    if (part == 0) SLAB_PUT(SLAB_C2B + o, t);
  }
  // conv2 data gradient: 14 tiles (one output row each, lanes x >= 14 duplicate x = 13)
  // x 20 K-steps in two halves.  Waves 0-5 run rows w and w + 8 TOGETHER (one WF
  // fragment load feeds both rows' MFMAs), waves 6-7 row w.  K-step kk: kyp = kk / 4
  // (compile-time), o = 4 (kk % 4) + fg, so every A load is a per-(lane, kyp) base
  // address + an immediate offset: no per-load address arithmetic.  The wave-uniform switch
  // picks a straight-line instance without the y-padding K-steps (max 28 MFMAs per wave).
  {
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const bool two = wv < 6;
    const int y0 = wv, y1 = two ? wv + 8 : wv, x = min(fr, 13);
    const unsigned char* r3b = reinterpret_cast<const unsigned char*>(R3);
    const bf16x8* wfl = WF + fg * 16 + fr;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    switch (wv) {
      case 0: dgrad_rows<0, true>(r3b, wfl, fg, x, acc0, acc1); break;
      case 1: dgrad_rows<1, true>(r3b, wfl, fg, x, acc0, acc1); break;
      case 2: dgrad_rows<2, true>(r3b, wfl, fg, x, acc0, acc1); break;
      case 3: dgrad_rows<3, true>(r3b, wfl, fg, x, acc0, acc1); break;
      case 4: dgrad_rows<4, true>(r3b, wfl, fg, x, acc0, acc1); break;
      case 5: dgrad_rows<5, true>(r3b, wfl, fg, x, acc0, acc1); break;
      case 6: dgrad_rows<6, false>(r3b, wfl, fg, x, acc0, acc1); break;
      default: dgrad_rows<7, false>(r3b, wfl, fg, x, acc0, acc1); break;
    }
    if (fr < 6) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int xo = 4 * fg + i;
        if (xo < 14) {
          DP1[fr * 196 + y0 * 14 + xo] = acc0[i];
          if (two) DP1[fr * 196 + y1 * 14 + xo] = acc1[i];
        }
      }
    }
  }
  // conv2 weight gradient: dW2[o][(c,ky,kx)] = sum_pix dY2[o][pix] * P1[c][y+ky][x+kx]
  // 10 column tiles, two per wave in one round, on waves 0, 2, 5, 6, 7: waves w and w + 4
  // share a SIMD, so this evens the per-SIMD load (paired rows on 0-5, single rows on 6-7,
  // conv2 bias gradient on 3).  The A operand (dY2 rows) depends only on the lane.
  if (wave == 0 || wave == 2 || wave >= 5) {
    const int slot = wave == 0 ? 0 : (wave == 2 ? 1 : wave - 3);
    const int nt_begin = 2 * slot, nt_end = nt_begin + 2;
    bf16x8 av[5];
#pragma unroll
    for (int sk = 0; sk < 5; ++sk) {
      const int y = 2 * sk + (fg >> 1), x0 = 8 * (fg & 1);
      av[sk] = *reinterpret_cast<const bf16x8*>(DY2 + fr * DY2_CS + y * 16 + x0);
    }
    for (int nt = nt_begin; nt < nt_end; nt += 2) {
      const bool two = nt + 1 < nt_end;
      int n[2], boff[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        n[u] = (nt + (two ? u : 0)) * 16 + fr;
        const int nc = min(n[u], 149);
        const int c = nc / 25, ky = (nc % 25) / 5, kx = nc % 5;
        boff[u] = (c * 14 + ky) * 13 + kx;
      }
      bf16x8 bv[2][5];
#pragma unroll
      for (int sk = 0; sk < 5; ++sk) {
        const int y = 2 * sk + (fg >> 1), x0 = 8 * (fg & 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) bv[u][sk] = R2[boff[u] + y * 13 + x0];
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int sk = 0; sk < 5; ++sk) {
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u] = mfma32(av[sk], bv[u][sk], acc[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if ((u == 0 || two) && n[u] < 150) {
#pragma unroll
          for (int i = 0; i < 4; ++i) SLAB_PUT(SLAB_C2W + (4 * fg + i) * 150 + n[u], acc[u][i]);
        }
      }
    }
  }
  // diagnostic: per-wave end of the phase-E work (block 0, lane 0 of each wave)
  if (stamps != nullptr && blockIdx.x == 0 && lane == 0) stamps[3000 + wave] = (long long)__builtin_amdgcn_s_memrealtime();
  lds_barrier();

  STAMP(6);
  // ============ phase F: conv1 weight gradient ==========================================
  // Waves 5-7 (no conv1-wgrad MFMAs) also stage the NEXT step's image + label: the sample
  // id is loaded under the F1 row build, the image under the F2 MMAs; the values live only
  // in those waves' branch, away from the register peak of the MFMA waves.
  int ns_next = -1;
  unsigned char* DY1 = smem + L_REGA + A_DY1;  // bf16 [6] x [28][32] (channel stride DY1_CH bytes)
  float* RS1 = reinterpret_cast<float*>(smem + L_REGA + A_RS1);
  if (tid < 168) {  // one dY1 row per thread: unpool dP1 by CODE1, ReLU-masked
    const int c = tid / 28, y = tid - 28 * (tid / 28), yb = (y & 1) << 1;
    int cd[14];
    float dv[14];
#pragma unroll
    for (int px = 0; px < 14; ++px) {
      const int q = c * 196 + (y >> 1) * 14 + px;
      cd[px] = CODE1[q];
      dv[px] = DP1[q];
    }
    float rs = 0.f;
    bf16x8* drow = reinterpret_cast<bf16x8*>(DY1 + c * DY1_CH + y * 64);
#pragma unroll
    for (int g8 = 0; g8 < 4; ++g8) {
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int x = 8 * g8 + j;
        float tv = 0.f;
        if (x < 28) tv = cd[x >> 1] == (yb | (x & 1)) ? dv[x >> 1] : 0.f;
        rs += tv;
        r[j] = (bf16)tv;
      }
      drow[g8] = r;
    }
    RS1[c * 28 + y] = rs;
    // the R1 rebuild (R2 is dead) in 768 half-row tasks: 2 on each thread past the dY1 rows,
    // the last 80 on threads 0..79 after their dY1 row (whole-row tasks left threads 168..207
    // with two full rows, 16 records, on the phase's critical path)
    static_assert(2 * (NT - 168) <= 768 && 768 - 2 * (NT - 168) <= 168, "R1 half-task split");
    if (tid < 768 - 2 * (NT - 168)) build_r1_half(IMGS, R1, 2 * (NT - 168) + tid);
  } else {
    if (staged && wave >= 5) {  // a vector load: the lgkmcnt(0) of the barriers does not wait for it
      const int32_t* p = (PERS ? pc.nid_slot[s & 1] : next_ids) + b;
      asm volatile("" : "+v"(p));
      ns_next = PERS ? ld_sc1(p) : *p;
    }
    build_r1_half(IMGS, R1, tid - 168);
    build_r1_half(IMGS, R1, tid - 168 + (NT - 168));
  }
  lds_barrier();
  STAMP(10);
  if (staged && wave >= 5 && ns_next >= 0) {
    const int t = tid - 320;  // 192 threads x 16 B = one image
    const uint4 v = reinterpret_cast<const uint4*>(images + (size_t)ns_next * IMG)[t];
    const int lab = t == 0 ? labels[ns_next] : 0;
    stage_im[(size_t)b * (IMG / 16) + t] = v;
    if (t == 0) stage_lab[b] = lab;
    if constexpr (PERS) {
      carry_im = v;
      carry_lab = lab;
    }
  }
  if (wave == 7) {  // conv1 bias gradient: 8 lanes per channel over its 28 row sums
    const int c = min(lane >> 3, 5), part = lane & 7;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) t += (part + 8 * k < 28) ? RS1[c * 28 + min(part + 8 * k, 27)] : 0.f;
    t = sum8(t);
    if (part == 0 && lane < 48) SLAB_PUT(SLAB_C1B + c, t);
  }
  if (wave < 5) {  // dW1[o][(c,ky,kx)] = sum_pix dY1[o][pix] * X[c][y+ky][x+kx]
    const int ent = smem[L_F1C + wave * 16 + fr];  // (kF1Col: column, bit 7 = padding lane)
    const int nc = ent & 127;
    const int c = nc / 25, ky = (nc % 25) / 5, kx = nc % 5;
    // rows o >= 6 of A read past dY1 into other (finite) LDS data: they only feed
    // accumulator rows that are discarded, so the loads stay branch-free
    const unsigned char* arow = DY1 + fr * DY1_CH + fg * 16;
    const bf16x8* brow = R1 + (c * 32 + ky) * 29 + 8 * fg + kx;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // one K-step = one 32-pixel output row; 7 per batch
      bf16x8 av[7], bv[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        av[k] = *reinterpret_cast<const bf16x8*>(arow + (7 * g + k) * 64);
        bv[k] = brow[(7 * g + k) * 29];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 7; ++k) acc = mfma32(av[k], bv[k], acc);
    }
    if (ent < 128) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 4 * fg + i;
        if (o < 6) SLAB_PUT(SLAB_C1W + o * 75 + nc, acc[i]);
      }
    }
  }
  if (codes_out != nullptr) {  // the ReLU + max-pool decisions of this sample (mask-aware oracle tests)
    for (int i = tid; i < CODES_PER_SAMPLE; i += NT)
      codes_out[(size_t)b * CODES_PER_SAMPLE + i] = i < 6 * 196 ? CODE1[i] : CODE2[i - 6 * 196];
  }
  if (stamp) {
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(7);
  }
  if constexpr (PERS) {
    pers_arrive_kind(0);  // slab + loss / correct drained: the conv workgroups go
    if (stamp) stamps[2398] = (long long)__builtin_amdgcn_s_memrealtime();
  }
#undef STAMP
#undef WSTAMP
#undef SLAB_PUT
  } while (PERS && ++s < nsteps);  // steps
  if (PERS && threadIdx.x == 0) st_tag(pc.gen + blockIdx.x, g0 + (unsigned)nsteps);
  if (btrace) stamps[16 + 4 * blockIdx.x + 2] = (long long)__builtin_amdgcn_s_memrealtime();
}

}  // namespace dnn

// ---- host launchers ---------------------------------------------------------------------
namespace dnn {

void init_kernels() {
  static bool done = false;
  if (done) return;
  const void* kerns[] = {(const void*)lenet_fused_kernel<true, false>, (const void*)lenet_fused_kernel<true, true>,
                         (const void*)lenet_fused_kernel<false, false>, (const void*)lenet_fused_kernel<true, true, true>,
                         (const void*)lenet_fused_kernel<true, true, true, true>,
                         (const void*)lenet_fused_kernel<true, true, true, true, 8>};
  for (const void* k : kerns) HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL));
  init_kernels_f32();
  done = true;
}

void launch_fused_train(const uint8_t* images, const int32_t* labels, const int32_t* order, int order_len,
                        int batch, int32_t* state, const float* master, const bf16* shadow, float* a0,
                        float* h1, float* h2, float* z1, float* z2, float* z3, float* slab, float* loss,
                        int32_t* correct, long long* stamps, const int32_t* next_ids, unsigned char* stage,
                        hipStream_t stream, uint8_t* codes) {
  init_kernels();
  if (stage != nullptr && next_ids == nullptr) throw std::runtime_error("fused_train: staging needs next_ids");
  auto* kern = stage ? &lenet_fused_kernel<true, true> : &lenet_fused_kernel<true, false>;
  hipLaunchKernelGGL(kern, dim3(batch), dim3(NT), LDS_TOTAL, stream, images, labels, order, order_len, batch, 0, state,
                     master, shadow, a0, h1, h2, z1, z2, z3, slab, loss, correct, stamps, codes, next_ids, stage,
                     ReduceArgs{}, PipeCtl{});
  HIP_CHECK(hipGetLastError());
}

void launch_fused_train_pipe(const uint8_t* images, const int32_t* labels, int order_len, int batch,
                             const float* master, const bf16* shadow, float* a0, float* h1, float* h2, float* z1,
                             float* z2, float* z3, float* slab, float* loss, int32_t* correct, long long* stamps,
                             const int32_t* next_ids, unsigned char* stage, const ReduceArgs& red, const PipeCtl& pc,
                             hipStream_t stream) {
  init_kernels();
  // the shapes the kernel assumes: every reduction block of a full launch (conv first), or the
  // bookkeeping alone; staged images; a ready wait only behind a full reduction
  if (stage == nullptr || next_ids == nullptr || pc.bvalid == nullptr || pc.ctr == nullptr || pc.err == nullptr ||
      pc.flg == nullptr)
    throw std::runtime_error(
        "fused_train_pipe: needs the stage, its next_ids / bvalid slot, the counters, flags and error word");
  if (!(pc.nred == PIPE_BLOCKS || pc.nred == 1) || (pc.wait && pc.nred != PIPE_BLOCKS) || (pc.par & ~1))
    throw std::runtime_error("fused_train_pipe: nred must be the whole reduction or the bookkeeping alone");
  if (!red.bookkeeping || red.batch != batch || red.xp_nranks != 0 || !red.fuse_sgd)
    throw std::runtime_error("fused_train_pipe: a local fused-SGD reduction with bookkeeping of this batch");
  if (pc.nred == PIPE_BLOCKS ? !(red.lo == 0 && red.hi >= ARENA) : !(red.lo == OFF_F1W && red.hi == OFF_F1W))
    throw std::runtime_error("fused_train_pipe: whole-arena reduction, or an empty range for the bookkeeping alone");
  if (batch < 1 || batch > 1024) throw std::runtime_error("fused_train_pipe: batch out of range");
  const int nrw = (pc.nred + 1) / 2;
  hipLaunchKernelGGL((lenet_fused_kernel<true, true, true>), dim3(nrw + batch), dim3(NT), LDS_TOTAL, stream, images,
                     labels, nullptr, order_len, batch, 0, red.state, master, shadow, a0, h1, h2, z1, z2, z3, slab,
                     loss, correct, stamps, nullptr, next_ids, stage, red, pc);
  HIP_CHECK(hipGetLastError());
}

// Largest batch whose persistent grid (PERS_WG reduction + batch sample workgroups, one per CU:
// each holds LDS_TOTAL of LDS) is co-resident on this device - a condition of every in-launch wait.
// The count comes from the runtime's occupancy calculator for THIS kernel at its launch shape
// (NT threads, LDS_TOTAL dynamic LDS: one workgroup per CU) times the CU count - not from an
// assumption - and keeps PERS_MARGIN CUs free for other work on the device (an RCCL kernel, the
// eval launch of another stream), so the grid stays co-resident next to them.
constexpr int PERS_MARGIN = 8;
int persist_resident_workgroups() {
  static int resident = -1;
  if (resident < 0) {
    init_kernels();
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(lenet_fused_kernel<true, true, true, true>), NT, LDS_TOTAL));
    int per_cu_x = 0;  // (the exchange instance: its own register count)
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu_x, reinterpret_cast<const void*>(lenet_fused_kernel<true, true, true, true, 8>), NT, LDS_TOTAL));
    resident = std::min(per_cu, per_cu_x) * cus;
  }
  return resident;
}
int persist_max_batch() {
  return std::max(0, std::min(persist_resident_workgroups() - PERS_WG - PERS_MARGIN, PERS_AROW));
}

// The persistent kernel's explicit parameter block, member for member (the AQL kernarg segment
// of a direct dispatch: the compiler lays kernel parameters out as this struct, and the kernel
// reads no hidden arguments - its kernarg segment is exactly these 648 bytes, checked against the
// loaded symbol at every dispatch).
struct PersKernargs {
  const uint8_t* images;
  const int32_t* labels;
  const int32_t* order;
  int order_len, batch, base_index;
  int32_t* state;
  const float* master;
  const bf16* shadow;
  float *a0, *h1, *h2, *z1, *z2, *z3, *slab, *loss;
  int32_t* correct;
  long long* stamps;
  uint8_t* codes;
  const int32_t* next_ids;
  unsigned char* stage;
  ReduceArgs ra;
  PipeCtl pc;
};
static_assert(offsetof(PersKernargs, ra) == 168 && offsetof(PersKernargs, pc) == 168 + sizeof(ReduceArgs),
              "kernel parameter layout");

int launch_fused_train_persist(const uint8_t* images, const int32_t* labels, int order_len, int batch,
                               const float* master, const bf16* shadow, float* a0, float* h1, float* h2, float* z1,
                               float* z2, float* z3, float* slab, float* loss, int32_t* correct, long long* stamps,
                               unsigned char* stage, const ReduceArgs& red, const PipeCtl& pc_in,
                               hipStream_t stream, bool direct) {
  init_kernels();
  // the shapes the kernel assumes (checked here: a mismatch would fault or hang on the device)
  if (batch < 1 || batch > persist_max_batch() || PERS_WG + batch > PERS_MAX_GRID)
    throw std::runtime_error("fused_train_persist: batch must be 1.." + std::to_string(persist_max_batch()) +
                             " (the whole grid co-resident)");
  if (pc_in.nsteps < 1 || pc_in.nsteps > (1 << 20)) throw std::runtime_error("fused_train_persist: nsteps out of range");
  if (stage == nullptr || pc_in.ctr == nullptr || pc_in.err == nullptr || !pc_in.bv_slot[0] || !pc_in.bv_slot[1] ||
      !pc_in.nid_slot[0] || !pc_in.nid_slot[1])
    throw std::runtime_error("fused_train_persist: needs the stage, the control block, the error word and both slots");
  if (!red.bookkeeping || red.batch != batch || !red.fuse_sgd || red.lo != 0 || red.hi < ARENA)
    throw std::runtime_error("fused_train_persist: a whole-arena fused-SGD reduction with bookkeeping");
  // the in-launch exchange: the serial one-launch exchange's arguments (whole arena, counters from
  // block 0, fp32 granules, pull or two-hop); grad_scale 1 (the tile update folds it: reduce_device.h)
  if (red.xp_nranks != 0 &&
      (red.xp_nranks < 1 || red.xp_nranks > XG_MAX_RANKS || (red.xp_mode & ~2) != 0 ||
       red.grad_scale != 1.f || red.xp_ctr == nullptr || red.xp_err == nullptr || red.xp_abort == nullptr ||
       red.xp_rank < 0 || red.xp_rank >= red.xp_nranks))
    throw std::runtime_error("fused_train_persist: the in-launch exchange takes the whole-arena one-launch exchange "
                             "(fp32 granules, pull or two-hop, grad_scale 1, counters set)");
  if (red.a0 != a0 || red.h1 != h1 || red.h2 != h2 || red.z1 != z1 || red.z2 != z2 || red.z3 != z3 ||
      red.slab != slab || red.loss != loss || red.correct != correct)
    throw std::runtime_error("fused_train_persist: the reduction reads the rows the samples write");
  PipeCtl pc = pc_in;  // control block layout (one uncached allocation of persist_ctl_bytes)
  unsigned char* base = reinterpret_cast<unsigned char*>(pc_in.ctr);
  pc.par = 0;
  pc.wait = 0;
  pc.nred = PIPE_BLOCKS;
  pc.gen = reinterpret_cast<unsigned*>(base);
  pc.flg = reinterpret_cast<unsigned*>(base + PERS_FLG_OFF);
  pc.arrive = reinterpret_cast<unsigned*>(base + pers_arrive_off(batch));
  auto* kern = red.xp_nranks == 0 ? &lenet_fused_kernel<true, true, true, true>
                                   : &lenet_fused_kernel<true, true, true, true, 8>;
  if (direct) {  // prepare (not launch) the same kernel object for this process's AQL queue
    PersKernargs ka{images, labels, nullptr, order_len, batch, 0, red.state, master, shadow, a0, h1, h2, z1, z2, z3,
                    slab, loss, correct, stamps, nullptr, pc.nid_slot[0], stage, red, pc};
    // every wait of the launch is bounded (pc.timeout_ticks), so the kernel ends within nsteps bounds
    const double bound_s = 10.0 + 2.0 * (double)pc.timeout_ticks * 1e-8 + 1e-3 * pc.nsteps;
    return aql_prepare(reinterpret_cast<const void*>(kern),
                       red.xp_nranks == 0 ? "lenet_fused_kernelILb1ELb1ELb1ELb1ELi0E" : "lenet_fused_kernelILb1ELb1ELb1ELb1ELi8E",
                       &ka, sizeof(ka), PERS_WG + batch, NT, LDS_TOTAL, bound_s, stream);
  }
  hipLaunchKernelGGL(kern, dim3(PERS_WG + batch), dim3(NT), LDS_TOTAL, stream, images, labels, nullptr, order_len,
                     batch, 0, red.state, master, shadow, a0, h1, h2, z1, z2, z3, slab, loss, correct, stamps, nullptr,
                     pc.nid_slot[0], stage, red, pc);
  HIP_CHECK(hipGetLastError());
  return -1;
}

void launch_fused_eval(const uint8_t* images, const int32_t* labels, const int32_t* order, int n, int base,
                       int count, const float* master, const bf16* shadow, float* loss, int32_t* correct,
                       hipStream_t stream) {
  init_kernels();
  if (count <= 0) return;
  hipLaunchKernelGGL((lenet_fused_kernel<false, false>), dim3(count), dim3(NT), LDS_TOTAL, stream, images, labels,
                     order, n, count, base, nullptr, master, shadow, nullptr, nullptr, nullptr, nullptr,
                     nullptr, nullptr, nullptr, loss, correct, nullptr, nullptr, nullptr, nullptr, ReduceArgs{},
                     PipeCtl{});
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

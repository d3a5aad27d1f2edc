// Implicit-GEMM 2-D convolution on MFMA for the generic layer engine (gfx950).
//
// Capability parity: aten::convolution / convolution_backward (SURVEY.md §2.5 K1, K4,
// K16, K18) for any stride-1, square-kernel, zero-padded Conv2d of a zoo model.  Replaces
// the engine's earlier im2col -> (cast) -> library GEMM -> col2im chain: the im2col view is
// gathered straight into LDS tiles inside the GEMM, so nothing B x C x K^2 x H x W sized is
// ever written to HBM, and bf16 operands are converted while staging (no cast kernels).
//
//   forward : y[b][m][p]  = sum_k W[m][k] * im2col(x)[k][(b, p)]  (+ bias[m])   M = Cout
//   dgrad   : the same kernel on dY with the flipped, channel-transposed weights and
//             pad' = K - 1 - pad (a stride-1 transposed convolution)              M = Cin
//   wgrad   : dW[m][j]   = sum_r dY[m][r] * im2col(x)[j][r],  r = (b, p)  (B*OH*OW long),
//             with an all-ones row j = Kd appended so the bias gradient comes out of the
//             same MFMAs: split over S workgroup slices into fp32 partials, then a
//             fixed-order sum (deterministic, no float atomics)
//
// Forward and dgrad run on an LDS-patch kernel (conv_fwd_patch_kernel, below) whenever its
// tiles fit the LDS budget - every zoo layer does - and on the general gather kernel
// otherwise.  Its weight images are packed once per step for all layers
// (launch_conv_pack_all), and its input patch moves as float4 pixel groups when image rows
// are whole 16-B vectors.  (An LDS-patch wgrad was measured and lost to the gather kernel
// below: profiles/r1_wgrad_patch_experiment.txt.)
//
// Tiling: a workgroup (4 waves) owns a BM x 64 output tile (BM = 16/32/64 from M); wave w
// owns columns [16 w, 16 w + 16) and all BM rows as BM/16 16x16 accumulators.  The
// reduction runs in 64-wide chunks staged through LDS in k-contiguous rows, so every MFMA
// operand is one LDS read: fp32 -> v_mfma_f32_16x16x4_f32 (16 per chunk, exact fp32
// products), bf16 -> v_mfma_f32_16x16x32_bf16 (2 per chunk, one ds_read_b128 per operand).
// The next chunk's global gathers are issued before the current chunk's MFMAs (register
// prefetch), so their latency overlaps the math and the other resident workgroups.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "launchers.h"

namespace dnn {
namespace {

constexpr int CT = 256;   // threads per workgroup
constexpr int BN = 64;    // output columns per workgroup
constexpr int BK = 64;    // reduction chunk
constexpr int KPT = 16;   // reduction elements staged per thread and chunk (BK * 64 rows / 256 threads)
constexpr int LDF = 68;   // fp32 LDS row stride (floats): 16-B aligned rows, conflict-free operand reads
constexpr int LDH = 72;   // bf16 LDS row stride (elements): 144-B rows

struct Geom {
  int B, C, H, W, K, pad, OH, OW;
};

// KPT consecutive rows k0 .. k0+KPT-1 of im2col(x) at output position (b, oy, ox), with
// k = (c, ky, kx); 0 outside the image and for k >= Kd.  One (c, ky, kx) decomposition per
// call, then an incremental walk (no per-element integer division: the divisions were the
// kernels' dominant VALU cost).  ONES: row k == Kd is all ones (the wgrad's bias column:
// db[m] = sum_r dY[m][r] * 1 comes out of the same MFMAs as dW).
template <bool ONES = false>
__device__ __forceinline__ void gather_rows(const float* __restrict__ x, const Geom& g, int k0, int Kd, int b, int oy,
                                            int ox, bool valid, float (&v)[KPT]) {
  const int KK = g.K * g.K;
  const int kc = min(k0, Kd - 1);
  int c = kc / KK;
  const int r = kc - c * KK;
  int ky = r / g.K, kx = r - ky * g.K;
  int iy = oy + ky - g.pad, ix = ox + kx - g.pad;
  int off = ((b * g.C + c) * g.H + iy) * g.W + ix;  // may be out of the image: only used when in bounds
#pragma unroll
  for (int e = 0; e < KPT; ++e) {
    const bool in = valid && k0 + e < Kd && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
    v[e] = in ? x[off] : ((ONES && valid && k0 + e == Kd) ? 1.f : 0.f);
    // advance k -> k + 1
    ++kx; ++ix; ++off;
    if (kx == g.K) {
      kx = 0; ix -= g.K; ++ky; ++iy; off += g.W - g.K;
      if (ky == g.K) { ky = 0; iy -= g.K; ++c; off += (g.H - g.K) * g.W; }
    }
  }
}

template <bool BF16>
struct Lds {
  using T = typename std::conditional<BF16, bf16, float>::type;
  static constexpr int LD = BF16 ? LDH : LDF;
};

template <bool BF16>
__device__ __forceinline__ void put(typename Lds<BF16>::T* s, int i, float v) {
  if constexpr (BF16) s[i] = (bf16)v; else s[i] = v;
}

// one BK chunk of MFMAs from the staged tiles: As[BM][LD] (row m, k-contiguous),
// Bs[BN][LD] (row = output column, k-contiguous)
template <bool BF16, int BM>
__device__ __forceinline__ void mma_chunk(const typename Lds<BF16>::T* As, const typename Lds<BF16>::T* Bs,
                                          f32x4 (&acc)[BM / 16], int wave, int lane) {
  constexpr int LD = Lds<BF16>::LD;
  const int r16 = lane & 15, q = lane >> 4;
  if constexpr (BF16) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(Bs + (wave * 16 + r16) * LD + kk + 8 * q);
#pragma unroll
      for (int i = 0; i < BM / 16; ++i) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(As + (16 * i + r16) * LD + kk + 8 * q);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i], 0, 0, 0);
      }
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const float bv = Bs[(wave * 16 + r16) * LD + kk + q];
#pragma unroll
      for (int i = 0; i < BM / 16; ++i) {
        const float av = As[(16 * i + r16) * LD + kk + q];
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i], 0, 0, 0);
      }
    }
  }
}

// ---- forward / dgrad: y[b][m][p] = sum_k w[m][k] im2col(x)[k][(b,p)] + bias[m] -----------------
template <bool BF16, int BM>
__global__ void __launch_bounds__(CT) conv_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ bias, float* __restrict__ y, Geom g,
                                                      int M) {
  using T = typename Lds<BF16>::T;
  constexpr int LD = Lds<BF16>::LD;
  __shared__ __attribute__((aligned(16))) T As[BM * LD];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int KK = g.K * g.K, Kd = g.C * KK, OHW = g.OH * g.OW;
  const long N = (long)g.B * OHW;
  const long n0 = (long)blockIdx.x * BN;
  const int m0 = blockIdx.y * BM;

  // B-tile role: one output column (lanes along consecutive positions: coalesced rows of
  // x), KPT consecutive k of the chunk per thread
  const int col = tid & 63, kg = tid >> 6;
  const long n = n0 + col;
  const bool nvalid = n < N;
  const long nc = nvalid ? n : N - 1;
  const int bb = (int)(nc / OHW), p = (int)(nc % OHW), oy = p / g.OW, ox = p % g.OW;
  // A-tile role: row tid / 4 of the weight tile, KPT consecutive k
  const int am = tid >> 2, ak = (tid & 3) * KPT;
  const bool avalid_m = am < BM && m0 + am < M;
  const float* wrow = w + (long)(avalid_m ? m0 + am : 0) * Kd;

  f32x4 acc[BM / 16];
#pragma unroll
  for (int i = 0; i < BM / 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  float av[KPT], bv[KPT];
  auto load = [&](int k0) {  // global -> registers (the next chunk's loads fly during this chunk's MFMAs)
#pragma unroll
    for (int e = 0; e < KPT; ++e) {
      const int ka = k0 + ak + e;
      av[e] = (avalid_m && ka < Kd) ? wrow[ka] : 0.f;
    }
    gather_rows(x, g, k0 + kg * KPT, Kd, bb, oy, ox, nvalid, bv);
  };
  load(0);
  for (int k0 = 0; k0 < Kd; k0 += BK) {
    __syncthreads();  // the previous chunk's MFMAs are done with the tiles
    if (am < BM) {
#pragma unroll
      for (int e = 0; e < KPT; ++e) put<BF16>(As, am * LD + ak + e, av[e]);
    }
#pragma unroll
    for (int e = 0; e < KPT; ++e) put<BF16>(Bs, col * LD + kg * KPT + e, bv[e]);
    __syncthreads();
    if (k0 + BK < Kd) load(k0 + BK);
    mma_chunk<BF16, BM>(As, Bs, acc, wave, lane);
  }

  // epilogue: acc[i][j] = D[16 i + 4 q + j][16 wave + r16]
  const int r16 = lane & 15, q = lane >> 4;
  const long on = n0 + wave * 16 + r16;
  if (on < N) {
    const int ob = (int)(on / OHW), op = (int)(on % OHW);
#pragma unroll
    for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + 16 * i + 4 * q + j;
        if (m < M) y[((long)ob * M + m) * OHW + op] = acc[i][j] + (bias != nullptr ? bias[m] : 0.f);
      }
    }
  }
}

// ---- wgrad: part[s][m][j] = sum_{r in slice s} dy[m][r] im2col(x)[j][r] -----------------------
// UNPOOL: dy is the gradient of the 2x2 max-pool that followed this conv's ReLU ([B][M][OH/2][OW/2])
// with its argmax codes; the full-resolution gradient is formed on the load (the value where the
// code names the position, else 0) instead of by a relu_pool_bwd launch.
template <bool BF16, int BM, bool UNPOOL = false>
__global__ void __launch_bounds__(CT) conv_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        float* __restrict__ part, Geom g, int M, int chunks_per_slice,
                                                        const uint8_t* __restrict__ code = nullptr) {
  using T = typename Lds<BF16>::T;
  constexpr int LD = Lds<BF16>::LD;
  __shared__ __attribute__((aligned(16))) T As[BM * LD];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int KK = g.K * g.K, Kd = g.C * KK, OHW = g.OH * g.OW;
  const long R = (long)g.B * OHW;
  const int j0 = blockIdx.x * BN, m0 = blockIdx.y * BM, s = blockIdx.z;
  const long r_begin = (long)s * chunks_per_slice * BK;
  const long r_end = min(R, r_begin + (long)chunks_per_slice * BK);

  // both tiles: lanes along BK consecutive r (contiguous positions), KPT rows per thread.  (A
  // readfirstlane-uniform row group - scalar branches, row tables in SGPRs - measured slower:
  // 100 SGPR spills; profiles/r2/layer_fusion/README.md.)
  const int rl = tid & 63, rowg = (tid >> 6) * KPT;

  f32x4 acc[BM / 16];
#pragma unroll
  for (int i = 0; i < BM / 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Every load is a raw buffer load whose offset is out of range (the hardware returns 0) when
  // the element is: no exec-masked loads, no 64-bit address math.  The KPT im2col rows of this
  // thread are chunk-invariant: their (c, ky, kx) decomposition is done once, as a row offset
  // and the (ky - pad, kx - pad) shift; per chunk only the position (b, oy, ox) moves, walked
  // incrementally (the per-chunk 64-bit division by OH*OW and the per-call (c, ky, kx)
  // divisions were most of this kernel's VALU work).
  constexpr unsigned OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x), 0, g.B * g.C * g.H * g.W * (int)sizeof(float), 0x00020000);
  int rowoff[KPT];        // element offset of row k relative to the position's (b, 0, oy, ox)
  unsigned shift[KPT];    // (ky - pad + 128) | (kx - pad + 128) << 8, or ~0 for k >= Kd (never in bounds)
  unsigned ones = 0;      // bit e: row k == Kd (the bias column: value 1)
  {
    const int k0 = j0 + rowg, kc = min(k0, Kd - 1);
    int c = kc / KK;
    const int rr = kc - c * KK;
    int ky = rr / g.K, kx = rr - ky * g.K;
#pragma unroll
    for (int e = 0; e < KPT; ++e) {
      const bool kin = k0 + e < Kd;
      rowoff[e] = (c * g.H + ky - g.pad) * g.W + kx - g.pad;
      shift[e] = kin ? (unsigned)(ky - g.pad + 128) | ((unsigned)(kx - g.pad + 128) << 8) : ~0u;
      if (k0 + e == Kd) ones |= 1u << e;
      if (++kx == g.K) { kx = 0; if (++ky == g.K) { ky = 0; ++c; } }
    }
  }
  // this lane's position, walked by BK per chunk
  const int rs = (int)min(r_begin + rl, R - 1);
  int pb = rs / OHW, prem = rs - pb * OHW;
  int poy = prem / g.OW, pox = prem - poy * g.OW;
  const int dq = BK / g.OW, dr = BK - dq * g.OW;

  float av[KPT], bv[KPT];
  auto load = [&](long r0) {
    const bool rv = r0 + rl < r_end;
    const int bb = pb, oy = poy, ox = pox;
    if constexpr (UNPOOL) {
      const int OH2 = g.OH >> 1, OW2 = g.OW >> 1, py = min(oy >> 1, OH2 - 1), px = min(ox >> 1, OW2 - 1);
      const bool inb = (oy >> 1) < OH2 && (ox >> 1) < OW2;
      const uint8_t sub = (uint8_t)(((oy & 1) << 1) | (ox & 1));
      // raw buffer loads (out-of-range offsets read 0), 32-bit offsets: no masked loads
      const int P2 = OH2 * OW2, pp = (bb * M + m0 + rowg) * P2 + py * OW2 + px;
      const __amdgpu_buffer_rsrc_t dr2 = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(dy), 0, g.B * M * P2 * (int)sizeof(float), 0x00020000);
      const __amdgpu_buffer_rsrc_t cr2 = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint8_t*>(code), 0, g.B * M * P2, 0x00020000);
      float a[KPT];
      unsigned cd[KPT];
#pragma unroll
      for (int e = 0; e < KPT; ++e) {
        const bool mv = rowg + e < BM && m0 + rowg + e < M;
        const int o = pp + e * P2;
        a[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dr2, mv ? o * 4 : (int)OOB, 0, 0));
        cd[e] = __builtin_amdgcn_raw_buffer_load_b8(cr2, mv ? o : (int)OOB, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < KPT; ++e) {
        const bool mv = rowg + e < BM && m0 + rowg + e < M;
        av[e] = (mv && rv && inb && cd[e] == sub) ? a[e] : 0.f;
      }
    } else {
      const __amdgpu_buffer_rsrc_t dr_ = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(dy), 0, g.B * M * OHW * (int)sizeof(float), 0x00020000);
      const int dbase = (bb * M + m0 + rowg) * OHW + oy * g.OW + ox;
#pragma unroll
      for (int e = 0; e < KPT; ++e) {
        const bool mv = rowg + e < BM && m0 + rowg + e < M && rv;
        const unsigned off = mv ? (unsigned)(dbase + e * OHW) * 4u : OOB;
        av[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dr_, (int)off, 0, 0));
      }
    }
    const int pbase = bb * g.C * g.H * g.W + oy * g.W + ox;
#pragma unroll
    for (int e = 0; e < KPT; ++e) {
      const int iy = oy + (int)(shift[e] & 0xffu) - 128, ix = ox + (int)((shift[e] >> 8) & 0xffu) - 128;
      const bool in = rv && shift[e] != ~0u && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      const unsigned off = in ? (unsigned)(pbase + rowoff[e]) * 4u : OOB;
      const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)off, 0, 0));
      bv[e] = ((ones >> e) & 1u) ? (rv ? 1.f : 0.f) : v;
    }
    // advance the position by BK for the next chunk
    pox += dr; poy += dq;
    if (pox >= g.OW) { pox -= g.OW; ++poy; }
    while (poy >= g.OH) { poy -= g.OH; ++pb; }
    if (pb >= g.B) { pb = g.B - 1; }  // past the end: every element of it is masked (rv false)
  };
  if (r_begin < r_end) load(r_begin);
  for (long r0 = r_begin; r0 < r_end; r0 += BK) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < KPT; ++e) {
      if (rowg + e < BM) put<BF16>(As, (rowg + e) * LD + rl, av[e]);
      put<BF16>(Bs, (rowg + e) * LD + rl, bv[e]);
    }
    __syncthreads();
    if (r0 + BK < r_end) load(r0 + BK);
    mma_chunk<BF16, BM>(As, Bs, acc, wave, lane);
  }

  const int r16 = lane & 15, q = lane >> 4;
  const int j = j0 + wave * 16 + r16;
  if (j <= Kd) {  // column Kd = the bias gradient
#pragma unroll
    for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int m = m0 + 16 * i + 4 * q + jj;
        if (m < M) part[((long)s * M + m) * (Kd + 1) + j] = acc[i][jj];
      }
    }
  }
}

// dw[e] = sum_s part[s][e] in a fixed order (deterministic).  A workgroup owns 64
// consecutive elements; wave w of SW sums slices w, w+SW, ... (8 loads in flight per
// batch), then wave 0 adds the SW wave sums in order.  Grid = n / 64 workgroups: the
// earlier one-thread-per-element loop over all S slices was latency-bound at 26-56 us.
// part rows are [M][Kd + 1]: column Kd goes to db, the rest to dw.
constexpr int SW = 16;  // waves per slice-sum workgroup
__global__ void __launch_bounds__(SW * 64) slice_sum_kernel(const float* __restrict__ part, int S, long n, int Kd,
                                                            float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[SW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + lane;
  const bool ev = e < n;
  const float* p = part + (ev ? e : 0);
  float acc = 0.f;
  for (int s0 = wave; s0 < S; s0 += 8 * SW) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = s0 + SW * u;
      v[u] = s < S ? p[(long)s * n] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && ev) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < SW; ++w) v += red[w][lane];
    const int m = (int)(e / (Kd + 1)), j = (int)(e - (long)m * (Kd + 1));
    if (j < Kd) dw[(long)m * Kd + j] = v;
    else db[m] = v;
  }
}

// wf[c][o][ky][kx] = w[o][c][K-1-ky][K-1-kx]  (dgrad weights)
__global__ void __launch_bounds__(CT) flip_weights_kernel(const float* __restrict__ w, int O, int C, int K,
                                                          float* __restrict__ wf) {
  const int n = O * C * K * K;
  for (int e = blockIdx.x * CT + threadIdx.x; e < n; e += gridDim.x * CT) {
    const int kx = e % K, ky = (e / K) % K, o = (e / (K * K)) % O, c = e / (K * K * O);
    wf[e] = w[((o * C + c) * K + (K - 1 - ky)) * K + (K - 1 - kx)];
  }
}

// ---- fast forward / dgrad: LDS-resident input patch + packed weights ---------------------------
// The general kernel above re-gathers every im2col element from global memory (K^2 reads
// of each input value per M-tile).  This path stages, per 32-channel chunk, the input
// rows a 64-position output tile needs as a zero-padded patch P[r][x][c] (channels
// innermost) and the weights as A[tap][m][c], both in LDS.  With the reduction ordered
// k = (ky, kx, c), the operand of one tap is then a plain shifted view of the patch: a
// lane's eight consecutive k are eight consecutive channels of one patch pixel - one
// ds_read_b128 - and no index arithmetic runs in the MFMA loop (a per-lane base plus a
// wave-uniform tap offset).  Each input element is read from HBM/L2 once per tile.
//   bf16: v_mfma_f32_16x16x32_bf16, one per (tap, 16-row subtile); 32-channel chunks
//   fp32: v_mfma_f32_16x16x4f32, CCH / 4 per (tap, subtile); 8 / 16 / 32-channel chunks
//         (the smallest that holds C: the reference LeNet has C = 3 and 6)
constexpr int PNT = 64;  // output positions per workgroup tile (4 waves x 16 columns)
// register batch of one chunk per thread: AV 16-B weight vectors, PV patch elements - sized
// per channel chunk so the small-C (LeNet) variants keep their occupancy
template <int CCH> struct Batch { static constexpr int AV = 6, PV = 20; };     // 32-ch chunks (vgg)
template <> struct Batch<16> { static constexpr int AV = 7, PV = 13; };        // lenet conv2 dgrad
template <> struct Batch<8> { static constexpr int AV = 4, PV = 8; };          // lenet conv1 / conv2

template <bool BF16, int CCH>
struct PatchT {
  using T = typename std::conditional<BF16, bf16, float>::type;
  // channel stride of one patch pixel / weight row: 80 B (bf16), 48 / 80 / 144 B (fp32) -
  // 16-B aligned, and 16 consecutive pixels land on distinct 16-B bank groups
  static constexpr int CCP = BF16 ? 40 : CCH + 4;
};

struct PGeom {
  int B, C, H, W, K, pad, OH, OW, M;
  int R, Wp, tiles, Cp, Mp;  // patch rows, padded width, tiles per image, padded C / M
  int ppt;                   // output positions per tile (PNT; pooled: rpt whole rows x OW)
  int rpt;                   // pooled: output rows per tile (even), else 0
};

// wp[(tap * Mp + m) * Cp + c] = w[m][c][ky][kx]            (forward)
//                             = w[c][m][K-1-ky][K-1-kx]    (flip: dgrad, w is [C][M][K][K])
// zero for m >= M or c >= C
template <typename T>
__global__ void __launch_bounds__(CT) pack_weights_kernel(const float* __restrict__ w, int M, int C, int K, int Mp,
                                                          int Cp, int flip, T* __restrict__ wp) {
  const int KK = K * K, n = KK * Mp * Cp;
  for (int e = blockIdx.x * CT + threadIdx.x; e < n; e += gridDim.x * CT) {
    const int c = e % Cp, m = (e / Cp) % Mp, tap = e / (Cp * Mp);
    const int ky = tap / K, kx = tap - ky * K;
    float v = 0.f;
    if (m < M && c < C)
      v = flip ? w[((c * M + m) * K + (K - 1 - ky)) * K + (K - 1 - kx)] : w[((m * C + c) * K + ky) * K + kx];
    wp[e] = (T)v;
  }
}

// Epilogues (EPI):
//   EPI_PLAIN  y = conv + bias.
//   EPI_POOL   ReLU + 2x2 max-pool (first maximum wins, code 4 = max <= 0 - relu_pool_fwd_kernel's
//              exact rule): tiles are rpt whole output rows, the tile's conv outputs go through
//              LDS, y is the pooled [B][M][OH/2][OW/2] output and code its argmax codes; the
//              full-resolution output is never written.
//   EPI_STATS  y as EPI_PLAIN, plus the following BatchNorm's batch statistics: per channel the
//              tile's (sum y, sum y^2) in fp64 over its positions (fixed order) into
//              stats[(m * P + tile) * 2 + {0, 1}], P = B * tiles; images past the step state's
//              valid count contribute 0 (the padded tail batch, as chan_partial_kernel).
//   EPI_BNBWD  (a data gradient whose output is the gradient of a BatchNorm + ReLU (+ max-pool)
//              output) y as EPI_PLAIN, plus that BatchNorm's backward statistics: per channel the
//              tile's (sum dz, sum dz * xhat) in fp64 - chan_partial_kernel<1, ACT>'s terms, same
//              layout as EPI_STATS.  ReLU: dz = y where the BatchNorm output is > 0 (the bit-exact
//              affine recompute of the backward kernels), xhat = (z - mean) * invstd.  ReLU +
//              pool: y is the pooled gradient; it lands on the window's argmax position (code
//              < 4; code 4 = max <= 0: no gradient), so dz = y there and xhat is taken at that
//              full-resolution position of z.
//   EPI_UNPOOL (input side; epilogue as EPI_PLAIN) x is the gradient of the 2x2 max-pool that
//              followed a ReLU ([B][C][H/2][W/2]) and `code` its argmax codes: the patch loads
//              unpool on the fly, x(c, iy, ix) = code == ((iy & 1) << 1 | (ix & 1)) ? x_pooled : 0
//              - the data gradient of a pooled conv without relu_pool_bwd's full-size round trip
//              (scalar patch path, register batch only: conv_fwd_unpool_ok)
constexpr int EPI_PLAIN = 0, EPI_POOL = 1, EPI_STATS = 2, EPI_BNBWD = 3, EPI_UNPOOL = 4;
struct BnTerms {  // EPI_BNBWD: the BatchNorm whose output gradient this kernel produces
  const float* z;       // its input [B][M][zH][zW]
  const float* mean;    // saved batch mean / inverse std, affine weight / bias [M]
  const float* invstd;
  const float* gamma;
  const float* beta;
  const uint8_t* code;  // ReLU + 2x2 max-pool after the BatchNorm: its argmax codes [B][M][OH][OW] (this
                        // kernel's output grid), else nullptr (ReLU only: zH, zW = OH, OW)
  int zH, zW;
};
// U8 (float4 patch path): the layer's input is the training step's ingest - the patch loads
// read the u8 dataset images of the batch's sample ids directly and normalise them as
// ingest_kernel does (bit-identical), the workgroup that owns an input row (row-aligned
// tiles: `own` rows each, the first / last tile also the rows above / below) stores the
// normalised values to x_out for the weight gradient, and tile 0 copies the label - the
// ingest launch of the step disappears.
struct InArgs {
  const uint8_t* images;  // [N][C][H][W] u8 dataset
  const int32_t* ids;     // [B] sample id of each batch row
  const int32_t* labels;  // [N]
  float* x_out;           // [B][C][H][W] normalised input
  int32_t* lab_out;       // [B]
  int own;                // input rows owned per tile
};

template <bool BF16, int BM, int CCH, bool V4, int EPI = EPI_PLAIN, bool U8 = false>
__global__ void __launch_bounds__(CT) conv_fwd_patch_kernel(const float* __restrict__ x,
                                                            const typename PatchT<BF16, CCH>::T* __restrict__ wp,
                                                            const float* __restrict__ bias, float* __restrict__ y,
                                                            PGeom g, uint8_t* __restrict__ code = nullptr,
                                                            double* __restrict__ stats = nullptr,
                                                            const int32_t* __restrict__ state = nullptr,
                                                            const BnTerms bt = BnTerms{},
                                                            const InArgs in = InArgs{}) {
  constexpr bool POOL = EPI == EPI_POOL;
  constexpr bool UNP = EPI == EPI_UNPOOL;
  static_assert(!U8 || (V4 && !UNP), "ingest loads are on the float4 patch path");
  static_assert(!UNP || !V4, "the unpooling loads are on the scalar patch path");
  static_assert(!BF16 || CCH == 32, "bf16 chunks are one 32-deep MFMA K-step");
  using T = typename PatchT<BF16, CCH>::T;
  constexpr int CCP = PatchT<BF16, CCH>::CCP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KK = g.K * g.K;
  T* As = reinterpret_cast<T*>(smem);  // [KK][BM][CCP]
  T* Ps = As + KK * BM * CCP;          // [R][Wp][CCP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r16 = lane & 15, q = lane >> 4;
  const int tile = blockIdx.x;
  const int b = tile / g.tiles, p0 = (tile - b * g.tiles) * g.ppt;
  const int m0 = blockIdx.y * BM;
  const int OHW = g.OH * g.OW;
  const int oy_lo = p0 / g.OW, iy0 = oy_lo - g.pad;

  // this lane's output column (position) and its patch base (lanes past the tile's ppt
  // positions compute a clamped copy and store nothing)
  const int local = wave * 16 + r16;
  const int pn = local < g.ppt ? p0 + local : OHW;
  const int pc = min(p0 + min(local, g.ppt - 1), OHW - 1);
  const int oy = pc / g.OW, ox = pc - oy * g.OW;
  const int bbase = ((oy - oy_lo) * g.Wp + ox) * CCP + (BF16 ? 8 * q : q);

  f32x4 acc[BM / 16];
#pragma unroll
  for (int i = 0; i < BM / 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Staging of one chunk = ONE batch of independent global loads per thread (weights: AV
  // 16-B vectors, patch: PV scalars, flat indices so all 64 lanes of every wave load),
  // held in registers and stored to LDS after the previous chunk's MFMAs; the next
  // chunk's batch is issued right after the barrier, so its latency overlaps the MFMAs.
  // (The earlier row-per-wave staging paid ~8 serial memory latencies per chunk and left
  // lanes >= Wp idle: 36-41 us per 16x16-layer launch.)  Shapes whose chunk exceeds the
  // register batch stage the remainder directly (a slower, still correct path).
  constexpr int VE = 16 / sizeof(T);  // elements per 16-B vector
  constexpr int VPR = CCH / VE;       // vectors per weight row
  constexpr int AV = Batch<CCH>::AV, PV = Batch<CCH>::PV;
  const int nv = KK * BM * VPR;       // weight vectors per chunk
  const int np = g.R * CCH * g.Wp;    // patch elements per chunk: (r, c, xp), xp fastest
  // flat patch index e = tid + i * CT -> (row = r * CCH + c, xp), walked incrementally
  const int dq = CT / g.Wp, dr = CT - dq * g.Wp;
  const int row_t = tid / g.Wp, xp_t = tid - row_t * g.Wp;

  // Per-thread offsets are chunk-invariant and hoisted (32-bit, one VGPR per element);
  // a chunk adds c0.  Patch loads are raw buffer loads over image b: positions in the
  // zero padding, rows past R and channels past C get an offset >= num_records, which the
  // hardware returns as 0 - no per-element exec masks.
  // UNP: x / code are the pooled [C][H/2][W/2] planes; a position's code sits at its float
  // offset / 4, so one offset (and OOB / 4, still >= the code records) serves both loads
  const int PH = g.H >> 1, PW = g.W >> 1;
  const int plane = UNP ? PH * PW : g.H * g.W;
  const int sid = U8 ? in.ids[b] : 0;
  const __amdgpu_buffer_rsrc_t xr =
      U8 ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in.images) + (long)sid * g.C * plane, 0,
                                             g.C * plane, 0x00020000)
         : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x) + (long)b * g.C * plane, 0,
                                             g.C * plane * (int)sizeof(float), 0x00020000);
  if (U8 && tid == 0 && blockIdx.y == 0 && tile == b * g.tiles) in.lab_out[b] = in.labels[sid];
  // U8: x_out of image b (no records for the other M-tiles: their stores are dropped)
  const __amdgpu_buffer_rsrc_t xo = __builtin_amdgcn_make_buffer_rsrc(
      U8 ? in.x_out + (long)b * g.C * plane : nullptr, 0,
      (U8 && blockIdx.y == 0) ? g.C * plane * (int)sizeof(float) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
      UNP ? code + (long)b * g.C * plane : nullptr, 0, UNP ? g.C * plane : 0, 0x00020000);
  constexpr unsigned OOB = 0x80000000u;  // >= num_records for every chunk (C*H*W*4 < 2^31)
  const unsigned cstep = (unsigned)(plane * (int)sizeof(float));  // bytes per channel
  unsigned long long psel = 0;  // UNP: 2-bit position (in its 2x2 window) of patch element i
  // LDS destinations are hoisted too; out-of-range entries go to a dummy slot past the
  // patch (Ps + R*Wp*CCP), so the stores need no exec masks either.
  const int dummy = (int)(Ps - As) + g.R * g.Wp * CCP;
  int aoff[AV], adst[AV], pdst[PV];
  unsigned poff[PV];
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    const int v = min(tid + i * CT, nv - 1);
    const int row = v / VPR, u = v - row * VPR;  // row = tap * BM + m (compile-time divisors)
    const int tap = row / BM, m = row - tap * BM;
    aoff[i] = (tap * g.Mp + m0 + m) * g.Cp + u * VE;
    adst[i] = tid + i * CT < nv ? row * CCP + u * VE : dummy;
  }
  if constexpr (!V4) {
    int row = row_t, xp = xp_t;
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int r = row / CCH, c = row - r * CCH, iy = iy0 + r, ix = xp - g.pad;
      if constexpr (UNP) {
        const bool ok = r < g.R && (unsigned)iy < (unsigned)(2 * PH) && (unsigned)ix < (unsigned)(2 * PW);
        poff[i] = ok ? (unsigned)(((c * PH + (iy >> 1)) * PW + (ix >> 1)) * (int)sizeof(float)) : OOB;
        psel |= (unsigned long long)(((iy & 1) << 1) | (ix & 1)) << (2 * i);
      } else {
        const bool ok = r < g.R && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
        poff[i] = ok ? (unsigned)(((c * g.H + iy) * g.W + ix) * (int)sizeof(float)) : OOB;
      }
      pdst[i] = r < g.R ? (int)(Ps - As) + (r * g.Wp + xp) * CCP + c : dummy;
      xp += dr; row += dq;
      if (xp >= g.Wp) { xp -= g.Wp; ++row; }
    }
  }
  // V4 (W % 4 == 0): the patch moves as float4 groups of 4 image pixels (4x fewer loads and
  // offset computations - the scalar path's per-element address math was ~900 of the
  // kernel's ~1000 VALU instructions per wave); the x-padding columns are zeroed once.
  constexpr int PG = 6;               // float4 groups per thread in the register batch
  const int G = g.W >> 2;             // groups per patch row
  const int ng = V4 ? g.R * CCH * G : 0;
  const unsigned gq0 = V4 ? (unsigned)tid / (unsigned)G : 0u;
  const int gdq = V4 ? CT / G : 0, gdr = V4 ? CT - gdq * G : 0;
  unsigned goff[PG];
  unsigned xoff[U8 ? PG : 1];  // U8: x_out byte offset of group i (OOB: another tile owns its row)
  int gdst[PG];
  if constexpr (V4) {
    unsigned row = gq0;
    int gx = tid - (int)gq0 * G;
    const int t = tile - b * g.tiles;
    const int own_lo = t == 0 ? -(1 << 30) : t * in.own - g.pad;
    const int own_hi = t == g.tiles - 1 ? (1 << 30) : (t + 1) * in.own - g.pad;
#pragma unroll
    for (int i = 0; i < PG; ++i) {
      const unsigned r = row / CCH, c = row & (CCH - 1);
      const int iy = iy0 + (int)r;
      const bool ok = r < (unsigned)g.R && (unsigned)iy < (unsigned)g.H;
      goff[i] = ok ? (unsigned)(((int)c * g.H + iy) * g.W + 4 * gx) * 4u : OOB;
      if constexpr (U8) xoff[i] = (ok && iy >= own_lo && iy < own_hi) ? goff[i] : OOB;
      gdst[i] = r < (unsigned)g.R ? (int)(Ps - As) + ((int)r * g.Wp + 4 * gx + g.pad) * CCP + (int)c : dummy;
      gx += gdr; row += gdq;
      if (gx >= G) { gx -= G; ++row; }
    }
    // x-padding columns: always zero, never written by the group loads
    const int pc = g.Wp - g.W, nz = g.R * pc * CCH;
    for (int e = tid; e < nz; e += CT) {
      const int c = e % CCH, rp = e / CCH, r = rp / pc, k = rp - r * pc;
      Ps[(r * g.Wp + (k < g.pad ? k : g.W + k)) * CCP + c] = (T)0.f;
    }
  }
  // native vector types, not HIP's uint4 / float4 structs: arrays of those were copied to
  // scratch memory (112 B per lane) instead of living in registers
  u32x4 areg[AV];
  float preg[PV];
  unsigned creg[UNP ? PV : 1];
  unsigned ureg[U8 ? PG : 1];  // U8: 4 image bytes per group
  f32x4 greg[PG];
  auto p_val = [&](int row, int xp, int c0) {  // remainder path
    const int r = row / CCH, c = row - r * CCH, iy = iy0 + r, ix = xp - g.pad;
    const bool ok = r < g.R && c0 + c < g.C && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
    return ok ? x[((long)(b * g.C + c0 + c) * g.H + iy) * g.W + ix] : 0.f;
  };
  auto p_store = [&](int row, int xp, float v) {
    const int r = row / CCH, c = row - r * CCH;
    if (r < g.R) Ps[(r * g.Wp + xp) * CCP + c] = (T)v;
  };
  auto load_batch = [&](int c0) {
#pragma unroll
    for (int i = 0; i < AV; ++i) areg[i] = *reinterpret_cast<const u32x4*>(wp + aoff[i] + c0);
    const unsigned cb = (unsigned)c0 * cstep;
    if constexpr (U8) {  // byte offset = float offset / 4 (OOB / 4 is still past the records)
#pragma unroll
      for (int i = 0; i < PG; ++i) ureg[i] = __builtin_amdgcn_raw_buffer_load_b32(xr, (int)((goff[i] + cb) >> 2), 0, 0);
    } else if constexpr (V4) {
#pragma unroll
      for (int i = 0; i < PG; ++i)
        greg[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(goff[i] + cb), 0, 0));
    } else {
#pragma unroll
      for (int i = 0; i < PV; ++i) {
        preg[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)(poff[i] + cb), 0, 0));
        if constexpr (UNP) creg[i] = __builtin_amdgcn_raw_buffer_load_b8(cr, (int)((poff[i] + cb) >> 2), 0, 0);
      }
    }
  };
  auto store_batch = [&](int c0) {
#pragma unroll
    for (int i = 0; i < AV; ++i) *reinterpret_cast<u32x4*>(As + adst[i]) = areg[i];
    if constexpr (U8) {
      const unsigned cb = (unsigned)c0 * cstep, lim = (unsigned)(g.C * plane * (int)sizeof(float));
#pragma unroll
      for (int i = 0; i < PG; ++i) {
        // padding / rows past R / channels past C: 0 (not the normalised value of a 0 byte);
        // torchvision op order with IEEE-rounded division, as ingest_kernel
        const bool inr = goff[i] + cb < lim;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          greg[i][k] = inr ? __fdiv_rn(__fdiv_rn((float)((ureg[i] >> (8 * k)) & 0xffu), 255.0f) - 0.5f, 0.5f) : 0.f;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, greg[i]), xo, (int)(xoff[i] + cb), 0, 0);
      }
    }
    if constexpr (V4) {
#pragma unroll
      for (int i = 0; i < PG; ++i) {
        As[gdst[i]] = (T)greg[i][0];
        As[gdst[i] + CCP] = (T)greg[i][1];
        As[gdst[i] + 2 * CCP] = (T)greg[i][2];
        As[gdst[i] + 3 * CCP] = (T)greg[i][3];
      }
      for (int e = tid + PG * CT; e < ng; e += CT) {  // remainder groups
        const int row = e / G, gx = e - row * G, r = row / CCH, c = row - r * CCH, iy = iy0 + r;
        const bool ok = r < g.R && c0 + c < g.C && (unsigned)iy < (unsigned)g.H;
        const float* src = x + ((long)(b * g.C + c0 + c) * g.H + iy) * g.W + 4 * gx;
        T* dst = Ps + (r * g.Wp + 4 * gx + g.pad) * CCP + c;
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k * CCP] = (T)(ok ? src[k] : 0.f);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PV; ++i) {
        if constexpr (UNP) As[pdst[i]] = (T)(creg[i] == (unsigned)((psel >> (2 * i)) & 3u) ? preg[i] : 0.f);
        else As[pdst[i]] = (T)preg[i];
      }
    }
    // remainder beyond the register batch (large kernels / wide images only)
    for (int v = tid + AV * CT; v < nv; v += CT) {
      const int row = v / VPR, u = v - row * VPR;
      const int tap = row / BM, m = row - tap * BM;
      *reinterpret_cast<u32x4*>(As + row * CCP + u * VE) =
          *reinterpret_cast<const u32x4*>(wp + (tap * g.Mp + m0 + m) * g.Cp + u * VE + c0);
    }
    for (int e = V4 ? np : tid + PV * CT; e < np; e += CT) {
      const int row = e / g.Wp, xp = e - row * g.Wp;
      p_store(row, xp, p_val(row, xp, c0));
    }
  };

  load_batch(0);
  for (int c0 = 0; c0 < g.Cp; c0 += CCH) {
    if (c0) __syncthreads();  // previous chunk's MFMAs are done with As / Ps
    store_batch(c0);
    __syncthreads();
    if (c0 + CCH < g.Cp) load_batch(c0 + CCH);  // in flight during this chunk's MFMAs
    for (int ky = 0; ky < g.K; ++ky) {
      for (int kx = 0; kx < g.K; ++kx) {
        const int tap = ky * g.K + kx;
        const T* pb = Ps + bbase + (ky * g.Wp + kx) * CCP;
        const T* ab = As + (tap * BM + r16) * CCP + (BF16 ? 8 * q : q);
        if constexpr (BF16) {
          const bf16x8 bv = *reinterpret_cast<const bf16x8*>(pb);
#pragma unroll
          for (int i = 0; i < BM / 16; ++i) {
            const bf16x8 av = *reinterpret_cast<const bf16x8*>(ab + 16 * i * CCP);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i], 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < CCH; kk += 4) {
            const float bv = pb[kk];
#pragma unroll
            for (int i = 0; i < BM / 16; ++i)
              acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(ab[16 * i * CCP + kk], bv, acc[i], 0, 0, 0);
          }
        }
      }
    }
  }

  // epilogue: acc[i][j] = D[16 i + 4 q + j][16 wave + r16]
  if constexpr (POOL) {
    __syncthreads();  // every wave is done with As / Ps: the tile's outputs reuse the LDS
    float* ot = reinterpret_cast<float*>(smem);  // [BM][PNT]
#pragma unroll
    for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = 16 * i + 4 * q + j, m = m0 + ml;
        ot[ml * PNT + local] = acc[i][j] + ((bias != nullptr && m < g.M) ? bias[m] : 0.f);
      }
    }
    __syncthreads();
    const int OH2 = g.OH >> 1, OW2 = g.OW >> 1, pr_n = g.rpt >> 1, np = pr_n * OW2;
    const int py0 = (p0 / g.OW) >> 1;
    for (int e = tid; e < BM * np; e += CT) {
      const int ml = e / np, pl = e - ml * np, pr = pl / OW2, px = pl - pr * OW2;
      const int py = py0 + pr, m = m0 + ml;
      if (py >= OH2 || m >= g.M) continue;
      const float* t = ot + ml * PNT + 2 * pr * g.OW + 2 * px;
      float best = t[0];
      int arg = 0;
      const float v1 = t[1], v2 = t[g.OW], v3 = t[g.OW + 1];
      if (v1 > best) { best = v1; arg = 1; }
      if (v2 > best) { best = v2; arg = 2; }
      if (v3 > best) { best = v3; arg = 3; }
      const long o = ((long)(b * g.M + m) * OH2 + py) * OW2 + px;
      y[o] = fmaxf(best, 0.f);
      code[o] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
    }
    return;
  }
  if (pn < OHW) {
#pragma unroll
    for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + 16 * i + 4 * q + j;
        if (m < g.M) y[((long)b * g.M + m) * OHW + pn] = acc[i][j] + (bias != nullptr ? bias[m] : 0.f);
      }
    }
  }
  if constexpr (EPI == EPI_STATS) {
    const int bvalid = state != nullptr ? min(state[ST_BVALID], g.B) : g.B;
    __syncthreads();  // every wave is done with As / Ps: the tile's outputs reuse the LDS
    float* ot = reinterpret_cast<float*>(smem);  // [BM][PNT]
#pragma unroll
    for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = 16 * i + 4 * q + j, m = m0 + ml;
        ot[ml * PNT + local] =
            (pn < OHW && m < g.M) ? acc[i][j] + (bias != nullptr ? bias[m] : 0.f) : 0.f;  // same value as y
      }
    }
    __syncthreads();
    // TPC consecutive threads per channel, PNT / TPC consecutive positions each, then a xor
    // butterfly over the TPC lanes (fixed order; every lane ends with the same fp64 sums)
    constexpr int TPC = CT / BM, PPT = PNT / TPC;
    static_assert(TPC <= 64 && 64 % TPC == 0 && PNT % TPC == 0, "channel group inside one wave");
    const int ml = tid / TPC, pi = tid - ml * TPC;
    double s0 = 0.0, s1 = 0.0;
    if (b < bvalid) {
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const double v = (double)ot[ml * PNT + pi * PPT + k];
        s0 += v;
        s1 += v * v;
      }
    }
#pragma unroll
    for (int off = 1; off < TPC; off <<= 1) {
      s0 += __shfl_xor(s0, off);
      s1 += __shfl_xor(s1, off);
    }
    if (pi == 0 && m0 + ml < g.M) {
      const long P = (long)g.B * g.tiles, o = ((long)(m0 + ml) * P + tile) * 2;
      stats[o] = s0;
      stats[o + 1] = s1;
    }
  }
  if constexpr (EPI == EPI_BNBWD) {
    const int bvalid = state != nullptr ? min(state[ST_BVALID], g.B) : g.B;
    // the BatchNorm input under this lane's outputs (pooled: at the argmax position of each
    // output's window, so the codes are loaded first)
    const int pc_ = min(pn, OHW - 1);
    float zv[BM / 16][4];
    bool onv[BM / 16][4];
    if (bt.code != nullptr) {
      uint8_t cd[BM / 16][4];
#pragma unroll
      for (int i = 0; i < BM / 16; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) cd[i][j] = bt.code[((long)b * g.M + min(m0 + 16 * i + 4 * q + j, g.M - 1)) * OHW + pc_];
      const int py = pc_ / g.OW, px = pc_ - py * g.OW;
#pragma unroll
      for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = min(m0 + 16 * i + 4 * q + j, g.M - 1), c4 = cd[i][j] < 4 ? cd[i][j] : 0;
          zv[i][j] = bt.z[(((long)b * g.M + m) * bt.zH + 2 * py + (c4 >> 1)) * bt.zW + 2 * px + (c4 & 1)];
          onv[i][j] = cd[i][j] < 4;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = min(m0 + 16 * i + 4 * q + j, g.M - 1);
          zv[i][j] = bt.z[((long)b * g.M + m) * OHW + pc_];
          onv[i][j] = __fmaf_rn(__fmul_rn(__fsub_rn(zv[i][j], bt.mean[m]), bt.invstd[m]), bt.gamma[m], bt.beta[m]) > 0.f;
        }
      }
    }
    __syncthreads();  // every wave is done with As / Ps: the tile's terms reuse the LDS
    float* od = reinterpret_cast<float*>(smem);   // [BM][PNT] dz
    float* ox = od + BM * PNT;                    // [BM][PNT] xhat
#pragma unroll
    for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = 16 * i + 4 * q + j, m = min(m0 + ml, g.M - 1);
        const float mu = bt.mean[m], is = bt.invstd[m];
        const bool ok = pn < OHW && m0 + ml < g.M;
        const float dyv = acc[i][j] + (bias != nullptr ? bias[m] : 0.f);
        od[ml * PNT + local] = (ok && onv[i][j]) ? dyv : 0.f;
        ox[ml * PNT + local] = (zv[i][j] - mu) * is;
      }
    }
    __syncthreads();
    constexpr int TPC = CT / BM, PPT = PNT / TPC;
    static_assert(TPC <= 64 && 64 % TPC == 0 && PNT % TPC == 0, "channel group inside one wave");
    const int ml = tid / TPC, pi = tid - ml * TPC;
    double s0 = 0.0, s1 = 0.0;
    if (b < bvalid) {
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const double d = (double)od[ml * PNT + pi * PPT + k];
        s0 += d;
        s1 += d * (double)ox[ml * PNT + pi * PPT + k];
      }
    }
#pragma unroll
    for (int off = 1; off < TPC; off <<= 1) {
      s0 += __shfl_xor(s0, off);
      s1 += __shfl_xor(s1, off);
    }
    if (pi == 0 && m0 + ml < g.M) {
      const long P = (long)g.B * g.tiles, o = ((long)(m0 + ml) * P + tile) * 2;
      stats[o] = s0;
      stats[o + 1] = s1;
    }
  }
}

int pick_bm(int M) { return M <= 16 ? 16 : (M <= 32 ? 32 : 64); }

// LDS budget of the fast path (the default dynamic-LDS limit; >= 2 workgroups per CU)
constexpr size_t kPatchLdsMax = 64 * 1024;

struct FastPlan {
  bool ok = false;
  int bm = 16, gy = 1, cch = 32;
  PGeom pg{};
  size_t lds = 0, ws_bytes = 0;
};

// pool_bm > 0: the plan of the pooled-epilogue variant, with the M tile of the plain plan (the
// packed weight image's Mp must not change)
FastPlan plan_fast(int B, int C, int H, int W, int M, int K, int pad, bool bf, int pool_bm = 0) {
  FastPlan f;
  const int OH = H + 2 * pad - K + 1, OW = W + 2 * pad - K + 1;
  if (OH <= 0 || OW <= 0) return f;
  const int OHW = OH * OW;
  int tiles = (OHW + PNT - 1) / PNT, ppt = PNT, rpt = 0;
  int span = 1;  // most output rows one 64-position tile touches
  if (pool_bm > 0) {  // tiles of rpt whole rows (an even count, rpt * OW <= PNT)
    rpt = 2 * (PNT / (2 * OW));
    if (rpt < 2 || OH < 2) return f;
    ppt = rpt * OW;
    tiles = ((OH & ~1) + rpt - 1) / rpt;
    span = rpt;
  } else {
    for (int t = 0; t < tiles; ++t) {
      const int lo = t * PNT, hi = std::min(OHW, lo + PNT) - 1;
      span = std::max(span, hi / OW - lo / OW + 1);
    }
  }
  const int R = span + K - 1, Wp = W + 2 * pad;
  // M tile: <= 32 rows (enough workgroups on the small late layers), A fits the budget
  int bm = M <= 16 ? 16 : 32;
  const int cch = bf ? 32 : (C <= 8 ? 8 : (C <= 16 ? 16 : 32));
  const size_t es = bf ? 2 : 4, ccp = bf ? 40 : cch + 4;
  auto lds_of = [&](int bmv) { return ((size_t)K * K * bmv + (size_t)R * Wp + 4) * ccp * es; };  // + dummy pixels
  if (lds_of(bm) > kPatchLdsMax && bm == 32) bm = 16;
  if (pool_bm > 0) bm = pool_bm;
  if (lds_of(bm) > kPatchLdsMax) return f;
  f.ok = true;
  f.bm = bm;
  f.cch = cch;
  f.gy = (M + bm - 1) / bm;
  f.pg = PGeom{B, C, H, W, K, pad, OH, OW, M, R, Wp, tiles, (C + cch - 1) / cch * cch, f.gy * bm, ppt, rpt};
  f.lds = std::max(lds_of(bm), pool_bm > 0 ? (size_t)bm * PNT * sizeof(float) : (size_t)0);  // + pooled out tile
  if (f.lds > kPatchLdsMax) f.ok = false;
  f.ws_bytes = (size_t)K * K * f.pg.Mp * f.pg.Cp * es;
  return f;
}

struct EpiArgs {
  uint8_t* code = nullptr;          // EPI_POOL (output) / EPI_UNPOOL (input, unpool = true)
  bool unpool = false;
  double* stats = nullptr;          // EPI_STATS / EPI_BNBWD
  const int32_t* state = nullptr;   // EPI_STATS / EPI_BNBWD
  BnTerms bn{};                     // EPI_BNBWD (bn.z != nullptr)
  const InArgs* in = nullptr;       // U8 ingest loads (float4 path)
};
template <bool BF16, int CCH, bool V4, int EPI, bool U8 = false>
void fast_launch_v(const FastPlan& f, const typename PatchT<BF16, CCH>::T* wp, const float* x, const float* bias,
                   float* y, const EpiArgs& e, hipStream_t s) {
  dim3 grid((unsigned)(f.pg.B * f.pg.tiles), (unsigned)f.gy);
  const InArgs in = e.in ? *e.in : InArgs{};
  if (f.bm == 16)
    hipLaunchKernelGGL((conv_fwd_patch_kernel<BF16, 16, CCH, V4, EPI, U8>), grid, dim3(CT), f.lds, s, x, wp, bias, y,
                       f.pg, e.code, e.stats, e.state, e.bn, in);
  else
    hipLaunchKernelGGL((conv_fwd_patch_kernel<BF16, 32, CCH, V4, EPI, U8>), grid, dim3(CT), f.lds, s, x, wp, bias, y,
                       f.pg, e.code, e.stats, e.state, e.bn, in);
  HIP_CHECK(hipGetLastError());
}
template <bool BF16, int CCH, int EPI>
void fast_launch_e(const FastPlan& f, const typename PatchT<BF16, CCH>::T* wp, const float* x, const float* bias,
                   float* y, const EpiArgs& e, hipStream_t s) {
  if constexpr (EPI != EPI_UNPOOL && EPI != EPI_BNBWD) {
    if (e.in != nullptr) {  // ingest loads (conv_fwd_ingest_ok checked the plan)
      fast_launch_v<BF16, CCH, true, EPI, true>(f, wp, x, bias, y, e, s);
      return;
    }
  }
  // float4 patch groups when image rows are whole 16-B vectors
  if (EPI != EPI_UNPOOL && f.pg.W % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0)
    fast_launch_v<BF16, CCH, EPI != EPI_UNPOOL, EPI>(f, wp, x, bias, y, e, s);
  else fast_launch_v<BF16, CCH, false, EPI>(f, wp, x, bias, y, e, s);
}
// the epilogue follows from the arguments: code -> pooled, stats -> BatchNorm statistics
template <bool BF16, int CCH>
void fast_launch(const FastPlan& f, const typename PatchT<BF16, CCH>::T* wp, const float* x, const float* bias,
                 float* y, hipStream_t s, const EpiArgs& e = EpiArgs{}) {
  if (e.unpool) fast_launch_e<BF16, CCH, EPI_UNPOOL>(f, wp, x, bias, y, e, s);
  else if (e.code != nullptr) fast_launch_e<BF16, CCH, EPI_POOL>(f, wp, x, bias, y, e, s);
  else if (e.stats != nullptr && e.bn.z != nullptr) fast_launch_e<BF16, CCH, EPI_BNBWD>(f, wp, x, bias, y, e, s);
  else if (e.stats != nullptr) fast_launch_e<BF16, CCH, EPI_STATS>(f, wp, x, bias, y, e, s);
  else fast_launch_e<BF16, CCH, EPI_PLAIN>(f, wp, x, bias, y, e, s);
}

template <bool BF16>
void fast_dispatch(const FastPlan& f, const float* x, const float* w, int flip, const float* bias, float* y,
                   void* ws, hipStream_t s) {
  using T = typename std::conditional<BF16, bf16, float>::type;
  const PGeom& g = f.pg;
  T* wp = reinterpret_cast<T*>(ws);
  const int n = g.K * g.K * g.Mp * g.Cp;
  hipLaunchKernelGGL(pack_weights_kernel<T>, dim3(std::max(1, std::min((n + CT - 1) / CT, 1024))), dim3(CT), 0, s, w,
                     g.M, g.C, g.K, g.Mp, g.Cp, flip, wp);
  HIP_CHECK(hipGetLastError());
  if constexpr (BF16) {
    fast_launch<true, 32>(f, wp, x, bias, y, s);
  } else {
    if (f.cch == 8) fast_launch<false, 8>(f, wp, x, bias, y, s);
    else if (f.cch == 16) fast_launch<false, 16>(f, wp, x, bias, y, s);
    else fast_launch<false, 32>(f, wp, x, bias, y, s);
  }
}

template <bool BF16>
void fwd_dispatch(const float* x, const float* w, const float* bias, float* y, const Geom& g, int M, hipStream_t s) {
  const long N = (long)g.B * g.OH * g.OW;
  const int bm = pick_bm(M);
  dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((M + bm - 1) / bm));
  if (bm == 16) hipLaunchKernelGGL((conv_fwd_kernel<BF16, 16>), grid, dim3(CT), 0, s, x, w, bias, y, g, M);
  else if (bm == 32) hipLaunchKernelGGL((conv_fwd_kernel<BF16, 32>), grid, dim3(CT), 0, s, x, w, bias, y, g, M);
  else hipLaunchKernelGGL((conv_fwd_kernel<BF16, 64>), grid, dim3(CT), 0, s, x, w, bias, y, g, M);
  HIP_CHECK(hipGetLastError());
}

template <bool BF16, bool UNPOOL>
void wgrad_dispatch_u(const float* x, const float* dy, float* part, const Geom& g, int M, int S, int cps,
                      const uint8_t* code, hipStream_t s) {
  const int Kd = g.C * g.K * g.K;
  const int bm = pick_bm(M);
  dim3 grid((unsigned)((Kd + 1 + BN - 1) / BN), (unsigned)((M + bm - 1) / bm), (unsigned)S);  // + bias column
  if (bm == 16)
    hipLaunchKernelGGL((conv_wgrad_kernel<BF16, 16, UNPOOL>), grid, dim3(CT), 0, s, x, dy, part, g, M, cps, code);
  else if (bm == 32)
    hipLaunchKernelGGL((conv_wgrad_kernel<BF16, 32, UNPOOL>), grid, dim3(CT), 0, s, x, dy, part, g, M, cps, code);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<BF16, 64, UNPOOL>), grid, dim3(CT), 0, s, x, dy, part, g, M, cps, code);
  HIP_CHECK(hipGetLastError());
}
template <bool BF16>
void wgrad_dispatch(const float* x, const float* dy, float* part, const Geom& g, int M, int S, int cps,
                    const uint8_t* code, hipStream_t s) {
  if (code != nullptr) wgrad_dispatch_u<BF16, true>(x, dy, part, g, M, S, cps, code, s);
  else wgrad_dispatch_u<BF16, false>(x, dy, part, g, M, S, cps, nullptr, s);
}

Geom geom(int B, int C, int H, int W, int K, int pad) {
  Geom g{B, C, H, W, K, pad, H + 2 * pad - K + 1, W + 2 * pad - K + 1};
  if (B <= 0 || C <= 0 || K <= 0 || pad < 0 || g.OH <= 0 || g.OW <= 0)
    throw std::runtime_error("conv_igemm: invalid geometry");
  if ((long)B * C * H * W >= (1L << 31) || (long)B * g.OH * g.OW >= (1L << 31))
    throw std::runtime_error("conv_igemm: tensor too large for 32-bit gather offsets");
  return g;
}
}  // namespace

// Workspace bytes of launch_conv_fwd: the packed weights of the fast path, or the flipped
// fp32 weights of the general path's dgrad (flip), else 0.
size_t conv_fwd_workspace(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, int flip) {
  const FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  if (f.ok) return f.ws_bytes;
  return flip ? (size_t)M * C * K * K * sizeof(float) : 0;
}

// y = conv(x, w) + bias.  flip = 0: w is [M][C][K][K] (forward).  flip = 1: w is the
// forward weight [C][M][K][K] of the layer whose data gradient this computes (the kernel
// flips and transposes it while packing).  ws: conv_fwd_workspace() bytes.
void launch_conv_fwd(const float* x, const float* w, const float* bias, float* y, void* ws, int B, int C, int H, int W,
                     int M, int K, int pad, int bf16_ops, int flip, hipStream_t s) {
  const Geom g = geom(B, C, H, W, K, pad);
  const FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  if (f.ok) {
    if (bf16_ops) fast_dispatch<true>(f, x, w, flip, bias, y, ws, s);
    else fast_dispatch<false>(f, x, w, flip, bias, y, ws, s);
    return;
  }
  const float* wf = w;
  if (flip) {  // general path: materialise the flipped weights [M][C][K][K] in the workspace
    launch_flip_weights(w, C, M, K, reinterpret_cast<float*>(ws), s);
    wf = reinterpret_cast<const float*>(ws);
  }
  if (bf16_ops) fwd_dispatch<true>(x, wf, bias, y, g, M, s);
  else fwd_dispatch<false>(x, wf, bias, y, g, M, s);
}

// 1 when (B, C, H, W, M, K, pad, bf16) runs on the LDS-patch fast path (tests / profiling)
int conv_fwd_fast(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
  return plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0).ok ? 1 : 0;
}

long env_long(const char* name, long dflt) {
  const char* v = std::getenv(name);
  return (v != nullptr && *v != '\0') ? std::max(1L, std::atol(v)) : dflt;
}

// slices for the wgrad split: enough workgroups to fill the chip, >= 4 chunks per slice
void conv_wgrad_split(int B, int C, int H, int W, int M, int K, int pad, int* S, int* cps) {
  const Geom g = geom(B, C, H, W, K, pad);
  const long R = (long)B * g.OH * g.OW;
  const long chunks = (R + BK - 1) / BK;
  const int Kd = C * K * K, bm = pick_bm(M);
  const long tiles = (long)((Kd + 1 + BN - 1) / BN) * ((M + bm - 1) / bm);
  // ~2048 workgroups (8 per CU: a slice's chunks run back to back, so the chip must be
  // full), at most 512 slices (the slice sum reads S partials per element), at least 2
  // chunks per slice.  (A 64-slice cap left conv1's single tile with 64 workgroups of
  // 16 serial chunks each: 45 us; 1024 / 256 / 4 -> 2048 / 512 / 2 took lenet 91.6 -> 84.7 us,
  // cifar-vgg bf16 300.6 -> 296.3 us per step: profiles/r2/layer_fusion/wsplit/.)
  // (DNN_WGRAD_WGS / _MAX_SLICES / _MIN_CHUNKS override the three numbers: tuning runs)
  static const long wgs = env_long("DNN_WGRAD_WGS", 2048), max_s = env_long("DNN_WGRAD_MAX_SLICES", 512),
                    min_c = env_long("DNN_WGRAD_MIN_CHUNKS", 2),
                    max_kb = env_long("DNN_WGRAD_MAX_PART_KB", 1L << 30);  // partial bytes cap per layer
  const long slice_kb = std::max(1L, (long)M * (Kd + 1) * 4 / 1024);
  long want = std::max(1L, wgs / std::max(1L, tiles));
  want = std::min({want, max_s, std::max(1L, chunks / min_c), std::max(1L, max_kb / slice_kb)});
  const long per = (chunks + want - 1) / want;
  *cps = (int)per;
  *S = (int)((chunks + per - 1) / per);
}

// dw [M][C][K][K] and db [M] from one MFMA pass; part: S * M * (C K^2 + 1) floats.  dw == nullptr:
// the slice partials only (the caller sums them later, e.g. inside the SGD tail launch).
// pool_code != nullptr: dy is the pooled gradient of a fused conv + ReLU + max-pool (see UNPOOL)
void launch_conv_wgrad(const float* x, const float* dy, float* part, float* dw, float* db, int B, int C, int H, int W,
                       int M, int K, int pad, int bf16_ops, hipStream_t s, const uint8_t* pool_code) {
  const Geom g = geom(B, C, H, W, K, pad);
  int S = 1, cps = 1;
  conv_wgrad_split(B, C, H, W, M, K, pad, &S, &cps);
  if (pool_code != nullptr && (g.OH < 2 || g.OW < 2)) throw std::runtime_error("conv_wgrad: pooled dy of a < 2x2 map");
  if ((long)B * C * H * W * 4 >= (1L << 31) || (long)B * M * g.OH * g.OW * 4 >= (1L << 31))
    throw std::runtime_error("conv_wgrad: tensor too large for 32-bit buffer offsets");
  if (bf16_ops) wgrad_dispatch<true>(x, dy, part, g, M, S, cps, pool_code, s);
  else wgrad_dispatch<false>(x, dy, part, g, M, S, cps, pool_code, s);
  if (dw == nullptr) return;
  const int Kd = C * K * K;
  const long n = (long)M * (Kd + 1);
  hipLaunchKernelGGL(slice_sum_kernel, dim3((unsigned)((n + 63) / 64)), dim3(SW * 64), 0, s, part, S, n, Kd, dw, db);
  HIP_CHECK(hipGetLastError());
}

namespace {
constexpr int kMaxPack = 16;
struct PackItem {
  const float* w;
  void* dst;
  int M, C, K, Mp, Cp, flip, bf;
};
struct PackSet {
  PackItem it[kMaxPack];
  int start[kMaxPack + 1];  // element prefix sums
  int n;
};

// every job's packed image in one grid-stride launch (same element map as pack_weights_kernel)
__global__ void __launch_bounds__(CT) pack_multi_kernel(const PackSet ps) {
  const int total = ps.start[ps.n];
  for (int e = blockIdx.x * CT + threadIdx.x; e < total; e += gridDim.x * CT) {
    int j = 0;
    while (j + 1 < ps.n && e >= ps.start[j + 1]) ++j;
    const PackItem& p = ps.it[j];
    const int l = e - ps.start[j];
    const int c = l % p.Cp, m = (l / p.Cp) % p.Mp, tap = l / (p.Cp * p.Mp);
    const int ky = tap / p.K, kx = tap - ky * p.K;
    float v = 0.f;
    if (m < p.M && c < p.C)
      v = p.flip ? p.w[((c * p.M + m) * p.K + (p.K - 1 - ky)) * p.K + (p.K - 1 - kx)]
                 : p.w[((m * p.C + c) * p.K + ky) * p.K + kx];
    if (p.bf) reinterpret_cast<bf16*>(p.dst)[l] = (bf16)v;
    else reinterpret_cast<float*>(p.dst)[l] = v;
  }
}
}  // namespace

void launch_conv_pack_all(const ConvPackJob* jobs, int n, hipStream_t s) {
  for (int j0 = 0; j0 < n; j0 += kMaxPack) {
    PackSet ps{};
    ps.n = std::min(kMaxPack, n - j0);
    ps.start[0] = 0;
    for (int j = 0; j < ps.n; ++j) {
      const ConvPackJob& J = jobs[j0 + j];
      const FastPlan f = plan_fast(J.B, J.C, J.H, J.W, J.M, J.K, J.pad, J.bf16_ops != 0);
      if (!f.ok) throw std::runtime_error("conv_pack_all: layer is not on the LDS-patch path");
      // (forward: w is [M][C][K][K]; flip: w is the layer's [C][M][K][K], as in launch_conv_fwd)
      ps.it[j] = PackItem{J.w, J.dst, f.pg.M, f.pg.C, f.pg.K, f.pg.Mp, f.pg.Cp, J.flip, J.bf16_ops != 0};
      ps.start[j + 1] = ps.start[j] + f.pg.K * f.pg.K * f.pg.Mp * f.pg.Cp;
    }
    const int total = ps.start[ps.n];
    hipLaunchKernelGGL(pack_multi_kernel, dim3(std::max(1, std::min((total + CT - 1) / CT, 2048))), dim3(CT), 0, s,
                       ps);
    HIP_CHECK(hipGetLastError());
  }
}

void conv_pack_geometry(const ConvPackJob& J, int* M, int* C, int* K, int* Mp, int* Cp) {
  const FastPlan f = plan_fast(J.B, J.C, J.H, J.W, J.M, J.K, J.pad, J.bf16_ops != 0);
  if (!f.ok) throw std::runtime_error("conv_pack_geometry: layer is not on the LDS-patch path");
  *M = f.pg.M; *C = f.pg.C; *K = f.pg.K; *Mp = f.pg.Mp; *Cp = f.pg.Cp;
}

void launch_conv_fwd_packed(const float* x, const void* wp, const float* bias, float* y, int B, int C, int H, int W,
                            int M, int K, int pad, int bf16_ops, hipStream_t s) {
  geom(B, C, H, W, K, pad);
  const FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  if (!f.ok) throw std::runtime_error("conv_fwd_packed: layer is not on the LDS-patch path");
  if (bf16_ops) {
    fast_launch<true, 32>(f, reinterpret_cast<const bf16*>(wp), x, bias, y, s);
  } else {
    const float* w = reinterpret_cast<const float*>(wp);
    if (f.cch == 8) fast_launch<false, 8>(f, w, x, bias, y, s);
    else if (f.cch == 16) fast_launch<false, 16>(f, w, x, bias, y, s);
    else fast_launch<false, 32>(f, w, x, bias, y, s);
  }
}

void fast_launch_packed(const FastPlan& f, const void* wp, const float* x, const float* bias, float* y, int bf16_ops,
                        const EpiArgs& e, hipStream_t s) {
  if (bf16_ops) {
    fast_launch<true, 32>(f, reinterpret_cast<const bf16*>(wp), x, bias, y, s, e);
  } else {
    const float* w = reinterpret_cast<const float*>(wp);
    if (f.cch == 8) fast_launch<false, 8>(f, w, x, bias, y, s, e);
    else if (f.cch == 16) fast_launch<false, 16>(f, w, x, bias, y, s, e);
    else fast_launch<false, 32>(f, w, x, bias, y, s, e);
  }
}

// the pooled plan of a layer whose plain plan packed the weight image (same M tile)
FastPlan plan_pool(int B, int C, int H, int W, int M, int K, int pad, bool bf) {
  const FastPlan f0 = plan_fast(B, C, H, W, M, K, pad, bf);
  if (!f0.ok) return f0;
  return plan_fast(B, C, H, W, M, K, pad, bf, f0.bm);
}

int conv_fwd_pool_ok(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
  return plan_pool(B, C, H, W, M, K, pad, bf16_ops != 0).ok ? 1 : 0;
}

// y = maxpool2x2(relu(conv(x, w) + bias)) and its argmax codes, from the layer's packed image
void launch_conv_fwd_packed_pool(const float* x, const void* wp, const float* bias, float* y, uint8_t* code, int B,
                                 int C, int H, int W, int M, int K, int pad, int bf16_ops, hipStream_t s) {
  geom(B, C, H, W, K, pad);
  const FastPlan f = plan_pool(B, C, H, W, M, K, pad, bf16_ops != 0);
  if (!f.ok) throw std::runtime_error("conv_fwd_packed_pool: layer has no pooled LDS-patch plan");
  EpiArgs e;
  e.code = code;
  fast_launch_packed(f, wp, x, bias, y, bf16_ops, e, s);
}

// EPI_UNPOOL: the scalar patch path with every element of a chunk in the register batch
int conv_fwd_unpool_ok(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
  const FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  if (!f.ok || H < 2 || W < 2) return 0;
  const int pv = bf16_ops ? Batch<32>::PV : (f.cch == 8 ? Batch<8>::PV : (f.cch == 16 ? Batch<16>::PV : Batch<32>::PV));
  return (long)f.pg.R * f.cch * f.pg.Wp <= (long)pv * CT ? 1 : 0;
}

// y = conv(unpool(x, code), w) + bias from the packed image: x [B][C][H/2][W/2] is the pooled
// gradient of a ReLU + max-pool with argmax codes `code` (EPI_UNPOOL); H, W the unpooled size
void launch_conv_fwd_packed_unpool(const float* x, const uint8_t* code, const void* wp, float* y, int B, int C, int H,
                                   int W, int M, int K, int pad, int bf16_ops, hipStream_t s) {
  geom(B, C, H, W, K, pad);
  if (!conv_fwd_unpool_ok(B, C, H, W, M, K, pad, bf16_ops))
    throw std::runtime_error("conv_fwd_packed_unpool: layer has no unpooling LDS-patch plan");
  const FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  EpiArgs e;
  e.code = const_cast<uint8_t*>(code);
  e.unpool = true;
  fast_launch_packed(f, wp, x, nullptr, y, bf16_ops, e, s);
}

// U8 ingest loads: plan of the epilogue (epi 0 plain, 1 pooled, 2 BatchNorm statistics) with
// float4 rows, every chunk in the register batch, row-aligned tiles and every input row inside
// some tile's patch; returns the rows each tile owns (0: not possible)
static int ingest_plan(int B, int C, int H, int W, int M, int K, int pad, bool bf, int epi, FastPlan* out) {
  const FastPlan f = epi == 1 ? plan_pool(B, C, H, W, M, K, pad, bf) : plan_fast(B, C, H, W, M, K, pad, bf);
  if (!f.ok || W % 4 != 0) return 0;
  const PGeom& g = f.pg;
  if ((long)g.R * f.cch * (W / 4) > 6L * CT) return 0;  // PG groups per thread
  int own;
  if (epi == 1) {
    own = g.rpt;
  } else {
    if (g.ppt % g.OW != 0 || (g.OH * g.OW) % g.ppt != 0) return 0;
    own = g.ppt / g.OW;
  }
  // the last tile's patch must reach the last input row
  if ((g.tiles - 1) * own - pad + g.R < H) return 0;
  if (out) *out = f;
  return own;
}

int conv_fwd_ingest_ok(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, int epi) {
  return ingest_plan(B, C, H, W, M, K, pad, bf16_ops != 0, epi, nullptr) > 0 ? 1 : 0;
}

// The first conv of a training step with the ingest folded in: y (+ pooled codes / BatchNorm
// statistics partials) from the u8 images of the batch's sample ids; also stores the
// normalised input x_out [B][C][H][W] and the labels (see InArgs)
void launch_conv_fwd_packed_ingest(const uint8_t* images, const int32_t* ids, const int32_t* labels, float* x_out,
                                   int32_t* lab_out, const void* wp, const float* bias, float* y, uint8_t* code,
                                   double* stats, const int32_t* state, int B, int C, int H, int W, int M, int K,
                                   int pad, int bf16_ops, hipStream_t s) {
  geom(B, C, H, W, K, pad);
  const int epi = code != nullptr ? 1 : (stats != nullptr ? 2 : 0);
  FastPlan f;
  const int own = ingest_plan(B, C, H, W, M, K, pad, bf16_ops != 0, epi, &f);
  if (own == 0) throw std::runtime_error("conv_fwd_packed_ingest: layer has no ingest plan");
  if (epi == 2) f.lds = std::max(f.lds, (size_t)f.bm * PNT * sizeof(float));  // the statistics' output tile
  const InArgs in{images, ids, labels, x_out, lab_out, own};
  EpiArgs e;
  e.code = code;
  e.stats = stats;
  e.state = state;
  e.in = &in;
  fast_launch_packed(f, wp, nullptr, bias, y, bf16_ops, e, s);
}

int conv_fwd_stat_parts(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
  const FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  return f.ok ? f.pg.B * f.pg.tiles : 0;
}

// y = conv(x, w) + bias from the packed image, plus the BatchNorm statistics partials of y
// (stats: M * conv_fwd_stat_parts() * 2 doubles; see EPI_STATS)
void launch_conv_fwd_packed_stats(const float* x, const void* wp, const float* bias, float* y, double* stats,
                                  const int32_t* state, int B, int C, int H, int W, int M, int K, int pad, int bf16_ops,
                                  hipStream_t s) {
  geom(B, C, H, W, K, pad);
  FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  if (!f.ok) throw std::runtime_error("conv_fwd_packed_stats: layer is not on the LDS-patch path");
  f.lds = std::max(f.lds, (size_t)f.bm * PNT * sizeof(float));  // the epilogue's output tile
  EpiArgs e;
  e.stats = stats;
  e.state = state;
  fast_launch_packed(f, wp, x, bias, y, bf16_ops, e, s);
}

// data gradient (packed flipped image of the next conv) whose output y is the gradient of a
// BatchNorm + ReLU output, plus that BatchNorm's backward-statistics partials (EPI_BNBWD)
void launch_conv_fwd_packed_bnbwd(const float* x, const void* wp, float* y, double* stats, const int32_t* state,
                                  const float* bn_z, const float* bn_mean, const float* bn_invstd,
                                  const float* bn_gamma, const float* bn_beta, const uint8_t* bn_code, int zH, int zW,
                                  int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, hipStream_t s) {
  const Geom gg = geom(B, C, H, W, K, pad);
  if (bn_code == nullptr ? (zH != gg.OH || zW != gg.OW) : (zH / 2 != gg.OH || zW / 2 != gg.OW))
    throw std::runtime_error("conv_fwd_packed_bnbwd: BatchNorm map does not match the data-gradient grid");
  FastPlan f = plan_fast(B, C, H, W, M, K, pad, bf16_ops != 0);
  if (!f.ok) throw std::runtime_error("conv_fwd_packed_bnbwd: layer is not on the LDS-patch path");
  f.lds = std::max(f.lds, (size_t)2 * f.bm * PNT * sizeof(float));  // the epilogue's dz / xhat tiles
  EpiArgs e;
  e.stats = stats;
  e.state = state;
  e.bn = BnTerms{bn_z, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_code, zH, zW};
  fast_launch_packed(f, wp, x, nullptr, y, bf16_ops, e, s);
}

void launch_flip_weights(const float* w, int O, int C, int K, float* wf, hipStream_t s) {
  const int n = O * C * K * K;
  hipLaunchKernelGGL(flip_weights_kernel, dim3(std::max(1, std::min((n + CT - 1) / CT, 1024))), dim3(CT), 0, s, w, O,
                     C, K, wf);
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

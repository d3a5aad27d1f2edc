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
//   wgrad   : dW[m][j]   = sum_r dY[m][r] * im2col(x)[j][r],  r = (b, p)  (B*OH*OW long):
//             split over S workgroup slices into fp32 partials, then a fixed-order sum
//             (deterministic, no float atomics)
//
// Tiling: a workgroup (4 waves) owns a BM x 64 output tile (BM = 16/32/64 from M); wave w
// owns columns [16 w, 16 w + 16) and all BM rows as BM/16 16x16 accumulators.  The
// reduction runs in 64-wide chunks staged through LDS in k-contiguous rows, so every MFMA
// operand is one LDS read: fp32 -> v_mfma_f32_16x16x4_f32 (16 per chunk, exact fp32
// products), bf16 -> v_mfma_f32_16x16x32_bf16 (2 per chunk, one ds_read_b128 per operand).
// The next chunk's global gathers are issued before the current chunk's MFMAs (register
// prefetch), so their latency overlaps the math and the other resident workgroups.
#include <algorithm>
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
// kernels' dominant VALU cost).
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
    v[e] = in ? x[off] : 0.f;
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
template <bool BF16, int BM>
__global__ void __launch_bounds__(CT) conv_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        float* __restrict__ part, Geom g, int M, int chunks_per_slice) {
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

  // both tiles: lanes along BK consecutive r (contiguous positions), KPT rows per thread
  const int rl = tid & 63, rowg = (tid >> 6) * KPT;

  f32x4 acc[BM / 16];
#pragma unroll
  for (int i = 0; i < BM / 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  float av[KPT], bv[KPT];
  auto load = [&](long r0) {
    const long r = r0 + rl;
    const bool rv = r < r_end;
    const long rc = rv ? r : r_end - 1;
    const int bb = (int)(rc / OHW), p = (int)(rc % OHW), oy = p / g.OW, ox = p % g.OW;
    const float* dyb = dy + (long)bb * M * OHW + p;
#pragma unroll
    for (int e = 0; e < KPT; ++e) {
      const int m = m0 + rowg + e;
      const bool mv = rowg + e < BM && m < M;
      const float a = dyb[(long)(mv ? m : 0) * OHW];
      av[e] = (mv && rv) ? a : 0.f;
    }
    gather_rows(x, g, j0 + rowg, Kd, bb, oy, ox, rv, bv);
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
  if (j < Kd) {
#pragma unroll
    for (int i = 0; i < BM / 16; ++i) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int m = m0 + 16 * i + 4 * q + jj;
        if (m < M) part[((long)s * M + m) * Kd + j] = acc[i][jj];
      }
    }
  }
}

// dw[e] = sum_s part[s][e] in a fixed order (deterministic).  A workgroup owns 64
// consecutive elements; wave w sums slices w, w+4, w+8, ... (8 loads in flight per
// batch), then wave 0 adds the four wave sums in order.  Grid = n / 64 workgroups: the
// earlier one-thread-per-element loop over all S slices was latency-bound at 26-56 us.
__global__ void __launch_bounds__(CT) slice_sum_kernel(const float* __restrict__ part, int S, long n,
                                                       float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + lane;
  const bool ev = e < n;
  const float* p = part + (ev ? e : 0);
  float acc = 0.f;
  for (int s0 = wave; s0 < S; s0 += 32) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = s0 + 4 * u;
      v[u] = s < S ? p[(long)s * n] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && ev) out[e] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
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

int pick_bm(int M) { return M <= 16 ? 16 : (M <= 32 ? 32 : 64); }

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

template <bool BF16>
void wgrad_dispatch(const float* x, const float* dy, float* part, const Geom& g, int M, int S, int cps, hipStream_t s) {
  const int Kd = g.C * g.K * g.K;
  const int bm = pick_bm(M);
  dim3 grid((unsigned)((Kd + BN - 1) / BN), (unsigned)((M + bm - 1) / bm), (unsigned)S);
  if (bm == 16) hipLaunchKernelGGL((conv_wgrad_kernel<BF16, 16>), grid, dim3(CT), 0, s, x, dy, part, g, M, cps);
  else if (bm == 32) hipLaunchKernelGGL((conv_wgrad_kernel<BF16, 32>), grid, dim3(CT), 0, s, x, dy, part, g, M, cps);
  else hipLaunchKernelGGL((conv_wgrad_kernel<BF16, 64>), grid, dim3(CT), 0, s, x, dy, part, g, M, cps);
  HIP_CHECK(hipGetLastError());
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

void launch_conv_fwd(const float* x, const float* w, const float* bias, float* y, int B, int C, int H, int W, int M,
                     int K, int pad, int bf16_ops, hipStream_t s) {
  const Geom g = geom(B, C, H, W, K, pad);
  if (bf16_ops) fwd_dispatch<true>(x, w, bias, y, g, M, s);
  else fwd_dispatch<false>(x, w, bias, y, g, M, s);
}

// slices for the wgrad split: enough workgroups to fill the chip, >= 4 chunks per slice
void conv_wgrad_split(int B, int C, int H, int W, int M, int K, int pad, int* S, int* cps) {
  const Geom g = geom(B, C, H, W, K, pad);
  const long R = (long)B * g.OH * g.OW;
  const long chunks = (R + BK - 1) / BK;
  const int Kd = C * K * K, bm = pick_bm(M);
  const long tiles = (long)((Kd + BN - 1) / BN) * ((M + bm - 1) / bm);
  // ~512 workgroups, at most 64 slices (the fixed-order slice sum reads S partials per
  // element), at least 2 chunks per slice
  long want = std::max(1L, 512 / std::max(1L, tiles));
  want = std::min({want, 64L, std::max(1L, chunks / 2)});
  const long per = (chunks + want - 1) / want;
  *cps = (int)per;
  *S = (int)((chunks + per - 1) / per);
}

void launch_conv_wgrad(const float* x, const float* dy, float* part, float* dw, int B, int C, int H, int W, int M,
                       int K, int pad, int bf16_ops, hipStream_t s) {
  const Geom g = geom(B, C, H, W, K, pad);
  int S = 1, cps = 1;
  conv_wgrad_split(B, C, H, W, M, K, pad, &S, &cps);
  if (bf16_ops) wgrad_dispatch<true>(x, dy, part, g, M, S, cps, s);
  else wgrad_dispatch<false>(x, dy, part, g, M, S, cps, s);
  const long n = (long)M * C * K * K;
  hipLaunchKernelGGL(slice_sum_kernel, dim3((unsigned)((n + 63) / 64)), dim3(CT), 0, s, part, S, n, dw);
  HIP_CHECK(hipGetLastError());
}

void launch_flip_weights(const float* w, int O, int C, int K, float* wf, hipStream_t s) {
  const int n = O * C * K * K;
  hipLaunchKernelGGL(flip_weights_kernel, dim3(std::max(1, std::min((n + CT - 1) / CT, 1024))), dim3(CT), 0, s, w, O,
                     C, K, wf);
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

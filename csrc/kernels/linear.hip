// Linear layers of the generic layer engine on MFMA (gfx950): forward, data gradient and
// weight + bias gradient of y = x W^T + b, with an optional fused ReLU.
//
// Capability parity: aten::addmm / mm / sum(dim 0) / relu / threshold_backward of the fc layers
//  for any zoo model (lenet: 400-120-84-10, cifar-vgg:
// 4096-256-10) at batch B.  These GEMMs are tiny (B = 64 rows), so the library GEMM picked
// single-workgroup tiles that ran 5-19 us each (profiles/r2/linear/); here every 16 x 16
// output tile is its own workgroup, the reduction is split over up to 16 waves of it and
// summed in a fixed order through LDS (deterministic, no atomics), and every operand load of a
// 16-step batch is in flight before its first MFMA.
//
//   forward : y[b][n]  = act(sum_k x[b][k] W[n][k] + bias[n])        act = ReLU if relu
//   dgrad   : dx[b][k] = sum_n dz[b][n] W[n][k]                       dz = dy * (y > 0) if relu
//   wgrad   : dW[n][k] = sum_b dz[b][n] x[b][k],  db[n] = sum_b dz[b][n]  (the "ones" column k = K)
//
// All three are C[M][N] = sum_k A(m, k) B(k, n) on v_mfma_f32_16x16x4_f32 (exact fp32
// products, fp32 accumulation: the layer engine's Linear math stays fp32 in both dtype modes)
// with strided operand views; A may carry the ReLU mask of a saved activation.
#include <algorithm>
#include <cstdint>
#include <stdexcept>

#include "launchers.h"

namespace dnn {
namespace {

constexpr int LIN_MAX_WAVES = 16;

struct GemmArgs {
  const float* a;  long a_m, a_k;   // A(m, k) = a[m * a_m + k * a_k]
  const float* am;                  // optional ReLU mask source: A(m, k) *= (am[same index] > 0)
  const float* b;  long b_k, b_n;   // B(k, n) = b[k * b_k + n * b_n];  n == ones_col -> 1
  float* c;        long c_m;        // C[m][n] = c[m * c_m + n] for n < N
  float* c_ones;                    // C[m][ones_col] -> c_ones[m]  (bias gradient)
  const float* bias;                // + bias[n]
  int M, N, K, ones_col;            // ones_col = -1: none
  int relu;                         // forward: ReLU on the output
  int kpw;                          // reduction elements per wave (multiple of 64)
  int ncols;                        // output columns incl. the ones column (set by prepare)
  // fused softmax cross-entropy on the forward output (logits; N <= 16 classes, one column tile)
  const int32_t* labels;            // [M]
  const int32_t* state;             // device step state: samples >= state[ST_BVALID] are padding
  float* loss;                      // [M] per-sample loss (0 for padding)
  int32_t* correct;                 // [M] argmax == label (first maximum wins, like torch.argmax)
  float* dlogits;                   // [M][N] (softmax - onehot) / valid samples (0 for padding)
};

// Softmax cross-entropy of the 4 rows m = m0 + 4 kq + r of a logits tile (n0 = 0, N <= 16): the
// 16 lanes of a kq group hold one row, so its max / first argmax / exp-sum are butterfly
// reductions over those lanes (xor shuffles: every lane ends with the bit-identical value -
// fp32 max and add are commutative).  Loss = max + log(sum exp) - z[label]; the whole wave
// runs this (no lane leaves before a shuffle).
__device__ __forceinline__ void xent_rows(const GemmArgs& g, const f32x4& sum, const int (&lab)[4], int bvalid, int m0,
                                          int i, int kq, int lane) {
  const bool nv = i < g.N;
  const float bias = (g.bias != nullptr && nv) ? g.bias[i] : 0.f;
  const float inv = bvalid > 0 ? 1.f / (float)bvalid : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mm = m0 + 4 * kq + r;
    const float z = nv ? sum[r] + bias : -INFINITY;
    float mx = z;
    int am = nv ? i : 16;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const float o = __shfl_xor(mx, off);
      const int oa = __shfl_xor(am, off);
      if (o > mx || (o == mx && oa < am)) { mx = o; am = oa; }
    }
    const float e = nv ? expf(z - mx) : 0.f;
    float se = e;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) se += __shfl_xor(se, off);
    const int y = lab[r];
    const float zy = __shfl(z, (lane & ~15) | (y & 15));
    if (mm < g.M) {
      const bool valid = mm < bvalid;
      if (nv) {
        g.c[(long)mm * g.c_m + i] = z;
        g.dlogits[(long)mm * g.N + i] = valid ? (e / se - (i == y ? 1.f : 0.f)) * inv : 0.f;
      }
      if (i == 0) {
        g.loss[mm] = valid ? mx + logf(se) - zy : 0.f;
        g.correct[mm] = (valid && am == y) ? 1 : 0;
      }
    }
  }
}

// one 16 x 16 output tile per workgroup; wave w reduces k in [w kpw, (w + 1) kpw).  Every
// operand load of a 16-step batch is unconditional (clamped, in-bounds address) and issued
// before the first MFMA; out-of-range and masked operands are zeroed by selects afterwards
// (a load under a per-element branch made the compiler wait for it at the branch join:
// 16-32 serial memory latencies per batch).  MASK: A is multiplied by (am > 0).  XENT: the
// tile holds whole rows of logits and wave 0 finishes the softmax cross-entropy (forward and
// backward) of its 16 samples in the epilogue (see xent_rows).
//
// VEC (forward: A = x rows and B = W rows both contiguous along k, K % 4 == 0, 16-B aligned): lane
// (i, kq) takes the 16 CONSECUTIVE k = k0 + 16 kq + s of its rows instead of k = k0 + 4 s + kq, so
// its operands are 4 + 4 dwordx4 loads (the strided mapping issued 32 scalar loads of 16 rows x
// 16 B each); the k order inside an MFMA chain is a permutation of the same sum.
template <bool MASK, bool XENT = false, bool VEC = false>
__device__ __forceinline__ void small_gemm_tile(const GemmArgs& g, f32x4* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 16;
  if (m0 >= g.M || n0 >= g.ncols) return;  // whole workgroup: outside this GEMM's tile grid
  const int m = m0 + i, n = n0 + i;
  const bool mv = m < g.M, nv = n < g.N, ones = n == g.ones_col;
  const long ma = (long)min(m, g.M - 1) * g.a_m, nb = (long)min(n, g.N - 1) * g.b_n;
  const int k_lo = wave * g.kpw, k_hi = min(g.K, k_lo + g.kpw);
  // XENT: the step state and the 4 labels of this lane's rows are in flight with the operands
  int bvalid = g.M, lab[4] = {0, 0, 0, 0};
  if constexpr (XENT) {
    if (wave == 0) {
      bvalid = g.state != nullptr ? min(g.state[ST_BVALID], g.M) : g.M;
#pragma unroll
      for (int r = 0; r < 4; ++r) lab[r] = g.labels[min(m0 + 4 * kq + r, g.M - 1)];
    }
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = k_lo; k0 < k_hi; k0 += 64) {
    float av[16], bv[16], mk[16];
    if constexpr (VEC) {
      static_assert(!MASK, "VEC is the forward (unmasked) path");
      const int kb = k0 + 16 * kq;
      f32x4 ar[4], br[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {  // clamped group base: in bounds and 16-B aligned (K % 4 == 0)
        const int kg = min(kb + 4 * t, g.K - 4);
        ar[t] = *reinterpret_cast<const f32x4*>(g.a + ma + kg);
        br[t] = *reinterpret_cast<const f32x4*>(g.b + nb + kg);
      }
      __builtin_amdgcn_sched_barrier(0);  // all 8 loads in flight before the first use
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bool kin = kb + 4 * t < k_hi;  // whole groups: K % 4 == 0
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = (kin && mv) ? ar[t][e] : 0.f, b = (kin && nv) ? br[t][e] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
      }
      continue;
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const long kc = min(k0 + 4 * s + kq, g.K - 1);
      av[s] = g.a[ma + kc * g.a_k];
      if constexpr (MASK) mk[s] = g.am[ma + kc * g.a_k];
      bv[s] = g.b[kc * g.b_k + nb];
    }
    __builtin_amdgcn_sched_barrier(0);  // all 32 (48) loads in flight before the first use
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool kin = k0 + 4 * s + kq < k_hi;
      bool aon = kin && mv;
      if constexpr (MASK) aon = aon && mk[s] > 0.f;
      av[s] = aon ? av[s] : 0.f;
      bv[s] = kin ? (ones ? 1.f : (nv ? bv[s] : 0.f)) : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
  }
  f32x4 sum = acc;
  if (nw > 1) {  // waves' partial sums through LDS (dynamic: nw x 64 x 16 B)
    red[wave * 64 + lane] = acc;
    __syncthreads();
    if (wave != 0) return;
    sum = red[lane];
    for (int w = 1; w < nw; ++w) sum += red[w * 64 + lane];  // fixed order: deterministic
  }
  // lane (i, kq) holds C[m0 + 4 kq + r][n0 + i], r = 0..3
  if constexpr (XENT) {
    xent_rows(g, sum, lab, bvalid, m0, i, kq, lane);
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mm = m0 + 4 * kq + r;
    if (mm >= g.M) continue;
    float v = sum[r];
    if (ones) {
      g.c_ones[mm] = v;
      continue;
    }
    if (!nv) continue;
    if (g.bias != nullptr) v += g.bias[n];
    if (g.relu) v = fmaxf(v, 0.f);
    g.c[(long)mm * g.c_m + n] = v;
  }
}

// blockIdx.z selects the GEMM: the data and weight gradients of one layer share a launch (both
// only read dz, x and W).  Waves past a GEMM's own reduction split get an empty k range and
// add exact zeros to the fixed-order sum.
template <bool MASK>
__global__ void __launch_bounds__(64 * LIN_MAX_WAVES) small_gemm_kernel(const GemmArgs g0, const GemmArgs g1) {
  extern __shared__ f32x4 red[];
  if (blockIdx.z == 0) small_gemm_tile<MASK>(g0, red);
  else small_gemm_tile<MASK>(g1, red);
}

template <bool VEC>
__global__ void __launch_bounds__(64 * LIN_MAX_WAVES) small_gemm_xent_kernel(const GemmArgs g) {
  extern __shared__ f32x4 red[];
  small_gemm_tile<false, true, VEC>(g, red);
}

// forward GEMM with k-contiguous vector operand loads (see small_gemm_tile)
__global__ void __launch_bounds__(64 * LIN_MAX_WAVES) small_gemm_fwd_vec_kernel(const GemmArgs g) {
  extern __shared__ f32x4 red[];
  small_gemm_tile<false, false, true>(g, red);
}

// Split-K forward for long reductions (cifar-vgg's fc1: 64 x 4096 x 256 has only 64 output tiles,
// so one workgroup per tile fills 64 CUs and walks K = 4096 alone): grid z = split s takes
// k in [s Ks, (s + 1) Ks) of every tile and writes its fp32 partial tile to part[s]; a combine
// launch sums the S partials per output IN SPLIT ORDER (deterministic, no atomics) and applies
// the bias and the ReLU.
template <bool VEC>
__global__ void __launch_bounds__(64 * LIN_MAX_WAVES) splitk_gemm_kernel(const GemmArgs g, int ks, float* part) {
  extern __shared__ f32x4 red[];
  const int s = blockIdx.z, k0 = s * ks;
  GemmArgs gs = g;
  gs.a = g.a + (long)k0 * g.a_k;
  gs.b = g.b + (long)k0 * g.b_k;
  gs.K = min(ks, g.K - k0);
  gs.c = part + (long)s * g.M * g.N;
  gs.c_m = g.N;
  gs.bias = nullptr;
  gs.relu = 0;
  small_gemm_tile<false, false, VEC>(gs, red);
}

__global__ void __launch_bounds__(256) splitk_combine_kernel(const float* __restrict__ part, int S, int M, int N,
                                                             const float* __restrict__ bias, int relu,
                                                             float* __restrict__ y, long y_m) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= M * N) return;
  const int m = i / N, n = i - m * N;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += part[(long)s * M * N + i];  // split order: deterministic
  if (bias != nullptr) v += bias[n];
  if (relu) v = fmaxf(v, 0.f);
  y[(long)m * y_m + n] = v;
}

// the forward operands qualify for the vector loads: rows contiguous along k, K a multiple of 4,
// every row start 16-B aligned
bool fwd_vec_ok(const GemmArgs& g) {
  auto al = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  return g.a_k == 1 && g.b_k == 1 && g.K % 4 == 0 && g.K >= 4 && g.a_m % 4 == 0 && g.b_n % 4 == 0 && al(g.a) &&
         al(g.b) && g.am == nullptr && g.ones_col < 0;
}

// waves per tile: one 64-deep batch each (all of a tile's loads in flight at once), at most
// 16 waves; longer reductions loop.  Returns the waves this GEMM uses.
int prepare(GemmArgs& g) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) throw std::runtime_error("linear: empty GEMM");
  g.ncols = g.ones_col >= 0 ? g.ones_col + 1 : g.N;
  const int nw = std::max(1, std::min(LIN_MAX_WAVES, (g.K + 63) / 64));
  g.kpw = ((g.K + nw - 1) / nw + 63) / 64 * 64;
  return (g.K + g.kpw - 1) / g.kpw;
}

// LDS of the waves' fixed-order reduction (none for a single wave)
size_t lds_bytes(int waves) { return waves > 1 ? (size_t)waves * 64 * sizeof(f32x4) : 0; }

// one launch for one GEMM, or for two (same MASK) in grid z = 0 / 1
void launch(GemmArgs g0, const GemmArgs* g1p, hipStream_t s) {
  int waves = prepare(g0);
  unsigned gx = (unsigned)((g0.ncols + 15) / 16), gy = (unsigned)((g0.M + 15) / 16), gz = 1;
  GemmArgs g1 = g0;
  if (g1p != nullptr) {
    g1 = *g1p;
    if ((g1.am != nullptr) != (g0.am != nullptr)) throw std::runtime_error("linear: paired GEMMs differ in masking");
    waves = std::max(waves, prepare(g1));
    gx = std::max(gx, (unsigned)((g1.ncols + 15) / 16));
    gy = std::max(gy, (unsigned)((g1.M + 15) / 16));
    gz = 2;
  }
  const dim3 grid(gx, gy, gz), block(64 * waves);
  const size_t lds = lds_bytes(waves);
  if (g0.am != nullptr) hipLaunchKernelGGL(small_gemm_kernel<true>, grid, block, lds, s, g0, g1);
  else hipLaunchKernelGGL(small_gemm_kernel<false>, grid, block, lds, s, g0, g1);
  HIP_CHECK(hipGetLastError());
}

GemmArgs dgrad_args(const float* dy, const float* y, const float* w, float* dx, int B, int K, int N) {
  GemmArgs g{};
  g.a = dy; g.am = y; g.a_m = N; g.a_k = 1;
  g.b = w; g.b_k = K; g.b_n = 1;
  g.c = dx; g.c_m = K;
  g.M = B; g.N = K; g.K = N; g.ones_col = -1;
  return g;
}

GemmArgs wgrad_args(const float* dy, const float* y, const float* x, float* dw, float* db, int B, int K, int N) {
  GemmArgs g{};
  g.a = dy; g.am = y; g.a_m = 1; g.a_k = N;  // A(m = n, k = b) = dz[b][n]
  g.b = x; g.b_k = K; g.b_n = 1;             // B(k = b, n = k') = x[b][k'],  k' == K: 1
  g.c = dw; g.c_m = K; g.c_ones = db;
  g.M = N; g.N = K; g.K = B; g.ones_col = K;
  return g;
}

}  // namespace

// y[B][N] = act(x[B][K] W[N][K]^T + b)
void launch_linear_fwd(const float* x, const float* w, const float* b, float* y, int B, int K, int N, int relu,
                       hipStream_t s) {
  GemmArgs g{};
  g.a = x; g.a_m = K; g.a_k = 1;
  g.b = w; g.b_k = 1; g.b_n = K;
  g.c = y; g.c_m = N;
  g.bias = b;
  g.M = B; g.N = N; g.K = K; g.ones_col = -1; g.relu = relu;
  if (fwd_vec_ok(g)) {
    const int waves = prepare(g);
    hipLaunchKernelGGL(small_gemm_fwd_vec_kernel, dim3((unsigned)((N + 15) / 16), (unsigned)((B + 15) / 16)),
                       dim3(64 * waves), lds_bytes(waves), s, g);
    HIP_CHECK(hipGetLastError());
    return;
  }
  launch(g, nullptr, s);
}

// splits of a split-K forward: enough workgroups to fill the chip (>= 256 over the output tiles),
// each split a multiple of 64 (one wave batch) and at least 256 deep
int linear_splitk_splits(int B, int K, int N) {
  const int tiles = ((N + 15) / 16) * ((B + 15) / 16);
  int S = 1;
  while (tiles * S < 256 && K / (2 * S) >= 256) S *= 2;
  return S;
}

// y[B][N] = act(x[B][K] W[N][K]^T + b) as S split-K partial GEMMs + one combine launch;
// part: S * B * N floats of workspace
void launch_linear_fwd_splitk(const float* x, const float* w, const float* b, float* y, float* part, int S, int B,
                              int K, int N, int relu, hipStream_t s) {
  if (S < 1 || K < S) throw std::runtime_error("linear_fwd_splitk: bad split count");
  GemmArgs g{};
  g.a = x; g.a_m = K; g.a_k = 1;
  g.b = w; g.b_k = 1; g.b_n = K;
  g.M = B; g.N = N; g.K = K; g.ones_col = -1;
  const int ks = ((K + S - 1) / S + 63) / 64 * 64;
  const int splits = (K + ks - 1) / ks;
  GemmArgs gk = g;
  gk.K = ks;  // (the waves of one split; the last split may be shorter)
  const int waves = prepare(gk);
  g.kpw = gk.kpw;
  g.ncols = g.N;
  const dim3 grid((unsigned)((N + 15) / 16), (unsigned)((B + 15) / 16), (unsigned)splits);
  const bool vec = fwd_vec_ok(g) && ks % 4 == 0;
  if (vec) hipLaunchKernelGGL(splitk_gemm_kernel<true>, grid, dim3(64 * waves), lds_bytes(waves), s, g, ks, part);
  else hipLaunchKernelGGL(splitk_gemm_kernel<false>, grid, dim3(64 * waves), lds_bytes(waves), s, g, ks, part);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(splitk_combine_kernel, dim3((unsigned)((B * N + 255) / 256)), dim3(256), 0, s, part, splits, B, N,
                     b, relu, y, (long)N);
  HIP_CHECK(hipGetLastError());
}

// logits[B][N] = x W^T + b with the softmax cross-entropy of every row fused in (N <= 16)
void launch_linear_fwd_xent(const float* x, const float* w, const float* b, float* y, const int32_t* labels,
                            const int32_t* state, float* loss, int32_t* correct, float* dlogits, int B, int K, int N,
                            hipStream_t s) {
  if (N > 16) throw std::runtime_error("linear_fwd_xent: more than 16 classes");
  GemmArgs g{};
  g.a = x; g.a_m = K; g.a_k = 1;
  g.b = w; g.b_k = 1; g.b_n = K;
  g.c = y; g.c_m = N;
  g.bias = b;
  g.M = B; g.N = N; g.K = K; g.ones_col = -1;
  g.labels = labels; g.state = state; g.loss = loss; g.correct = correct; g.dlogits = dlogits;
  const int waves = prepare(g);
  const dim3 grid(1, (unsigned)((B + 15) / 16));
  if (fwd_vec_ok(g)) hipLaunchKernelGGL(small_gemm_xent_kernel<true>, grid, dim3(64 * waves), lds_bytes(waves), s, g);
  else hipLaunchKernelGGL(small_gemm_xent_kernel<false>, grid, dim3(64 * waves), lds_bytes(waves), s, g);
  HIP_CHECK(hipGetLastError());
}

// dx[B][K] = dz[B][N] W[N][K], dz = dy masked by y > 0 when y != nullptr (fused ReLU)
void launch_linear_dgrad(const float* dy, const float* y, const float* w, float* dx, int B, int K, int N,
                         hipStream_t s) {
  launch(dgrad_args(dy, y, w, dx, B, K, N), nullptr, s);
}

// dW[N][K] = dz^T x, db[N] = sum_b dz[b][n] (dz as in dgrad)
void launch_linear_wgrad(const float* dy, const float* y, const float* x, float* dw, float* db, int B, int K, int N,
                         hipStream_t s) {
  launch(wgrad_args(dy, y, x, dw, db, B, K, N), nullptr, s);
}

// both gradients of one layer in ONE launch (dx == nullptr: weight gradient only)
void launch_linear_bwd(const float* dy, const float* y, const float* w, const float* x, float* dx, float* dw,
                       float* db, int B, int K, int N, hipStream_t s) {
  const GemmArgs gw = wgrad_args(dy, y, x, dw, db, B, K, N);
  if (dx == nullptr) {
    launch(gw, nullptr, s);
    return;
  }
  const GemmArgs gd = dgrad_args(dy, y, w, dx, B, K, N);
  launch(gd, &gw, s);
}

}  // namespace dnn

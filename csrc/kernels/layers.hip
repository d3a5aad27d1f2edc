// Generic CNN layer kernels (gfx950) for the modular engine (runtime/layer_engine.py).
//
// The fused LeNet kernel (lenet_fused.hip) is the fast path for the reference model.
// These kernels make the framework usable for other CNN stacks built from the layer set
// the north star names - Conv2d, ReLU, MaxPool, BatchNorm, Linear, CrossEntropy, SGD -
// in fp32 (exact parity with the reference's fp32 CPU arithmetic) or with bf16 GEMM
// operands.  Capability parity: the ATen ops of SURVEY.md §2.5 K0-K23.
//
// Split of work (MI355X-first):
//  * Conv2d is an implicit-GEMM MFMA kernel family of its own (conv_igemm.hip); Linear
//    goes to the library GEMM (hipBLASLt via torch.matmul);
//  * everything else is a hand-written kernel: ingest (u8 gather + ToTensor/Normalize),
//    fused ReLU + 2x2 max-pool with a 2-bit argmax code (the same encoding as the fused
//    kernel: 4 = no gradient), BatchNorm2d train/eval forward + backward with the tail
//    batch masked out of the statistics, fused softmax cross-entropy forward + backward +
//    accuracy, step bookkeeping (shared with the fused path), flat momentum SGD.
//  * every reduction is a fixed-order tree (no float atomics): bitwise reproducible.
#include <cstdint>
#include <initializer_list>

#include "reduce_common.h"

namespace dnn {

namespace {

constexpr int LT = 256;  // threads per block of the element-wise kernels

__device__ __forceinline__ int valid_count(const int32_t* state, int batch) {
  return state ? min(state[ST_BVALID], batch) : batch;
}

// ---- ingest: gather the batch's u8 images by sample id, ToTensor + Normalize ----------
__global__ void __launch_bounds__(LT) ingest_kernel(const uint8_t* __restrict__ images,
                                                    const int32_t* __restrict__ labels,
                                                    const int32_t* __restrict__ ids, int batch, int per_img,
                                                    float* __restrict__ out, int32_t* __restrict__ lab_out) {
  const long i = (long)blockIdx.x * LT + threadIdx.x;
  const long total = (long)batch * per_img;
  if (i >= total) return;
  const int b = (int)(i / per_img), e = (int)(i - (long)b * per_img);
  const int sid = ids[b];
  const uint32_t u = images[(size_t)sid * per_img + e];
  // torchvision op order (data_parallelism_train.py:24-27), IEEE-rounded division
  out[i] = __fdiv_rn(__fdiv_rn((float)u, 255.0f) - 0.5f, 0.5f);
  if (e == 0) lab_out[b] = labels[sid];
}

// ---- fused ReLU + 2x2 max-pool (stride 2, floor) with a 2-bit argmax code -------------
// max_pool2d(relu(x)) == relu(max_pool2d(x)); code = first argmax (torch order) or 4 when
// the max is <= 0 (no gradient reaches the input: ReLU and pool backward in one test).
__global__ void __launch_bounds__(LT) relu_pool_fwd_kernel(const float* __restrict__ x, int BC, int H, int W,
                                                           float* __restrict__ y, uint8_t* __restrict__ code) {
  const int OH = H / 2, OW = W / 2;
  const int i = blockIdx.x * LT + threadIdx.x;
  if (i >= BC * OH * OW) return;
  const unsigned r = (unsigned)i / (unsigned)OW;
  const int ox = i - (int)r * OW;
  const int bc = (int)(r / (unsigned)OH), oy = (int)r - bc * OH;
  const float* p = x + ((size_t)bc * H + 2 * oy) * W + 2 * ox;
  float best = p[0];
  int arg = 0;
  const float v1 = p[1], v2 = p[W], v3 = p[W + 1];
  if (v1 > best) { best = v1; arg = 1; }
  if (v2 > best) { best = v2; arg = 2; }
  if (v3 > best) { best = v3; arg = 3; }
  y[i] = fmaxf(best, 0.f);
  code[i] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
}

__global__ void __launch_bounds__(LT) relu_pool_bwd_kernel(const float* __restrict__ dy,
                                                           const uint8_t* __restrict__ code, int BC, int H, int W,
                                                           float* __restrict__ dx) {
  const int i = blockIdx.x * LT + threadIdx.x;
  if (i >= BC * H * W) return;
  const int OH = H / 2, OW = W / 2;
  const unsigned r = (unsigned)i / (unsigned)W;
  const int xx = i - (int)r * W;
  const int bc = (int)(r / (unsigned)H), y = (int)r - bc * H;
  const int oy = y >> 1, ox = xx >> 1;
  float v = 0.f;
  if (oy < OH && ox < OW) {
    const int o = (bc * OH + oy) * OW + ox;
    if (code[o] == (uint8_t)(((y & 1) << 1) | (xx & 1))) v = dy[o];
  }
  dx[i] = v;
}

// ---- ReLU (for the fc stack) ------------------------------------------------------------
__global__ void __launch_bounds__(LT) relu_fwd_kernel(const float* __restrict__ x, long n, float* __restrict__ y) {
  const long i = (long)blockIdx.x * LT + threadIdx.x;
  if (i < n) y[i] = fmaxf(x[i], 0.f);
}
__global__ void __launch_bounds__(LT) relu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                      long n, float* __restrict__ dx) {
  const long i = (long)blockIdx.x * LT + threadIdx.x;
  if (i < n) dx[i] = y[i] > 0.f ? dy[i] : 0.f;
}

// ---- per-channel reductions over (batch, pixels): deterministic two-stage ---------------
// Stage 1: grid (P, C) blocks; block (p, c) owns channel c's planes of samples
// [p * ppb, (p + 1) * ppb) (ppb = planes per block, ~2048 elements) and reduces them into
// fp64 partials; stage 2 merges a channel's P partials in a fixed order.  The split depends
// only on (B, L), never on the valid count, so graph replays and tail batches reduce in the
// same order (bitwise reproducible).  fp64 partial sums make the one-pass E[x^2] - E[x]^2
// variance safe.  Threads walk (plane, vector) pairs incrementally - no per-element integer
// division - and move float4 vectors when the plane allows it (VW = 4; host-checked).
__host__ __device__ inline int chan_ppb(int B, int L) {
  const int p = (2048 + L - 1) / L;
  return p < 1 ? 1 : (p > B ? (B > 0 ? B : 1) : p);
}
__host__ __device__ inline int chan_parts_of(int B, int L) {
  const int ppb = chan_ppb(B, L);
  const int P = (B + ppb - 1) / ppb;
  return P < 1 ? 1 : P;
}

// f(b, l, o) for every VW-vector (plane b of channel c, first pixel l, element offset o) of
// planes [b0, b1); thread t takes vectors t, t + LT, ...
template <int VW, typename F>
__device__ __forceinline__ void plane_walk(int b0, int b1, int C, int c, int L, F&& f) {
  const int LV = L / VW;
  if (b1 <= b0 || LV <= 0) return;
  const int n = (b1 - b0) * LV;
  const int dq = LT / LV, dr = LT - dq * LV;
  int q = (int)threadIdx.x / LV, r = (int)threadIdx.x - q * LV;
  for (int t = threadIdx.x; t < n; t += LT) {
    const int l = r * VW;
    f(b0 + q, l, ((b0 + q) * C + c) * L + l);  // 32-bit: B*C*L < 2^31 (host check)
    r += dr;
    q += dq;
    if (r >= LV) { r -= LV; ++q; }
  }
}

template <int VW>
__device__ __forceinline__ void ldv(const float* __restrict__ p, float (&v)[VW]) {
  if constexpr (VW == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
#pragma unroll
    for (int j = 0; j < VW; ++j) v[j] = p[j];
  }
}
template <int VW>
__device__ __forceinline__ void stv(float* __restrict__ p, const float (&v)[VW]) {
  if constexpr (VW == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int j = 0; j < VW; ++j) p[j] = v[j];
  }
}

__device__ __forceinline__ void block_sum2_d(double& s0, double& s1, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_down(s0, off);
    s1 += __shfl_down(s1, off);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[2 * wave] = s0;
    red[2 * wave + 1] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < LT / 64; ++w) {
      a += red[2 * w];
      b += red[2 * w + 1];
    }
    s0 = a;
    s1 = b;
  }
}

// BatchNorm affine output with an explicit rounding sequence: the fused BN+ReLU backward
// recomputes it to rebuild the ReLU mask, and must get the forward's exact sign.
__device__ __forceinline__ float bn_affine(float x, float mean, float invstd, float g, float bb) {
  return __fmaf_rn(__fmul_rn(__fsub_rn(x, mean), invstd), g, bb);
}

// Activation fused after BatchNorm (ACT): 0 none, 1 ReLU, 2 ReLU + 2x2 max-pool (2-bit code).
struct ActArgs {
  const float* beta;     // ACT 1
  const uint8_t* code;   // ACT 2: [B][C][H/2][W/2]
  int W, OH;             // ACT 2: plane width, pooled height (H / 2)
};
// Gradient reaching the BN output at the VW pixels (b, c, l..l+VW-1), element offset o:
// ACT 0 reads dy; ACT 1 re-derives the ReLU mask from x; ACT 2 routes the pooled gradient
// through the code (VW pixels share one image row: W % VW == 0, host-checked).
template <int ACT, int VW>
__device__ __forceinline__ void grad_in(const float* __restrict__ dy, const ActArgs& aa, int b, int C, int c, int l,
                                        int o, const float (&xv)[VW], float mean, float invstd, float g,
                                        float (&d)[VW]) {
  if constexpr (ACT == 2) {
    const int W = aa.W, OW = W >> 1;
    const int yy = l / W, xx0 = l - yy * W, oy = yy >> 1;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const int xx = xx0 + j, ox = xx >> 1;
      d[j] = 0.f;
      if (oy < aa.OH && ox < OW) {
        const int po = ((b * C + c) * aa.OH + oy) * OW + ox;
        if (aa.code[po] == (uint8_t)(((yy & 1) << 1) | (xx & 1))) d[j] = dy[po];
      }
    }
  } else {
    ldv<VW>(dy + o, d);
    if constexpr (ACT == 1) {
      const float bb = aa.beta[c];
#pragma unroll
      for (int j = 0; j < VW; ++j)
        if (!(bn_affine(xv[j], mean, invstd, g, bb) > 0.f)) d[j] = 0.f;
    }
  }
}

// MODE 0: (sum x, sum x^2)   MODE 1: (sum dz, sum dz * xhat), dz = grad_in<ACT>   MODE 2: (sum a, 0)
template <int MODE, int ACT, int VW>
__global__ void __launch_bounds__(LT) chan_partial_kernel(const float* __restrict__ a, const float* __restrict__ x,
                                                          int B, int C, int L, const int32_t* __restrict__ state,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          double* __restrict__ part, const float* __restrict__ gamma,
                                                          ActArgs aa) {
  __shared__ double red[2 * (LT / 64)];
  const int c = blockIdx.y, p = blockIdx.x, P = gridDim.x;
  const int bv = valid_count(state, B), ppb = chan_ppb(B, L);
  const int b0 = p * ppb, b1 = min(min(B, b0 + ppb), bv);  // valid planes only
  const float mu = MODE == 1 ? mean[c] : 0.f, is = MODE == 1 ? invstd[c] : 0.f;
  const float g = (MODE == 1 && ACT == 1) ? gamma[c] : 0.f;
  double s0 = 0.0, s1 = 0.0;
  plane_walk<VW>(b0, b1, C, c, L, [&](int b, int l, int o) {
    if constexpr (MODE == 1) {
      float xv[VW], d[VW];
      ldv<VW>(x + o, xv);
      grad_in<ACT, VW>(a, aa, b, C, c, l, o, xv, mu, is, g, d);
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        s0 += (double)d[j];
        s1 += (double)d[j] * (double)((xv[j] - mu) * is);
      }
    } else {
      float v[VW];
      ldv<VW>(a + o, v);
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        s0 += (double)v[j];
        if (MODE == 0) s1 += (double)v[j] * (double)v[j];
      }
    }
  });
  block_sum2_d(s0, s1, red);
  if (threadIdx.x == 0) {
    part[((size_t)c * P + p) * 2] = s0;
    part[((size_t)c * P + p) * 2 + 1] = s1;
  }
}

__device__ __forceinline__ void merge_parts(const double* part, int c, int P, double& s0, double& s1) {
  s0 = 0.0;
  s1 = 0.0;
  for (int q = 0; q < P; ++q) {
    s0 += part[((size_t)c * P + q) * 2];
    s1 += part[((size_t)c * P + q) * 2 + 1];
  }
}

// ---- BatchNorm2d -------------------------------------------------------------------------
// Training: batch statistics over the VALID samples only (the padded tail batch of a
// captured step must not pollute them), biased variance for the normalisation, unbiased
// for the running estimate (torch semantics, momentum m).  Grid (P, C) like the partials:
// each block merges its channel's partials, then normalises (and activates) its planes.
template <int ACT, int VW>
__global__ void __launch_bounds__(LT) bn_apply_train_kernel(const float* __restrict__ x, int B, int C, int L,
                                                            const int32_t* __restrict__ state,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps, float m,
                                                            float* __restrict__ running_mean,
                                                            float* __restrict__ running_var, float* __restrict__ y,
                                                            float* __restrict__ save_mean,
                                                            float* __restrict__ save_invstd,
                                                            const double* __restrict__ part, int W,
                                                            uint8_t* __restrict__ code, int nparts) {
  __shared__ float st[2];
  __shared__ double red[2 * (LT / 64)];
  const int c = blockIdx.y, p = blockIdx.x;
  const int bv = valid_count(state, B), ppb = chan_ppb(B, L);
  // merge the channel's nparts partials (chan_partial_kernel's, or a conv epilogue's - one per
  // output tile) across the block: strided fp64 sums, then the fixed-order block sum
  double s0 = 0.0, s1 = 0.0;
  for (int q = threadIdx.x; q < nparts; q += LT) {
    s0 += part[((size_t)c * nparts + q) * 2];
    s1 += part[((size_t)c * nparts + q) * 2 + 1];
  }
  block_sum2_d(s0, s1, red);
  if (threadIdx.x == 0) {
    const double n = (double)bv * L;
    const double mean = n > 0 ? s0 / n : 0.0;
    const double var = n > 0 ? fmax(s1 / n - mean * mean, 0.0) : 0.0;
    const float invstd = rsqrtf((float)var + eps);
    st[0] = (float)mean;
    st[1] = invstd;
    if (p == 0) {
      save_mean[c] = (float)mean;
      save_invstd[c] = invstd;
      if (n > 0) {
        const double unb = n > 1 ? var * n / (n - 1) : var;
        running_mean[c] = (1.f - m) * running_mean[c] + m * (float)mean;
        running_var[c] = (1.f - m) * running_var[c] + m * (float)unb;
      }
    }
  }
  __syncthreads();
  const float mean = st[0], invstd = st[1], g = gamma[c], bb = beta[c];
  const int b0 = p * ppb, b1 = min(B, b0 + ppb);  // every plane: the padded tail is written as 0
  if constexpr (ACT == 2) {
    // BN -> ReLU -> 2x2 max-pool: one pooled output per thread (4 BN values, first max wins,
    // code 4 = max <= 0), exactly relu_pool_fwd_kernel applied to the BN output
    const int H = L / W, OH = H >> 1, OW = W >> 1;
    plane_walk<1>(b0, b1, C, c, OH * OW, [&](int b, int pl, int po) {
      float out = 0.f;
      uint8_t cd = 4;
      if (b < bv) {
        const int oy = pl / OW, ox = pl - oy * OW;
        const float* xp = x + ((long)(b * C + c) * H + 2 * oy) * W + 2 * ox;
        float best = bn_affine(xp[0], mean, invstd, g, bb);
        int arg = 0;
        const float v1 = bn_affine(xp[1], mean, invstd, g, bb), v2 = bn_affine(xp[W], mean, invstd, g, bb),
                    v3 = bn_affine(xp[W + 1], mean, invstd, g, bb);
        if (v1 > best) { best = v1; arg = 1; }
        if (v2 > best) { best = v2; arg = 2; }
        if (v3 > best) { best = v3; arg = 3; }
        out = fmaxf(best, 0.f);
        cd = best > 0.f ? (uint8_t)arg : (uint8_t)4;
      }
      y[po] = out;
      code[po] = cd;
    });
  } else {
    plane_walk<VW>(b0, b1, C, c, L, [&](int b, int l, int o) {
      float v[VW];
      if (b < bv) {
        ldv<VW>(x + o, v);
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          v[j] = bn_affine(v[j], mean, invstd, g, bb);
          if (ACT == 1) v[j] = fmaxf(v[j], 0.f);
        }
      } else {
#pragma unroll
        for (int j = 0; j < VW; ++j) v[j] = 0.f;
      }
      stv<VW>(y + o, v);
    });
  }
}

__global__ void __launch_bounds__(LT) bn_fwd_eval_kernel(const float* __restrict__ x, int B, int C, int L,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps,
                                                         const float* __restrict__ running_mean,
                                                         const float* __restrict__ running_var,
                                                         float* __restrict__ y) {
  const int i = blockIdx.x * LT + threadIdx.x;
  if (i >= B * C * L) return;
  const int c = (int)(((unsigned)i / (unsigned)L) % (unsigned)C);
  y[i] = (x[i] - running_mean[c]) * rsqrtf(running_var[c] + eps) * gamma[c] + beta[c];
}

template <int ACT, int VW>
__global__ void __launch_bounds__(LT) bn_bwd_apply_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                          int B, int C, int L, const int32_t* __restrict__ state,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ save_mean,
                                                          const float* __restrict__ save_invstd,
                                                          float* __restrict__ dx, float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta,
                                                          const double* __restrict__ part, ActArgs aa, int nparts) {
  __shared__ float st[2];
  __shared__ double red[2 * (LT / 64)];
  const int c = blockIdx.y, p = blockIdx.x;
  const int bv = valid_count(state, B), ppb = chan_ppb(B, L);
  // the channel's nparts partials (chan_partial_kernel's, or a conv data-gradient epilogue's),
  // merged across the block in a fixed order (as bn_apply_train_kernel)
  double s0 = 0.0, s1 = 0.0;
  for (int q = threadIdx.x; q < nparts; q += LT) {
    s0 += part[((size_t)c * nparts + q) * 2];
    s1 += part[((size_t)c * nparts + q) * 2 + 1];
  }
  block_sum2_d(s0, s1, red);
  if (threadIdx.x == 0) {
    const double n = (double)bv * L;
    st[0] = n > 0 ? (float)(s0 / n) : 0.f;
    st[1] = n > 0 ? (float)(s1 / n) : 0.f;
    if (p == 0) {
      dgamma[c] = (float)s1;
      dbeta[c] = (float)s0;
    }
  }
  __syncthreads();
  const float mdy = st[0], mdyx = st[1];
  const float mean = save_mean[c], invstd = save_invstd[c], g = gamma[c];
  const int b0 = p * ppb, b1 = min(B, b0 + ppb);
  plane_walk<VW>(b0, b1, C, c, L, [&](int b, int l, int o) {
    float r[VW];
    if (b < bv) {
      float xv[VW], d[VW];
      ldv<VW>(x + o, xv);
      grad_in<ACT, VW>(dy, aa, b, C, c, l, o, xv, mean, invstd, g, d);
#pragma unroll
      for (int j = 0; j < VW; ++j) r[j] = g * invstd * (d[j] - mdy - (xv[j] - mean) * invstd * mdyx);
    } else {
#pragma unroll
      for (int j = 0; j < VW; ++j) r[j] = 0.f;
    }
    stv<VW>(dx + o, r);
  });
}

// per-channel sum of a [B][C][L] tensor (conv bias gradient): stage 2
__global__ void __launch_bounds__(64) chan_sum_finalize_kernel(const double* __restrict__ part, int C, int P,
                                                               float* __restrict__ out) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= C) return;
  double s0, s1;
  merge_parts(part, c, P, s0, s1);
  out[c] = (float)s0;
}

// ---- fused softmax cross-entropy forward + backward + accuracy -----------------------------
// One thread per sample.  loss[b] / correct[b] per sample (0 for the padded tail),
// dlogits = (softmax - onehot) / bvalid  (CrossEntropyLoss mean reduction).
__global__ void __launch_bounds__(LT) xent_kernel(const float* __restrict__ logits, const int32_t* __restrict__ labels,
                                                  int B, int NC, const int32_t* __restrict__ state,
                                                  float* __restrict__ loss, int32_t* __restrict__ correct,
                                                  float* __restrict__ dlogits) {
  const int b = blockIdx.x * LT + threadIdx.x;
  if (b >= B) return;
  const int bv = valid_count(state, B);
  const float* z = logits + (size_t)b * NC;
  float* dz = dlogits ? dlogits + (size_t)b * NC : nullptr;
  if (b >= bv) {
    loss[b] = 0.f;
    correct[b] = 0;
    if (dz) for (int k = 0; k < NC; ++k) dz[k] = 0.f;
    return;
  }
  float mx = z[0];
  int arg = 0;
  for (int k = 1; k < NC; ++k) {
    if (z[k] > mx) { mx = z[k]; arg = k; }  // first max wins (torch.argmax)
  }
  float sum = 0.f;
  for (int k = 0; k < NC; ++k) sum += expf(z[k] - mx);
  const int y = labels[b];
  loss[b] = mx + logf(sum) - z[y];
  correct[b] = arg == y ? 1 : 0;
  if (dz) {
    const float inv = 1.f / (float)bv;
    for (int k = 0; k < NC; ++k) dz[k] = (expf(z[k] - mx) / sum - (k == y ? 1.f : 0.f)) * inv;
  }
}

// ---- step bookkeeping (epoch loss/accuracy, next batch ids) - shared with the fused path --
__global__ void __launch_bounds__(64) layer_bookkeeping_kernel(ReduceArgs a) { bookkeeping(a, threadIdx.x); }

// ---- flat momentum SGD over an arena (no bf16 shadow: generic models) -------------------------
// torch.optim.SGD (dampening 0, no nesterov) with the explicit fmas of sgd_update, so the
// value a packed conv-weight image receives below is bit-identical to the arena's.
__global__ void __launch_bounds__(LT) sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, long n, float lr, float momentum,
                                                      float grad_scale) {
  const long i = (long)blockIdx.x * LT + threadIdx.x;
  if (i >= n) return;
  float pn, mn;
  sgd_update(g[i] * grad_scale, p[i], m[i], lr, momentum, pn, mn);
  m[i] = mn;
  p[i] = pn;
}

// packed-image stores of an updated conv weight (arena element i, new value pn)
__device__ __forceinline__ void scatter_packed(const PackScatter& ps, long i, float pn) {
  for (int j = 0; j < ps.n; ++j) {
    const PackScatter::Item& it = ps.it[j];
    const long l = i - it.off;
    if (l < 0 || l >= it.len) continue;
    // layer weight [Cout][Cin][K][K]; the image holds (m, c, ky, kx) = (o, ci, y, x), or
    // (ci, o, K-1-y, K-1-x) for the flipped dgrad image (launch_conv_pack_all's element map)
    const int KK = it.K * it.K, cin = it.flip ? it.M : it.C;
    const int x = (int)(l % it.K), y = (int)((l / it.K) % it.K), ci = (int)((l / KK) % cin);
    const int o = (int)(l / ((long)KK * cin));
    const int mm = it.flip ? ci : o, cc = it.flip ? o : ci;
    const int tap = it.flip ? (it.K - 1 - y) * it.K + (it.K - 1 - x) : y * it.K + x;
    const long d = ((long)tap * it.Mp + mm) * it.Cp + cc;
    if (it.bf) reinterpret_cast<bf16*>(it.dst)[d] = (bf16)pn;
    else reinterpret_cast<float*>(it.dst)[d] = pn;
  }
}

// The step's tail in ONE launch of TT-thread workgroups, by workgroup role:
//   [0, ss.start[ss.n])  deferred conv weight gradients, 64 elements per workgroup: wave w of 16
//                        sums slices w, w + 16, ... (8 loads in flight per batch) and wave 0 adds
//                        the 16 wave sums in w order - slice_sum_kernel's exact layout and order,
//                        so the gradient is bit-identical to the two-launch path; then SGD;
//   next ceil(n / TT)    momentum SGD over the rest of the arena;
//   last (BOOK)          the step bookkeeping (epoch loss / accuracy, cursor, next batch ids).
// Every updated conv weight is also stored into the layer's packed forward / dgrad images (the
// next step's conv kernels read those: no pack launch at the next step's start).
constexpr int TT = 1024;
template <bool BOOK>
__global__ void __launch_bounds__(TT) sgd_tail_kernel(float* __restrict__ p, float* __restrict__ g,
                                                      float* __restrict__ m, long n, float lr, float momentum,
                                                      float grad_scale, const PackScatter ps, const SliceSet ss,
                                                      const ReduceArgs book) {
  const int nsg = ss.start[ss.n];
  if (BOOK && blockIdx.x == gridDim.x - 1) {
    if (threadIdx.x < 64) bookkeeping(book, threadIdx.x);
    return;
  }
  if ((int)blockIdx.x < nsg) {
    constexpr int SWV = TT / 64;  // waves over the slices
    __shared__ float red[SWV][64];
    int j = 0;
    while (j + 1 < ss.n && (int)blockIdx.x >= ss.start[j + 1]) ++j;
    const SliceJob& sj = ss.it[j];
    const long ne = (long)sj.M * (sj.Kd + 1);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long e = (long)((int)blockIdx.x - ss.start[j]) * 64 + lane;
    const bool ev = e < ne;
    const float* src = sj.part + (ev ? e : 0);
    float acc = 0.f;
    for (int s0 = w; s0 < sj.S; s0 += 8 * SWV) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int sl = s0 + SWV * u;
        v[u] = sl < sj.S ? src[(long)sl * ne] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    red[w][lane] = acc;
    __syncthreads();
    if (w != 0 || !ev) return;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < SWV; ++q) v += red[q][lane];
    const int mr = (int)(e / (sj.Kd + 1)), jc = (int)(e - (long)mr * (sj.Kd + 1));
    const long i = jc < sj.Kd ? sj.dw_off + (long)mr * sj.Kd + jc : sj.db_off + mr;
    g[i] = v;
    float pn, mn;
    sgd_update(v * grad_scale, p[i], m[i], lr, momentum, pn, mn);
    m[i] = mn;
    p[i] = pn;
    scatter_packed(ps, i, pn);
    return;
  }
  const long i = (long)((int)blockIdx.x - nsg) * TT + threadIdx.x;
  if (i >= n) return;
  for (int q = 0; q < ss.n; ++q) {  // owned by a slice role
    const SliceJob& sj = ss.it[q];
    if ((i >= sj.dw_off && i < sj.dw_off + (long)sj.M * sj.Kd) || (i >= sj.db_off && i < sj.db_off + sj.M)) return;
  }
  float pn, mn;
  sgd_update(g[i] * grad_scale, p[i], m[i], lr, momentum, pn, mn);
  m[i] = mn;
  p[i] = pn;
  scatter_packed(ps, i, pn);
}

inline unsigned blocks(long n) { return (unsigned)((n + LT - 1) / LT); }

}  // namespace

void launch_ingest(const uint8_t* images, const int32_t* labels, const int32_t* ids, int batch, int per_img,
                   float* out, int32_t* lab_out, hipStream_t s) {
  const long n = (long)batch * per_img;
  if (n) hipLaunchKernelGGL(ingest_kernel, dim3(blocks(n)), dim3(LT), 0, s, images, labels, ids, batch, per_img, out,
                            lab_out);
}
void launch_relu_pool_fwd(const float* x, int BC, int H, int W, float* y, uint8_t* code, hipStream_t s) {
  const long n = (long)BC * (H / 2) * (W / 2);
  if (n) hipLaunchKernelGGL(relu_pool_fwd_kernel, dim3(blocks(n)), dim3(LT), 0, s, x, BC, H, W, y, code);
}
void launch_relu_pool_bwd(const float* dy, const uint8_t* code, int BC, int H, int W, float* dx, hipStream_t s) {
  const long n = (long)BC * H * W;
  if (n) hipLaunchKernelGGL(relu_pool_bwd_kernel, dim3(blocks(n)), dim3(LT), 0, s, dy, code, BC, H, W, dx);
}
void launch_relu_fwd(const float* x, long n, float* y, hipStream_t s) {
  if (n) hipLaunchKernelGGL(relu_fwd_kernel, dim3(blocks(n)), dim3(LT), 0, s, x, n, y);
}
void launch_relu_bwd(const float* dy, const float* y, long n, float* dx, hipStream_t s) {
  if (n) hipLaunchKernelGGL(relu_bwd_kernel, dim3(blocks(n)), dim3(LT), 0, s, dy, y, n, dx);
}
int chan_parts(int B, int L) { return chan_parts_of(B, L); }

// float4 vectors when every plane row allows it (pool-routed gradients also need W % 4)
static bool vec4_ok(int L, int W, int act, std::initializer_list<const void*> ptrs) {
  if (L % 4 != 0 || (act == 2 && W % 4 != 0)) return false;
  for (const void* p : ptrs)
    if (p != nullptr && reinterpret_cast<uintptr_t>(p) % 16 != 0) return false;
  return true;
}
template <int ACT, int VW>
// ext_parts > 0: part already holds that many statistics partials per channel (the conv
// forward epilogue wrote them) - only the normalise / activate kernel runs
static void bn_fwd_launch(const float* x, int B, int C, int L, int W, const int32_t* state, const float* gamma,
                          const float* beta, float eps, float m, float* rmean, float* rvar, float* y, uint8_t* code,
                          float* smean, float* sinvstd, double* part, hipStream_t s, int ext_parts = 0) {
  const dim3 grid(chan_parts_of(B, L), C);
  if (ext_parts <= 0)
    hipLaunchKernelGGL((chan_partial_kernel<0, 0, VW>), grid, dim3(LT), 0, s, x, nullptr, B, C, L, state, nullptr,
                       nullptr, part, nullptr, ActArgs{});
  hipLaunchKernelGGL((bn_apply_train_kernel<ACT, VW>), grid, dim3(LT), 0, s, x, B, C, L, state, gamma, beta, eps, m,
                     rmean, rvar, y, smean, sinvstd, part, W, code, ext_parts > 0 ? ext_parts : (int)grid.x);
}
void launch_bn_fwd_train(const float* x, int B, int C, int L, const int32_t* state, const float* gamma,
                         const float* beta, float eps, float m, float* rmean, float* rvar, float* y, float* smean,
                         float* sinvstd, double* part, hipStream_t s) {
  if (!C) return;
  if (vec4_ok(L, 1, 0, {x, y}))
    bn_fwd_launch<0, 4>(x, B, C, L, 1, state, gamma, beta, eps, m, rmean, rvar, y, nullptr, smean, sinvstd, part, s);
  else
    bn_fwd_launch<0, 1>(x, B, C, L, 1, state, gamma, beta, eps, m, rmean, rvar, y, nullptr, smean, sinvstd, part, s);
}
void launch_bn_act_fwd_train(const float* x, int B, int C, int H, int W, const int32_t* state, const float* gamma,
                             const float* beta, float eps, float m, float* rmean, float* rvar, float* y, uint8_t* code,
                             float* smean, float* sinvstd, double* part, int act, hipStream_t s, int ext_parts) {
  if (!C) return;
  const int L = H * W;
  const bool v4 = vec4_ok(L, W, act == 2 ? 0 : act, {x, act == 2 ? nullptr : y});  // (pooled output: scalar)
#define BN_FWD(A, V) bn_fwd_launch<A, V>(x, B, C, L, W, state, gamma, beta, eps, m, rmean, rvar, y, code, smean, \
                                          sinvstd, part, s, ext_parts)
  if (act == 1) { if (v4) BN_FWD(1, 4); else BN_FWD(1, 1); }
  else if (act == 2) { if (v4) BN_FWD(2, 4); else BN_FWD(2, 1); }
  else { if (v4) BN_FWD(0, 4); else BN_FWD(0, 1); }
#undef BN_FWD
}
void launch_bn_fwd_eval(const float* x, int B, int C, int L, const float* gamma, const float* beta, float eps,
                        const float* rmean, const float* rvar, float* y, hipStream_t s) {
  const long n = (long)B * C * L;
  if (n) hipLaunchKernelGGL(bn_fwd_eval_kernel, dim3(blocks(n)), dim3(LT), 0, s, x, B, C, L, gamma, beta, eps, rmean,
                            rvar, y);
}
template <int ACT, int VW>
// ext_parts > 0: part already holds that many backward-statistics partials per channel (the
// producing conv data gradient's epilogue wrote them) - only the apply kernel runs
static void bn_act_bwd(const float* dy, const float* x, int B, int C, int L, const int32_t* state, const float* gamma,
                       const float* smean, const float* sinvstd, float* dx, float* dgamma, float* dbeta, double* part,
                       ActArgs aa, hipStream_t s, int ext_parts = 0) {
  const dim3 grid(chan_parts_of(B, L), C);
  if (ext_parts <= 0)
    hipLaunchKernelGGL((chan_partial_kernel<1, ACT, VW>), grid, dim3(LT), 0, s, dy, x, B, C, L, state, smean, sinvstd,
                       part, gamma, aa);
  hipLaunchKernelGGL((bn_bwd_apply_kernel<ACT, VW>), grid, dim3(LT), 0, s, dy, x, B, C, L, state, gamma, smean,
                     sinvstd, dx, dgamma, dbeta, part, aa, ext_parts > 0 ? ext_parts : (int)grid.x);
}
void launch_bn_bwd(const float* dy, const float* x, int B, int C, int L, const int32_t* state, const float* gamma,
                   const float* smean, const float* sinvstd, float* dx, float* dgamma, float* dbeta, double* part,
                   hipStream_t s) {
  if (!C) return;
  if (vec4_ok(L, 1, 0, {dy, x, dx}))
    bn_act_bwd<0, 4>(dy, x, B, C, L, state, gamma, smean, sinvstd, dx, dgamma, dbeta, part, ActArgs{}, s);
  else
    bn_act_bwd<0, 1>(dy, x, B, C, L, state, gamma, smean, sinvstd, dx, dgamma, dbeta, part, ActArgs{}, s);
}
void launch_bn_act_bwd(const float* dy, const float* x, int B, int C, int H, int W, const int32_t* state,
                       const float* gamma, const float* beta, const float* smean, const float* sinvstd,
                       const uint8_t* code, float* dx, float* dgamma, float* dbeta, double* part, int act,
                       hipStream_t s, int ext_parts) {
  if (!C) return;
  const int L = H * W;
  const ActArgs aa{beta, code, W, H / 2};
  const bool v4 = vec4_ok(L, W, act, {act == 2 ? nullptr : dy, x, dx});
#define BN_BWD(A, V) \
  bn_act_bwd<A, V>(dy, x, B, C, L, state, gamma, smean, sinvstd, dx, dgamma, dbeta, part, aa, s, ext_parts)
  if (act == 1) { if (v4) BN_BWD(1, 4); else BN_BWD(1, 1); }
  else if (act == 2) { if (v4) BN_BWD(2, 4); else BN_BWD(2, 1); }
  else { if (v4) BN_BWD(0, 4); else BN_BWD(0, 1); }
#undef BN_BWD
}
void launch_chan_sum(const float* a, int B, int C, int L, float* out, double* part, hipStream_t s) {
  if (!C) return;
  const int P = chan_parts_of(B, L);
  hipLaunchKernelGGL((chan_partial_kernel<2, 0, 1>), dim3(P, C), dim3(LT), 0, s, a, nullptr, B, C, L, nullptr,
                     nullptr, nullptr, part, nullptr, ActArgs{});
  hipLaunchKernelGGL(chan_sum_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, s, part, C, P, out);
}
void launch_xent(const float* logits, const int32_t* labels, int B, int NC, const int32_t* state, float* loss,
                 int32_t* correct, float* dlogits, hipStream_t s) {
  if (B) hipLaunchKernelGGL(xent_kernel, dim3(blocks(B)), dim3(LT), 0, s, logits, labels, B, NC, state, loss, correct,
                            dlogits);
}
void launch_layer_bookkeeping(const ReduceArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(layer_bookkeeping_kernel, dim3(1), dim3(64), 0, s, a);
}
void launch_sgd_flat(float* p, const float* g, float* m, long n, float lr, float momentum, float grad_scale,
                     hipStream_t s) {
  if (n) hipLaunchKernelGGL(sgd_flat_kernel, dim3(blocks(n)), dim3(LT), 0, s, p, g, m, n, lr, momentum, grad_scale);
}

void launch_sgd_tail(float* p, float* g, float* m, long n, float lr, float momentum, float grad_scale,
                     const ConvPackJob* jobs, int njobs, const float* arena, const SliceJob* slices, int nslices,
                     const ReduceArgs* book, hipStream_t s) {
  PackScatter ps{};
  if (njobs > PackScatter::kMax) throw std::runtime_error("sgd_tail: too many packed conv images");
  for (int j = 0; j < njobs; ++j) {
    const ConvPackJob& J = jobs[j];
    PackScatter::Item& it = ps.it[ps.n++];
    conv_pack_geometry(J, &it.M, &it.C, &it.K, &it.Mp, &it.Cp);
    it.off = J.w - arena;
    it.len = (long)it.M * it.C * it.K * it.K;
    if (it.off < 0 || it.off + it.len > n) throw std::runtime_error("sgd_tail: packed weight outside the arena");
    it.dst = J.dst;
    it.flip = J.flip;
    it.bf = J.bf16_ops;
  }
  SliceSet ss{};
  if (nslices > SliceSet::kMax) throw std::runtime_error("sgd_tail: too many deferred slice sums");
  ss.start[0] = 0;
  for (int j = 0; j < nslices; ++j) {
    const SliceJob& sj = slices[j];
    if (sj.S <= 0 || sj.M <= 0 || sj.Kd <= 0 || sj.dw_off < 0 || sj.dw_off + (long)sj.M * sj.Kd > n || sj.db_off < 0 ||
        sj.db_off + sj.M > n)
      throw std::runtime_error("sgd_tail: slice job outside the arena");
    ss.it[ss.n++] = sj;
    ss.start[j + 1] = ss.start[j] + (int)(((long)sj.M * (sj.Kd + 1) + 63) / 64);
  }
  const unsigned nb = (unsigned)(ss.start[ss.n] + (n + TT - 1) / TT) + (book != nullptr ? 1u : 0u);
  if (book != nullptr)
    hipLaunchKernelGGL(sgd_tail_kernel<true>, dim3(nb), dim3(TT), 0, s, p, g, m, n, lr, momentum, grad_scale, ps,
                       ss, *book);
  else
    hipLaunchKernelGGL(sgd_tail_kernel<false>, dim3(nb), dim3(TT), 0, s, p, g, m, n, lr, momentum, grad_scale, ps,
                       ss, ReduceArgs{});
  HIP_CHECK(hipGetLastError());
}

}  // namespace dnn

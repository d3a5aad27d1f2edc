// Device code of the batch gradient reduction + momentum SGD of the grad_reduce kernel
// (reduce_sgd.hip) and the step bookkeeping shared with the layer engine's kernels
// (layers.hip).  See reduce_sgd.hip for the parity notes.
#pragma once
#include "launchers.h"

namespace dnn {

// The pipelined step's reduction (lenet_fused.hip, PIPE): the new parameters and their bf16
// images are stored WRITE-THROUGH (sc1), because the sample workgroups of the same launch load
// them (sc1 loads) once the storing block has drained its stores and added to its ready counter
// (MI355X guide §6 G16 R1).  The momentum is read by the next launch only: plain stores.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(bf16* p, bf16 v) {
  __hip_atomic_store(reinterpret_cast<unsigned short*>(p), __builtin_bit_cast(unsigned short, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// write_shadow (common.h) with write-through stores where the samples of the same launch read
// the bytes: the kernel-ready images and the fc3 rows.  The row-major conv copy and every bias
// copy are read by later launches only (the samples take the biases from the fp32 master): plain.
__device__ __forceinline__ void write_shadow_wt(bf16* __restrict__ sh, int e, float p) {
  const bf16 v = (bf16)p;
  if (e >= OFF_F3W && e < OFF_F3W + 840) st_wt(sh + e, v);
  else sh[e] = v;
  if (e >= OFF_C1W && e < OFF_C1W + 450) {
    const int r = e - OFF_C1W, n = r / 75, rem = r - 75 * n, c = rem / 25, ky = (rem % 25) / 5, kx = rem % 5;
    st_wt(sh + SH_W1F + ((c * 5 + ky) * 16 + 2 * n) * 8 + kx, v);  // (common.h write_shadow: both shifts)
    st_wt(sh + SH_W1F + ((c * 5 + ky) * 16 + 2 * n + 1) * 8 + kx + 1, v);
  } else if (e >= OFF_C2W && e < OFF_C2W + 2400) {
    const int r = e - OFF_C2W, n = r / 150, rem = r - 150 * n, c = rem / 25, ky = (rem % 25) / 5, kx = rem % 5;
    st_wt(sh + SH_W2F + ((c * 5 + ky) * 16 + n) * 8 + kx, v);
    st_wt(sh + SH_WF + (((4 - ky) * 16 + n) * 16 + c) * 8 + (4 - kx), v);
  } else if (e >= OFF_F2W && e < OFF_F2W + 10080) {
    const int r = e - OFF_F2W, o = r / 120, i = r - 120 * o;
    st_wt(sh + SH_W2T + i * 96 + o, v);
  } else if (e >= OFF_F3W && e < OFF_F3W + 840) {
    const int r = e - OFF_F3W, o = r / 84, i = r - 84 * o;
    st_wt(sh + SH_W3T + i * 16 + o, v);
  }
}

__device__ __forceinline__ bool is_bias(int e) {
  return (e >= OFF_C1B && e < OFF_C1B + 6) || (e >= OFF_C2B && e < OFF_C2B + 16) || (e >= OFF_F1B && e < OFF_F1B + 120) ||
         (e >= OFF_F2B && e < OFF_F2B + 84) || (e >= OFF_F3B && e < OFF_F3B + 10);
}

// SGD epilogue with the master/momentum values already in registers (prefetched
// together with the gradient operands, so the update costs no extra memory latency).
// WT: write-through parameter / image stores (the pipelined step).
template <bool WT = false>
__device__ __forceinline__ void sgd_finish(int e, float g, float p_old, float m_old, const ReduceArgs& a) {
  g *= a.grad_scale;
  if (a.fuse_sgd) {
    float p, m;
    sgd_update(g, p_old, m_old, a.lr, a.momentum, p, m);
    a.mom[e] = m;
    if constexpr (WT) {
      // the samples read the biases from the fp32 master, every weight from the bf16 images:
      // only those bytes go write-through; the rest of master is read by the next launch
      if (is_bias(e)) st_wt(a.master + e, p);
      else a.master[e] = p;
      write_shadow_wt(a.shadow, e, p);
    } else {
      a.master[e] = p;
      write_shadow(a.shadow, e, p);
    }
  } else {
    a.grad[e] = g;
  }
}

// Where a lane's reduced elements go (at most 4 per lane; j is a compile-time index once the
// callers' loops are unrolled, so the exchange sink's arrays stay in registers).
//  * DirectSink: finish at once (local SGD step, or gradient output); WtSink: the same with
//    write-through stores (the pipelined step's in-launch reduction).
//  * XpSink (one-launch xGMI all-reduce, reduce_sgd.hip): the gradient goes to this rank's
//    granule slot now as one 8-byte {value, step} word (system-coherent store); the update
//    runs after the lane has read the same element from every peer.
template <bool WT>
struct DirectSinkT {
  static constexpr bool kTile = WT;  // fc1 / fc2 tiles finish in put_tile (below)
  static constexpr bool kTileInfo = false;  // (XpSinkT<PK, true> records its fc tile: see there)
  static constexpr bool kOpaqueLane = false;
  // WT, optional: put_tile's write-through stores wait until *gate >= gate_target (the pipelined
  // step's conv ready counter): the samples' poll of that counter then does not queue behind the
  // MLP tiles' write-through traffic (lenet_fused.hip PIPE flags & 32)
  const unsigned* gate = nullptr;
  unsigned gate_target = 0;
  __device__ __forceinline__ void put(int, int e, float g, float p, float m, const ReduceArgs& a) {
    sgd_finish<WT>(e, g, p, m, a);
  }
  // A finished fc1 / fc2 weight-gradient tile (lane (i, kq) holds rows o0 + 4 kq + j of column
  // i0 + i): SGD per element (master / momentum plain: the samples read no fc weight from the
  // fp32 master), then the bf16 images with 8-byte write-through stores instead of one 2-byte
  // store per element - a 4 x 4 transpose inside each lane quad (DPP rotations) gives lane u
  // the 4 consecutive columns of row o0 + 4 kq + u for the row-major copy; the transposed fc2
  // image [i][o] takes the lane's own 4 consecutive rows as they are.
  template <int LAYER>
  __device__ __forceinline__ void put_tile(const f32x4& acc, const float (&pv)[4], const float (&mv)[4],
                                           const int (&e)[4], int o0, int i0, int lane, const ReduceArgs& a);
};
using DirectSink = DirectSinkT<false>;
using WtSink = DirectSinkT<true>;

// The fp32 engine's persistent launch (lenet_f32.hip PERS): its samples read EVERY weight from
// the fp32 master, so every new parameter is stored write-through there at once; the momentum and
// the bf16 shadow are read by later steps of the same block / later launches only, so their
// stores are held back (up to 4 per lane) and issued by flush() after the block signalled ready -
// the drain before the ready word then waits for the master stores alone.  No tile path: the fc
// tiles finish per element, with DirectSink's arithmetic (bit-identical to the serial fp32 step).
struct WtF32Sink {
  static constexpr bool kTile = false;
  static constexpr bool kTileInfo = false;
  static constexpr bool kOpaqueLane = true;
  int e[4];
  float p[4], m[4];
  bool v[4] = {false, false, false, false};
  __device__ __forceinline__ void put(int j, int e_, float g, float p_old, float m_old, const ReduceArgs& a) {
    g *= a.grad_scale;
    sgd_update(g, p_old, m_old, a.lr, a.momentum, p[j], m[j]);
    e[j] = e_;
    v[j] = true;
    st_wt(a.master + e_, p[j]);
  }
  __device__ __forceinline__ void flush(const ReduceArgs& a) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (v[j]) {
        a.mom[e[j]] = m[j];
        write_shadow(a.shadow, e[j], p[j]);
      }
  }
  template <int LAYER>
  __device__ __forceinline__ void put_tile(const f32x4&, const float (&)[4], const float (&)[4], const int (&)[4], int,
                                           int, int, const ReduceArgs&) {}
};

// lane u of a quad reads lane (u + R) & 3's value
template <int R>
__device__ __forceinline__ unsigned qrot(unsigned v) {
  constexpr int c = (R & 3) | (((1 + R) & 3) << 2) | (((2 + R) & 3) << 4) | (((3 + R) & 3) << 6);
  return (unsigned)__builtin_amdgcn_mov_dpp((int)v, c, 0xf, 0xf, false);
}
__device__ __forceinline__ unsigned sel4(const unsigned (&x)[4], int k) {
  return k == 0 ? x[0] : k == 1 ? x[1] : k == 2 ? x[2] : x[3];
}
// b[u][v] = a[v][u] over the 4 lanes u of a quad (a[lane][element])
// (lane u receives a[k][u] from lane k = (u + r) & 3, which sends its element (k - r) & 3 = u)
__device__ __forceinline__ void quad_transpose(const unsigned (&x)[4], unsigned (&y)[4], int u) {
  const unsigned r0 = sel4(x, u), r1 = qrot<1>(sel4(x, (u - 1) & 3)), r2 = qrot<2>(sel4(x, (u - 2) & 3)),
                 r3 = qrot<3>(sel4(x, (u - 3) & 3));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = (k - u) & 3;
    y[k] = r == 0 ? r0 : r == 1 ? r1 : r == 2 ? r2 : r3;
  }
}

__device__ __forceinline__ void st_wt8(bf16* p, unsigned lo, unsigned hi) {  // 4 bf16, 8-B aligned
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)lo | ((unsigned long long)hi << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The write-through SGD + image update of a finished fc1 / fc2 weight-gradient tile (lane (i, kq)
// holds rows o0 + 4 kq + j of column i0 + i): SGD per element (master / momentum plain: the
// samples read no fc weight from the fp32 master), then the bf16 images with 8-byte write-through
// stores - a 4 x 4 transpose inside each lane quad (DPP rotations) gives lane u the 4 consecutive
// columns of row o0 + 4 kq + u for the row-major copy; the transposed fc2 image [i][o] takes the
// lane's own 4 consecutive rows as they are.  Every lane of the wave calls it (DPP).
template <int LAYER>
__device__ __forceinline__ void wt_tile_update(const f32x4& acc, const float (&pv)[4], const float (&mv)[4],
                                               const int (&e)[4], int o0, int i0, int lane, const ReduceArgs& a) {
  constexpr int O = LAYER == 0 ? 120 : 84, I = LAYER == 0 ? 400 : 120, OFF = LAYER == 0 ? OFF_F1W : OFF_F2W;
  const int i = lane & 15, kq = lane >> 4, u = lane & 3;
  const bool iv = i0 + i < I;
  unsigned bv[4];  // this lane's column, rows o0 + 4 kq + j: bf16 bits (0 outside the layer)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool ok = iv && o0 + 4 * kq + j < O;
    float p = 0.f;
    if (ok) {
      float m;
      sgd_update(acc[j] * a.grad_scale, pv[j], mv[j], a.lr, a.momentum, p, m);
      a.mom[e[j]] = m;
      a.master[e[j]] = p;
    }
    bv[j] = ok ? (unsigned)__builtin_bit_cast(unsigned short, (bf16)p) : 0u;
  }
  // row-major bf16 copy: lane u of the quad -> row o0 + 4 kq + u, columns i0 + (i & ~3) .. + 3
  unsigned t[4];
  quad_transpose(bv, t, u);
  const int row = o0 + 4 * kq + u, c0 = i0 + (i & ~3);
  if (row < O && c0 < I) st_wt8(a.shadow + OFF + row * I + c0, t[0] | (t[1] << 16), t[2] | (t[3] << 16));
  if constexpr (LAYER == 1) {  // fc2^T image [i][96]: this lane's 4 consecutive rows o0 + 4 kq ..
    if (iv && o0 + 4 * kq < O) st_wt8(a.shadow + SH_W2T + (i0 + i) * 96 + o0 + 4 * kq, bv[0] | (bv[1] << 16),
                                      bv[2] | (bv[3] << 16));
  }
}

template <bool WT>
template <int LAYER>
__device__ __forceinline__ void DirectSinkT<WT>::put_tile(const f32x4& acc, const float (&pv)[4], const float (&mv)[4],
                                                         const int (&e)[4], int o0, int i0, int lane,
                                                         const ReduceArgs& a) {
  if (gate != nullptr && lane == 0) {  // bounded: the samples' own wait on this counter has the timeout
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gate_target &&
           wall_clock64() - t0 < 200000000ll)
      __builtin_amdgcn_s_sleep(4);
  }
  wt_tile_update<LAYER>(acc, pv, mv, e, o0, i0, lane, a);
}
//    PK (bf16 granules, xp_mode bit 4): the lane's elements travel in pairs (0, 1) and (2, 3)
//    as ONE granule {bf16 | bf16, step} each, published by the exchange once both are known.
//    WT (the persistent launch's in-launch exchange, lenet_fused.hip PERS): the update after the
//    exchange stores what the samples of the same launch read write-through - an fc1 / fc2 tile
//    through wt_tile_update (the lane records its tile: tile_info), every other element as
//    sgd_finish<true> does.  F32 (with WT: the fp32 kernel's persistent launch, lenet_f32.hip
//    PERS): its samples read every weight from the fp32 master, so every new parameter is stored
//    write-through there (WtF32Sink's stores), the momentum and the bf16 shadow plainly.
template <bool PK, bool WT = false, bool F32 = false>
struct XpSinkT {
  static_assert(!F32 || (WT && !PK), "the fp32 persistent exchange: write-through, fp32 granules");
  static constexpr bool kPK = PK, kWT = WT, kF32 = F32;
  static constexpr bool kTile = false;
  static constexpr bool kTileInfo = WT && !F32;
  static constexpr bool kOpaqueLane = F32;  // (the fp32 launch: 128 VGPRs, see WtF32Sink)
  static constexpr int kRC = F32 ? 2 : 8;     // peer ranks per polling round (reduce_device.h gather_rank_sum)
  int tl = -1, to0 = 0, ti0 = 0;  // WT: the fc tile (layer, o0, i0) this lane's elements belong to
  template <int LAYER>
  __device__ __forceinline__ void tile_info(int o0, int i0) {
    tl = LAYER;
    to0 = o0;
    ti0 = i0;
  }
  template <int LAYER>
  __device__ __forceinline__ void put_tile(const f32x4&, const float (&)[4], const float (&)[4], const int (&)[4], int,
                                           int, int, const ReduceArgs&) {}
  unsigned long long* own;  // where the granules go: this rank's pull slot (null: not published)
  unsigned long long tag;   // step << 32
  int e[4] = {0, 0, 0, 0};
  float g[4] = {0.f, 0.f, 0.f, 0.f}, p[4], m[4];
  bool v[4] = {false, false, false, false};
  // WT: the prefetched master / momentum values wait out the exchange in LDS instead of 8
  // registers ([8][stride] floats from this thread's slot: p[j] at j * stride, m[j] at (4 + j) *
  // stride) - the persistent launch's reduction path is at the 256-VGPR limit (its workgroups use
  // no other LDS).  The stash must be set.
  int stash = 0, stride = 0;  // this thread's first stash float, floats between its values
  __device__ __forceinline__ static float* lds() {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    return reinterpret_cast<float*>(smem);
  }
  __device__ __forceinline__ float pv(int j) const {
    if constexpr (WT) return lds()[stash + j * stride];
    else return p[j];
  }
  __device__ __forceinline__ float mv(int j) const {
    if constexpr (WT) return lds()[stash + (4 + j) * stride];
    else return m[j];
  }
  __device__ __forceinline__ void put(int j, int e_, float g_, float p_, float m_, const ReduceArgs& a) {
    g_ *= a.grad_scale;
    e[j] = e_; g[j] = g_; v[j] = true;
    if constexpr (WT) {
      lds()[stash + j * stride] = p_;
      lds()[stash + (4 + j) * stride] = m_;
    } else {
      p[j] = p_;
      m[j] = m_;
    }
    if (!PK && own != nullptr)  // (two-hop form: null on the owner of the block's elements)
      __hip_atomic_store(own + e_, tag | __float_as_uint(g_), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
};
using XpSink = XpSinkT<false>;

// fc weight-gradient tiles: dW[o][i] = sum_b z[b][o] * x[b][i]  (K = batch), one 16x16
// output tile per wave on v_mfma_f32_16x16x4_f32 (exact fp32 fma chains, fixed order).
template <int LAYER> struct Fc;
template <> struct Fc<0> { static constexpr int O = 120, I = 400, IT = 25, OFF = OFF_F1W, ZLD = Z1_LD, XLD = A0_LD; };
template <> struct Fc<1> { static constexpr int O = 84, I = 120, IT = 8, OFF = OFF_F2W, ZLD = Z2_LD, XLD = H1_LD; };
template <> struct Fc<2> { static constexpr int O = 10, I = 84, IT = 6, OFF = OFF_F3W, ZLD = Z3_LD, XLD = H2_LD; };
constexpr int FC_T0 = 8 * 25, FC_T1 = 6 * 8, FC_T2 = 1 * 6;
constexpr int FC_TILES = FC_T0 + FC_T1 + FC_T2;   // 254 wave-tiles
constexpr int TILE_BLOCKS = (FC_TILES + 3) / 4;  // 4 waves per block

// A per-sample row element: plain, or (SC: the persistent launch, lenet_fused.hip PERS) an sc1
// load of a row the sample workgroups of the same launch stored write-through
template <bool SC>
__device__ __forceinline__ float ldrow(const float* p) {
  if constexpr (SC)
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
  else return *p;
}

// SC / rp (the persistent launch): sc1 row loads, rows of parity rp (rp * batch rows further on)
template <int LAYER, class Sink, bool SC = false>
__device__ __forceinline__ void fc_tile(int t, const ReduceArgs& a, Sink& sk, int rp = 0) {
  using L = Fc<LAYER>;
  const float* z = LAYER == 0 ? a.z1 : (LAYER == 1 ? a.z2 : a.z3);
  const float* x = LAYER == 0 ? a.a0 : (LAYER == 1 ? a.h1 : a.h2);
  if constexpr (SC) {  // (the persistent launch's row parity)
    z += (long)rp * a.batch * L::ZLD;
    x += (long)rp * a.batch * L::XLD;
  }
  int lane = threadIdx.x & 63;
  // (kOpaqueLane: the fp32 persistent launch calls this once per step at 128 VGPRs - an opaque
  // lane keeps its per-lane offsets inside the step instead of hoisted out of the step loop)
  if constexpr (Sink::kOpaqueLane) asm volatile("" : "+v"(lane));
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
  // two interleaved accumulator chains (even / odd K-steps, summed at the end): the dependent
  // MFMA chain per tile is 8 deep instead of 16 (this tile is the reduce launch's critical path)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int omc = ov ? om : 0, inc = iv ? in : 0;
  for (int b0 = 0; b0 < a.batch; b0 += 64) {
    // every operand load is unconditional (clamped address) and issued before the first
    // MFMA; out-of-range operands are zeroed by a select afterwards
    float av[16], bv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int b = min(b0 + 4 * s + kq, a.batch - 1);
      av[s] = ldrow<SC>(z + b * L::ZLD + omc);
      bv[s] = ldrow<SC>(x + b * L::XLD + inc);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool bvld = b0 + 4 * s + kq < a.batch;
      av[s] = (bvld && ov) ? av[s] : 0.f;
      bv[s] = (bvld && iv) ? bv[s] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s + 1], bv[s + 1], acc1, 0, 0, 0);
    }
  }
  acc += acc1;
  if constexpr (Sink::kTileInfo) sk.template tile_info<LAYER>(o0, i0);
  if constexpr (Sink::kTile && LAYER < 2) {  // the pipelined step: wide write-through image stores
    sk.template put_tile<LAYER>(acc, pv, mv, e, o0, i0, lane, a);
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = o0 + 4 * kq + j;
    if (o < L::O && iv) sk.put(j, e[j], acc[j], pv[j], mv[j], a);
  }
}

// Column sums (fc biases: sum_b z[b][o]; conv slab columns: sum_b slab[b][j]) with SPLIT = 4
// consecutive lanes per column: lane part q sums rows {64 c + 16 q + k}, then the 4
// partials combine as (p0 + p1) + (p2 + p3) through lane shuffles - a fixed order (bitwise
// reproducible), 16-load chains
// instead of 64, 4x the threads in flight.
constexpr int SPLIT = 4;
template <bool SC = false>
__device__ __forceinline__ float column_sum_split(const float* src, int ld, int col, int batch, int q) {
  float g = 0.f;
  for (int b0 = 0; b0 < batch; b0 += 64) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = ldrow<SC>(src + min(b0 + 16 * q + k, batch - 1) * ld + col);
    __builtin_amdgcn_sched_barrier(0);  // all 16 loads in flight before the first wait
#pragma unroll
    for (int k = 0; k < 16; ++k) g += (b0 + 16 * q + k < batch) ? v[k] : 0.f;
  }
  g += __shfl_xor(g, 1);  // (p0 + p1), (p2 + p3) ...
  g += __shfl_xor(g, 2);  // ... then their sum, identical in all 4 lanes
  return g;
}

// fc-bias slots: columns padded per source to multiples of 16 (one wave = 16 columns), so
// each wave reads ONE source (wave-uniform base pointer): fc1 [0,128)
// (120 used), fc2 [128,224) (84 used), fc3 [224,240) (10 used); slot = column * 4 + q.
constexpr int FCB_ELEMS = 120 + 84 + 10;
constexpr int FCB_COLS = 128 + 96 + 16;
constexpr int FCB_SLOTS = FCB_COLS * SPLIT;  // 960
template <class Sink, bool SC = false>
__device__ __forceinline__ void fcb_task(int t, const ReduceArgs& a, Sink& sk, int rp = 0) {
  const int tc = min(t, FCB_SLOTS - 1);
  const int grp = __builtin_amdgcn_readfirstlane(tc / (16 * SPLIT));  // wave-uniform source
  const int colp = tc / SPLIT, q = t % SPLIT;
  // each source has its own column-sum call: a select of the three row pointers was folded into a
  // dynamic index into the by-value argument block, which the compiler copied to scratch
  int ld, col, n, off;
  if (grp < 8) { ld = Z1_LD; col = colp; n = 120; off = OFF_F1B; }
  else if (grp < 14) { ld = Z2_LD; col = colp - 128; n = 84; off = OFF_F2B; }
  else { ld = Z3_LD; col = colp - 224; n = 10; off = OFF_F3B; }
  const int cc = min(col, n - 1);  // padding lanes recompute a real column (no divergence)
  const int dst = off + cc;
  const float pv = a.master[dst], mv = a.mom[dst];  // (unused if !fuse_sgd)
  const long rb = SC ? (long)rp * a.batch : 0;  // (the persistent launch's row parity)
  float g;  // every lane shuffles: no early exit
  if (grp < 8)
    g = column_sum_split<SC>(a.z1 + rb * Z1_LD, Z1_LD, cc, a.batch, q);
  else if (grp < 14)
    g = column_sum_split<SC>(a.z2 + rb * Z2_LD, Z2_LD, cc, a.batch, q);
  else
    g = column_sum_split<SC>(a.z3 + rb * Z3_LD, Z3_LD, cc, a.batch, q);
  if (t < FCB_SLOTS && col < n && q == 0) sk.put(0, dst, g, pv, mv, a);
}

constexpr int CONV_ELEMS = SLAB;
constexpr int CONV_SLOTS = CONV_ELEMS * SPLIT;  // 11,488
__device__ __forceinline__ int conv_dst(int e) {
  if (e < SLAB_C1B) return OFF_C1W + e;
  if (e < SLAB_C2W) return OFF_C1B + (e - SLAB_C1B);
  if (e < SLAB_C2B) return OFF_C2W + (e - SLAB_C2W);
  return OFF_C2B + (e - SLAB_C2B);
}
template <class Sink, bool SC = false>
__device__ __forceinline__ void conv_task(int t, const ReduceArgs& a, Sink& sk, int rp = 0) {
  const float* src = a.slab;
  if constexpr (SC) src += (long)rp * a.batch * SLAB;
  const int e = min(t / SPLIT, CONV_ELEMS - 1), q = t % SPLIT;
  const int dst = conv_dst(e);
  const float pv = a.master[dst], mv = a.mom[dst];  // (unused if !fuse_sgd)
  const float g = column_sum_split<SC>(src, SLAB, e, a.batch, q);
  if (t < CONV_SLOTS && q == 0) sk.put(0, dst, g, pv, mv, a);
}

// Epoch statistics of the step that just ran + publication of the next step's cursor,
// valid count and sample ids.  One wave (lanes 0..63), fixed summation order.
__device__ __forceinline__ void bookkeeping(const ReduceArgs& a, int lane) {
    const float* loss = a.loss;
    const int32_t* correct = a.correct;
    float ls = 0.f;
    int cs = 0;
    // bvalid of the step whose statistics are added: read before any slot is published (the
    // pipelined step's bk_bv_in and bk_bv_out may be the same word)
    const int bv = a.bk_bv_in != nullptr ? *a.bk_bv_in : a.state[ST_BVALID];
    for (int b = lane; b < (a.bk_stats ? a.batch : 0); b += 64) {
      ls += loss[b];
      cs += correct[b];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) { ls += __shfl_down(ls, off); cs += __shfl_down(cs, off); }
    const int next = a.state[ST_CURSOR] + a.bk_adv;
    if (lane == 0 && bv > 0 && a.bk_stats) {
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
    if (a.next_ids != nullptr) {  // and the step after it (image staging, lenet_fused.hip)
      for (int b = lane; b < a.batch; b += 64) {
        const long g = base + a.batch + b;
        a.next_ids[b] = g < a.order_len ? a.order[g] : -1;
      }
    }
    const long rem = (long)a.order_len - base;
    const int nbv = rem < a.batch ? (rem > 0 ? (int)rem : 0) : a.batch;
    if (lane == 0) {
      a.state[ST_CURSOR] = next;
      *(a.bk_bv_out != nullptr ? a.bk_bv_out : a.state + ST_BVALID) = nbv;
    }
}

}  // namespace dnn

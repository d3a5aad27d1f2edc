// Fused per-sample forward + data-backward + conv weight-gradient kernel, fp32 (gfx950).
//
// Capability parity: the reference trains in fp32 (models/model.py:13-18,
// data_parallelism_train.py:187-199); this is the fp32 counterpart of lenet_fused.hip (bf16
// MFMA operands).  One workgroup runs, for ONE CIFAR image, the ToTensor/Normalize ingest
// (data_parallelism_train.py:24-27), conv/relu/maxpool/linear/CrossEntropy forward and every
// backward op down to the conv weight gradients, writing the same
// per-sample rows as the bf16 kernel (pooled conv2 output, MLP activations and deltas, the
// conv weight/bias-gradient slab, loss, correct) - the batch reduction + SGD (grad_reduce,
// reduce_sgd.hip) is shared and already fp32.
//
// Every multiply-add is an fp32 fma with fp32 operands: results differ from PyTorch's fp32 CPU
// path only by summation order (~1e-6 relative; tests/test_kernels_gpu.py pins 1e-4).
//
// MI355X design (why VALU and not MFMA here): f32-input MFMA runs at the f32 VALU rate
// (v_mfma_f32_16x16x4_f32: 32 MAC/clk/SIMD = v_pk_fma_f32, MI355X_MICROARCH.md), so MFMA only
// pays where its 16-wide tiles are full.  This net's convolutions have 6 output channels
// (conv1 fwd/wgrad, conv2 dgrad) - a 16-wide MFMA tile would waste 62 % - so every product is a
// register-blocked packed fma (v_pk_fma_f32: two outputs per instruction) on the VALU:
//  * one workgroup = one sample = 16 waves (1024 threads); everything lives in LDS (~137 KB),
//    except fc1 (192 KB fp32 > LDS): each wave streams 8 of its rows ONCE from L2 into
//    registers, uses them for the forward GEMV, keeps them through the loss, and reuses the
//    same registers for the fc1 data gradient - no second pass over fc1;
//  * ReLU + 2x2 maxpool fused into the conv epilogues with a 2-bit argmax code (4 = no
//    gradient), exactly as lenet_fused.hip (first max wins, like torch.max_pool2d);
//  * the conv1 weight gradient exploits the max-pool sparsity: dY = unpool(d pooled) has ONE
//    nonzero per 2x2 window, so dW1 sums over the <= 196 active argmax pixels instead of the 784
//    dense ones (4x fewer products; zeros add nothing in fp32);
//  * the conv2 weight gradient is the one GEMM whose M (16 output channels) fills an MFMA tile:
//    it runs dense (k = the 100 unpooled pixels) on v_mfma_f32_16x16x4_f32 in 5 waves, beside the
//    data gradient's VALU work in the other 11;
//  * fixed summation orders everywhere (no atomics): bitwise reproducible run to run.
#include "pers_common.h"
#include "runtime/aql_dispatch.h"

namespace dnn {
namespace f32k {

constexpr int NT = 1024;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// ---- LDS map (bytes) ----------------------------------------------------------------
// Strides chosen against the 64 x 4 B LDS banks (MI355X_MICROARCH.md §LDS; searched with a bank
// model for each access pattern): X rows of 46 floats make conv1's 8-byte patch reads
// conflict-free; P1 channels of 198 floats keep conv2's weight-gradient reads <= 2-way; the conv1
// weight gradient reads a re-strided copy XW (rows 33, channels 1061: conflict-free) that phase E
// builds in the dead fc2 region.
constexpr int X_RS = 46, X_CH = 32 * X_RS;        // normalised image [3][32][46]
constexpr int XW_RS = 33, XW_CH = 1061;           // its copy for the conv1 weight gradient
constexpr int P1_CH = 198;                        // pooled conv1 output [6][198] (14 x 14 used)
constexpr int WD_LD = 28;                         // conv2 dgrad weights [6 c][16 o][28] (25 used),
constexpr int WD_CPAD = 4;                        // + 4 floats per c: c and c + 1 rows 16 B apart in the banks
constexpr int L_X = 0;                  // f32 [3][X_CH] normalised image                17664
// forward weights by output-channel PAIR p: [p][c][ky][6 (kx, padded)][2 (o = 2p, 2p + 1)], so
// one 16-B read delivers two taps of both channels (the packed-fma operand pairs), a kernel row
// in three reads
constexpr int WP_R = 12, WP_C = 5 * WP_R;  // floats per (pair, c, ky) / per (pair, c)
constexpr int L_WT1 = L_X + 17664;      // f32 [3 p][3 c][WP_C] conv1 weights             2160
constexpr int L_WT2 = L_WT1 + 2160;     // f32 [8 p][6 c][WP_C] conv2 weights            11520
constexpr int L_WD = L_WT2 + 11520;     // f32 [6][16][WD_LD] (+ c pad) conv2 dgrad weights 10848
constexpr int L_P1 = L_WD + 10848;      // f32 [6][P1_CH] pooled conv1 output          4752
constexpr int L_C1 = L_P1 + 4752;       // u8  [6][196] conv1 pool codes                1184
constexpr int L_A0 = L_C1 + 1184;       // f32 [400] pooled conv2 output (flatten order) 1600
constexpr int L_C2 = L_A0 + 1600;       // u8  [400] conv2 pool codes                     400
constexpr int L_BIAS = L_C2 + 400;      // f32 [c1 6 | c2 16 | f1 120 | f2 84 | f3 10]    960
constexpr int L_H1 = L_BIAS + 960;      // f32 [128]                                      512
constexpr int L_H2 = L_H1 + 512;        // f32 [96]                                       384
constexpr int L_DZ3 = L_H2 + 384;       // f32 [16]                                        64
constexpr int L_DZ2 = L_DZ3 + 64;       // f32 [96]                                       384
constexpr int L_DZ1 = L_DZ2 + 384;      // f32 [128]                                      512
constexpr int L_DA0 = L_DZ1 + 512;      // f32 [400]                                     1600
constexpr int L_F2 = L_DA0 + 1600;      // f32 fc2 [84][120]                            40320
constexpr int L_F3 = L_F2 + 40320;      // f32 fc3 [10][84]                              3360
constexpr int L_PART = L_F3 + 3360;     // f32 partial sums: conv2 fwd / fc1 dgrad / dW1 25600
constexpr int DY2_LD = 20;              // dY2 rows of 20: 16-B aligned 8-wide windows
constexpr int DY2_CH = 18 * DY2_LD + 4;  //   channels 364 floats apart: the conv2 weight gradient's
                                         //   b32 reads of 16 channels are 2-way, not 4-way
constexpr int L_DY2 = L_PART + 25600;   // f32 [16][DY2_CH] dY2 zero-padded (4 left/top)  23296
// conv weight-gradient tables, built from the pool codes while wave 0 runs fc3 + the loss:
// the ACTIVE windows (ReLU passed) of each channel, compacted in window order, as {dY value,
// pixel offset}; the offsets are known from the forward pass, the values are filled in by the
// data-gradient epilogues.  Inactive windows carry no gradient, so the weight-gradient loops
// walk only the active ones (about half) without a branch.
constexpr int T1_LD = 218;               // <= 196 active windows + 22 zero pad entries (even: 16-B pairs)
constexpr int L_T1 = L_DY2 + 16 * DY2_CH * 4;  // f2 [6][T1_LD] {dP1, offset in XW}        10464
constexpr int L_T2 = L_T1 + 6 * T1_LD * 8;  // f2 [16][25] {dA0, offset in P1}             3200
constexpr int L_PS1 = L_T2 + 3200;       // u8 [6][196] window -> table slot (255: inactive) 1176
constexpr int L_PS2 = L_PS1 + 1176;      // u8 [400]                                         400
constexpr int L_NACT = L_PS2 + 400;      // i32 [6 conv1 | 16 conv2] active-window counts     88
constexpr int LDS_TOTAL = L_NACT + 88;   // 162,448 B
static_assert(L_WT1 % 16 == 0 && L_WT2 % 16 == 0 && L_WD % 16 == 0 && L_F2 % 16 == 0 && L_DY2 % 16 == 0,
              "16-B aligned b128 regions");
static_assert(L_T1 % 16 == 0 && L_T2 % 8 == 0 && L_NACT % 4 == 0, "table alignment");
static_assert(3 * XW_CH * 4 <= 40320, "XW fits the dead fc2 region");
static_assert(LDS_TOTAL <= 163840, "LDS budget");
constexpr int B_C1 = 0, B_C2 = 6, B_F1 = 22, B_F2 = 142, B_F3 = 226;  // bias offsets (floats)
constexpr int W1_PARTS = 11;  // conv1 weight gradient: the active windows in 11 slices
static_assert(16 * 400 * 4 <= 25600 && W1_PARTS * 450 * 4 <= 25600 && 4 * 168 * 4 * 8 <= 25600, "partials");

// ToTensor + Normalize((.5,.5,.5),(.5,.5,.5)) exactly as PyTorch's fp32 ops: u / 255 correctly
// rounded (the double quotient of u / 255 is never within a double ulp of a float rounding
// boundary - its bits repeat u with period 8 - so rounding it to float IS the correctly rounded
// float quotient), then (t - 0.5) rounded, then / 0.5 (exact).
__device__ __forceinline__ float u8norm(uint32_t u) {
  const float t = (float)((double)u / 255.0);
  return (t - 0.5f) * 2.0f;
}

// Barrier for LDS hand-offs only: s_waitcnt lgkmcnt(0) + s_barrier.  __syncthreads() would also
// wait for vmcnt(0) - every outstanding global load AND store of the wave (gfx9 counts stores in
// vmcnt) - so a row store or the in-flight fc1 stream would stall every barrier behind it.  The
// compiler still waits for each global load before the first use of its register.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// v if keep, else +0 - as a bit mask, so the compiler cannot turn the (always safe) LDS load
// into a branch per element (a select makes it load only under the condition: one LDS round
// trip per element)
__device__ __forceinline__ float masked(float v, bool keep) {
  return __uint_as_float(__float_as_uint(v) & (keep ? 0xffffffffu : 0u));
}

// ---- the persistent launch (PERS) ------------------------------------------------------------
// The bf16 kernel's persistent launch (lenet_fused.hip PERS: one launch runs pc.nsteps steps,
// reduction and sample workgroups hand off through generation-relative arrival / ready tags),
// for the fp32 kernel's 1024-thread workgroups.  A conv reduction block (or the bookkeeping) gets
// a workgroup of its own (the other three quarters idle): four 256-thread blocks on one CU
// finished their slab reductions ~0.6 us apart each - their 16-deep dword load chains queue at
// the CU's texture path - so the last block of a 4-block workgroup set the conv hand-off ~1.8 us
// after the first (profiles/r5/fp32_pers).  The MLP blocks, off the critical path, run four per
// workgroup.  Map: workgroup wg < PF_CONV_WG: conv block wg (45 = the bookkeeping); then MLP
// blocks 4 (wg - PF_CONV_WG) + quarter.  Samples wait for every workgroup's ready word before a
// step (the conv1 group finishes last anyway - the hand-off runs conv1 -> conv1) and load the
// weights with sc1 loads of the fp32 master, which the reduction stores write-through
// (WtF32Sink).
constexpr int PF_CONV_WG = PIPE_CONV_BLOCKS + 1;                // conv + bookkeeping workgroups
constexpr int PF_WG = PF_CONV_WG + (PIPE_MLP_BLOCKS + 3) / 4;  // reduction workgroups
static_assert(PF_WG <= PERS_RROW, "one ready word per reduction workgroup in a sample's row");

__device__ __forceinline__ void pf_arrive(const PipeCtl& pc, int kind, int b, unsigned tag, int lane) {
  const int w0 = kind ? PF_CONV_WG : 0, nw = kind ? PF_WG - PF_CONV_WG : PF_CONV_WG;
  if (lane < nw) st_tag(pc.arrive + (long)(w0 + lane) * PERS_AROW + b, tag);
}

// one wave waits until every reduction workgroup's word of this sample's ready row reached tgt
// (bounded like pers_wait_rows: the sticky error word, never a hang)
__device__ __forceinline__ void pf_wait_ready(const PipeCtl& pc, int b, unsigned tgt, int lane) {
  if (ld_tag(pc.err) != 0u) return;
  const unsigned* row = pc.flg + (long)b * PERS_RROW + min(lane, PF_WG - 1);
  const long long t0 = wall_clock64();
  while (true) {
    if (__all(tag_ge(ld_tag(row), tgt))) break;
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > pc.timeout_ticks) {
      if (lane == 0) __hip_atomic_store(pc.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// Reduction workgroup wg: its four blocks, every step in order - wait for the rows (conv
// workgroups: the conv arrival, which every sample stores after its MLP rows too), reduce + SGD
// (write-through master), then this workgroup's word in every sample's ready row.
// stamps (diagnostic, tools/phase_trace_f32.py --pers): the last step's rows seen / body done /
// ready stored of workgroup wg at stamps[6144 + 4 wg + k]
// XNR > 1 (the per-step all-reduce inside the fp32 persistent launch, up to XNR ranks): each
// block reduces its elements as above, then exchanges them exactly as the serial one-launch
// exchange does (reduce_device.h xp_exchange / xp_exchange_rsag with the F32 sink: the same
// granule protocol, block -> counter map gb = rblk, two-hop owner map and rank-order sum, so the
// parameters are bit-identical to it) and stores the new parameters write-through to the fp32
// master before the workgroup signals ready.  Idle quarters take no counter; the launch advances
// every block's counter by nsteps at its end (lenet_fused.hip pers_reduce's rule).
template <int XNR>
__device__ __forceinline__ void pers_reduce_f32(const ReduceArgs& a, const PipeCtl& pc, int wg, long long* stamps) {
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8), rtid = threadIdx.x & 255, lane = threadIdx.x & 63;
  const bool bk = wg == PIPE_CONV_BLOCKS && q == 0;
  int rblk = -1;  // (-1: idle)
  if (wg < PIPE_CONV_BLOCKS) {
    if (q == 0) rblk = PIPE_MLP_BLOCKS + wg;
  } else if (wg >= PF_CONV_WG) {
    const int mm = 4 * (wg - PF_CONV_WG) + q;
    if (mm < PIPE_MLP_BLOCKS) rblk = mm;
  }
  const unsigned g0 = __builtin_amdgcn_readfirstlane(ld_tag(pc.gen + blockIdx.x));
  // (XNR) this quarter's exchange counter: the grad_reduce block index (bookkeeping: the last one)
  const int gb = bk ? PIPE_MLP_BLOCKS + PIPE_CONV_BLOCKS : rblk;
  const unsigned xc0 = XNR > 1 && gb >= 0 ? __builtin_amdgcn_readfirstlane(a.xp_ctr[gb]) : 0u;
  if (bk && rtid < 64) bookkeeping_pers(a, pc, lane, -1);
  const unsigned* arr = pc.arrive + (long)wg * PERS_AROW;
  for (int t = 0; t < pc.nsteps; ++t) {
    int tid_o = threadIdx.x;  // (opaque: the lane's address math stays inside the step)
    asm volatile("" : "+v"(tid_o));
    const int lane_o = tid_o & 63;
    if (tid_o < 64) pers_wait_rows(pc, arr, a.batch, g0 + (unsigned)t + 1u, lane_o);
    const bool st = stamps != nullptr && threadIdx.x == 0 && t == pc.nsteps - 1;
    if (st) stamps[6144 + 4 * wg] = (long long)__builtin_amdgcn_s_memrealtime();
    __syncthreads();
    WtF32Sink sk;
    if (bk) {
      if (rtid < 64) bookkeeping_pers(a, pc, lane_o, t);
    } else if (rblk >= 0) {
      if constexpr (XNR > 1) {
        const unsigned step = xc0 + (unsigned)t + 1u;
        const bool failed = __hip_atomic_load(a.xp_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
        XpSinkT<false, true, true> xs;
        xs.tag = (unsigned long long)step << 32;
        xs.stash = tid_o;  // (8 x NT floats of the reduction workgroup's otherwise unused LDS)
        xs.stride = NT;
        const bool publish = (a.xp_mode & 2) == 0 || gb % a.xp_nranks != a.xp_rank;
        xs.own = publish ? reinterpret_cast<unsigned long long*>(a.xp_region[a.xp_rank] + a.xp_gslot_off +
                                                                 (step & 1u) * a.xp_gslot_bytes)
                         : nullptr;
        if (grad_reduce_body<XpSinkT<false, true, true>, true>(a, xs, rblk, tid_o & 255, t & 1)) {
          if ((a.xp_mode & 2) == 0) xp_exchange<XNR>(a, xs, step, failed, rblk, tid_o & 255);
          else xp_exchange_rsag<XNR>(a, xs, step, failed, rblk, tid_o & 255);
        }
      } else {
        grad_reduce_body<WtF32Sink, true>(a, sk, rblk, tid_o & 255, t & 1);
      }
    }
    if (st) stamps[6145 + 4 * wg] = (long long)__builtin_amdgcn_s_memrealtime();
    // (diagnostic: the last step's per-wave body done / drained, stamps[6400 + 32 wg + 2 wave + k])
    const bool wst = stamps != nullptr && (threadIdx.x & 63) == 0 && t == pc.nsteps - 1;
    if (wst) stamps[6400 + 32 * wg + 2 * (threadIdx.x >> 6)] = (long long)__builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
    if (wst) stamps[6401 + 32 * wg + 2 * (threadIdx.x >> 6)] = (long long)__builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (st) stamps[6146 + 4 * wg] = (long long)__builtin_amdgcn_s_memrealtime();
    if (tid_o < 64)
      for (int b = lane_o; b < a.batch; b += 64) st_tag(pc.flg + (long)b * PERS_RROW + wg, g0 + (unsigned)t + 1u);
    sk.flush(a);  // momentum + bf16 shadow: off the hand-off's critical path (drained by the next step's wait)
  }
  if (threadIdx.x == 0) st_tag(pc.gen + blockIdx.x, g0 + (unsigned)pc.nsteps);
  if constexpr (XNR > 1) {
    if (gb >= 0 && rtid == 0) a.xp_ctr[gb] = xc0 + (unsigned)pc.nsteps;  // (the next launch reads it)
  }
}

// Parameter loads: plain, or (WT: the persistent launch) sc1 loads of the write-through master
template <bool WT>
struct MasterRd {
  const float* ms;
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit MasterRd(const float* master) : ms(master) {
    if constexpr (WT) r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(master), 0, ARENA * 4, 0x00020000);
  }
  __device__ __forceinline__ float f(int i) const {
    if constexpr (WT)
      return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(ms + i), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT));
    else return ms[i];
  }
  __device__ __forceinline__ f4 v4(int i) const {  // 4 floats at element i (16-B aligned)
    if constexpr (WT) return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, i * 4, 0, 16));
    else return *reinterpret_cast<const f4*>(ms + i);
  }
};

// The kernel's arguments (one block for both launch forms)
struct F32Args {
  const uint8_t* images;
  const int32_t* labels;
  const int32_t* order;  // TRAIN: this step's sample ids [batch] (PERS: the first step's)
  int order_len, batch, base_index;
  const int32_t* state;
  const float* master;   // fp32 parameter arena
  float *a0, *h1, *h2, *z1, *z2, *z3, *slab, *loss;  // per-sample rows (PERS: parity 0; parity 1 follows)
  int32_t* correct;
  long long* stamps;     // diagnostic: block 0's phase timeline (s_memrealtime, 100 MHz)
};

// ONE sample's step (workgroup = sample b).  PERS: step s of the persistent launch - sample is
// this step's id (-1: none), ns_next receives the next step's (read before the conv arrival).
template <bool TRAIN, bool PERS>
__device__ __forceinline__ void f32_step(const F32Args& A, const PipeCtl& pc, int b, int sample, int s, unsigned g0,
                                         int& ns_next) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // (PERS: the lane's indices come from an opaque copy of threadIdx.x in every step, so their
  // address math is not hoisted out of the step loop and kept live across it)
  int tid_o = threadIdx.x;
  if constexpr (PERS) asm volatile("" : "+v"(tid_o));
  const int tid = tid_o, lane = tid & 63, wave = tid >> 6;
  const int batch = A.batch;
  const uint8_t* const images = A.images;
  const int32_t* const labels = A.labels;
  // (PERS: the phase stamps of the last step; per-step stamps of sample 0 at [2048 + k * 1024 + s]:
  // k = 0 step start, 1 ready wait passed, 2 MLP arrival stored, 3 conv arrival stored)
  long long* const stamps = PERS ? (s == pc.nsteps - 1 ? A.stamps : nullptr) : A.stamps;
  const bool pstamp = PERS && A.stamps != nullptr && b == 0 && s < 1024;
  auto pst = [&](int k, bool who) {
    if (pstamp && who) A.stamps[2048 + 1024 * k + s] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  pst(0, tid == 0);
  const MasterRd<PERS> mr(A.master);
  // PERS: this step's rows are parity s & 1
  const long rsh = PERS ? (long)(s & 1) * batch : 0;
  float* const a0_out = A.a0 + rsh * A0_LD;
  float* const h1_out = A.h1 + rsh * H1_LD;
  float* const h2_out = A.h2 + rsh * H2_LD;
  float* const z1_out = A.z1 + rsh * Z1_LD;
  float* const z2_out = A.z2 + rsh * Z2_LD;
  float* const z3_out = A.z3 + rsh * Z3_LD;
  float* const slab_out = A.slab + rsh * SLAB;
  float* const loss_out = A.loss + rsh;
  int32_t* const correct_out = A.correct + rsh;
  // a row element: plain, or (PERS) written through - the reduction of the same launch reads it
  auto put_row = [&](float* p, float v) {
    if constexpr (PERS) st_wt(p, v);
    else *p = v;
  };
  // PERS: every wave drained its stores -> barrier -> one wave stores the arrival tags of this
  // sample for the conv workgroups (kind 0; first the next step's sample id, read before the
  // bookkeeping of this step can overwrite its slot) or the MLP workgroups (kind 1)
  auto arrive = [&](int kind) {
    if (kind == 0) {
      ns_next = __builtin_amdgcn_readfirstlane(ld_sc1(pc.nid_slot[s & 1] + b));
      // fault injection (flags & 256, tests only): sample 0 arrives for the conv workgroups of
      // step 1 three wait timeouts late (lenet_fused.hip's)
      if ((pc.flags & 256) && b == 0 && s == 1 && tid == 0) {
        const long long t0 = wall_clock64();
        while (wall_clock64() - t0 < 3 * pc.timeout_ticks) __builtin_amdgcn_s_sleep(64);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave == 0) pf_arrive(pc, kind, b, g0 + (unsigned)s + 1u, lane);
    if (kind == 0) pst(3, tid == 0);
  };
  const bool stamp = stamps != nullptr && b == 0 && tid == 0;
#define STAMP(i) do { if (stamp) stamps[i] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
  // (diagnostic: when lane t of block 0 finished its part of a concurrent phase)
#define LANE_STAMP(i, t)                                                                   \
  do {                                                                                     \
    if (stamps != nullptr && b == 0 && tid == (t)) {                                       \
      __builtin_amdgcn_s_waitcnt(0);                                                       \
      stamps[i] = (long long)__builtin_amdgcn_s_memrealtime();                             \
    }                                                                                      \
  } while (0)
  // (diagnostic: when each wave of block 0 reached a barrier, stamps[base + wave])
#define WAVE_STAMP(base)                                                                      \
  do {                                                                                     \
    if (stamps != nullptr && b == 0 && lane == 0) stamps[(base) + wave] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
  STAMP(0);
  float* X = reinterpret_cast<float*>(smem + L_X);
  // the image ingest: 16 pixels of row (c, y) = tid / 2, columns 16 (tid & 1) .. (tid < 192)
  auto ingest = [&](int id) {
    if (tid < 192) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (!PERS || id >= 0) v = reinterpret_cast<const uint4*>(images + (size_t)id * IMG)[tid];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const int row = tid >> 1, c = row >> 5, y = row & 31;
      float* dst = X + c * X_CH + y * X_RS + 16 * (tid & 1);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        reinterpret_cast<f2*>(dst)[k] = f2{u8norm((w[k >> 1] >> (16 * (k & 1))) & 0xffu),
                                           u8norm((w[k >> 1] >> (16 * (k & 1) + 8)) & 0xffu)};
    }
  };
  int bvalid = 1;
  bool valid;
  if constexpr (PERS) {
    // the image first (its sample id was published two steps ahead: no wait needed) - it lands
    // in LDS while wave 0 waits for the previous step's reduction (from step 1 on); then this
    // step's valid count from its bookkeeping slot (published with the ready words)
    ingest(sample);
    if (s > 0 && wave == 0) pf_wait_ready(pc, b, g0 + (unsigned)s, lane);
    lds_barrier();
    pst(1, tid == 0);
    bvalid = __builtin_amdgcn_readfirstlane(ld_sc1(pc.bv_slot[s & 1]));
    valid = b < bvalid;
  } else if (TRAIN) {
    bvalid = A.state[ST_BVALID];
    valid = b < bvalid;
  } else {
    valid = (long)A.base_index + b < A.order_len;
  }
  if (!valid) {  // tail of the last batch: zero rows, the reduction adds nothing
    if (TRAIN) {
      for (int i = tid; i < A0_LD; i += NT) put_row(a0_out + (size_t)b * A0_LD + i, 0.f);
      if (tid < H1_LD) { put_row(h1_out + (size_t)b * H1_LD + tid, 0.f); put_row(z1_out + (size_t)b * Z1_LD + tid, 0.f); }
      if (tid < H2_LD) { put_row(h2_out + (size_t)b * H2_LD + tid, 0.f); put_row(z2_out + (size_t)b * Z2_LD + tid, 0.f); }
      if (tid < Z3_LD) put_row(z3_out + (size_t)b * Z3_LD + tid, 0.f);
      for (int i = tid; i < SLAB; i += NT) put_row(slab_out + (size_t)b * SLAB + i, 0.f);
      if (tid == 0) { put_row(loss_out + b, 0.f); put_row(reinterpret_cast<float*>(correct_out + b), 0.f); }
    }
    if constexpr (PERS) {
      arrive(1);
      arrive(0);
    }
    return;
  }
  float* WT1 = reinterpret_cast<float*>(smem + L_WT1);
  float* WT2 = reinterpret_cast<float*>(smem + L_WT2);
  float* WD = reinterpret_cast<float*>(smem + L_WD);
  float* P1 = reinterpret_cast<float*>(smem + L_P1);
  uint8_t* C1 = smem + L_C1;
  float* A0 = reinterpret_cast<float*>(smem + L_A0);
  uint8_t* C2 = smem + L_C2;
  float* BIAS = reinterpret_cast<float*>(smem + L_BIAS);
  float* H1 = reinterpret_cast<float*>(smem + L_H1);
  float* H2 = reinterpret_cast<float*>(smem + L_H2);
  float* DZ3 = reinterpret_cast<float*>(smem + L_DZ3);
  float* DZ2 = reinterpret_cast<float*>(smem + L_DZ2);
  float* DZ1 = reinterpret_cast<float*>(smem + L_DZ1);
  float* DA0 = reinterpret_cast<float*>(smem + L_DA0);
  float* F2 = reinterpret_cast<float*>(smem + L_F2);
  float* F3 = reinterpret_cast<float*>(smem + L_F3);
  float* PART = reinterpret_cast<float*>(smem + L_PART);
  float* DY2 = reinterpret_cast<float*>(smem + L_DY2);
  f2* T1 = reinterpret_cast<f2*>(smem + L_T1);
  f2* T2 = reinterpret_cast<f2*>(smem + L_T2);
  uint8_t* PS1 = smem + L_PS1;
  uint8_t* PS2 = smem + L_PS2;
  int* NACT = reinterpret_cast<int*>(smem + L_NACT);

  // ============ phase A: ingest + weight staging ========================================
  {
    if constexpr (!PERS) ingest(sample);  // (PERS: above, before the wait)
    for (int i = tid; i < 450; i += NT) {
      const int o = i / 75, k = i - 75 * o, c = k / 25;
      const int t = k - 25 * c, ky = t / 5;
      WT1[((o >> 1) * 3 + c) * WP_C + ky * WP_R + 2 * (t - 5 * ky) + (o & 1)] = mr.f(OFF_C1W + i);
    }
    if (tid < 236) {
      int src;
      if (tid < B_C2) src = OFF_C1B + tid;
      else if (tid < B_F1) src = OFF_C2B + tid - B_C2;
      else if (tid < B_F2) src = OFF_F1B + tid - B_F1;
      else if (tid < B_F3) src = OFF_F2B + tid - B_F2;
      else src = OFF_F3B + tid - B_F3;
      BIAS[tid] = mr.f(src);
    }
  }
  // the weights conv1 does not need are loaded into registers now and stored to LDS after the
  // conv1 products: their global-load latency hides under conv1 instead of phase A's barrier
  f4 lf2[3], lf3;
  float lw2[3];
  {
#pragma unroll
    for (int k = 0; k < 3; ++k) lf2[k] = mr.v4(OFF_F2W + 4 * min(tid + NT * k, 2519));
    lf3 = mr.v4(OFF_F3W + 4 * min(tid, 209));
#pragma unroll
    for (int k = 0; k < 3; ++k) lw2[k] = mr.f(OFF_C2W + min(tid + NT * k, 2399));
  }
  lds_barrier();
  STAMP(1);

  // ============ phase B: conv1 (3->6, 5x5) + bias + ReLU + 2x2 maxpool ==================
  // task = (channel pair p, pool window q): 4 pixels x 2 channels of packed accumulators
  if (tid < 588) {
    const int p = tid / 196, q = tid - 196 * p, qy = q / 14, qx = q - 14 * qy;
    f2 acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float xs[6][6];
      const float* xr = X + c * X_CH + (2 * qy) * X_RS + 2 * qx;
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const f2 t = *reinterpret_cast<const f2*>(xr + r * X_RS + 2 * j);
          xs[r][2 * j] = t.x;
          xs[r][2 * j + 1] = t.y;
        }
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        f2 wv[6];
        const f4* wr = reinterpret_cast<const f4*>(WT1 + (p * 3 + c) * WP_C + ky * WP_R);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const f4 t = wr[j];
          wv[2 * j] = f2{t.x, t.y};
          wv[2 * j + 1] = f2{t.z, t.w};
        }
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) {
          const f2 w = wv[kx];
          acc[0] += w * xs[ky][kx];
          acc[1] += w * xs[ky][kx + 1];
          acc[2] += w * xs[ky + 1][kx];
          acc[3] += w * xs[ky + 1][kx + 1];
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = 2 * p + h;
      const float bias = BIAS[B_C1 + o];
      float best = acc[0][h] + bias;
      int arg = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        const float v = acc[i][h] + bias;
        if (v > best) { best = v; arg = i; }
      }
      P1[o * P1_CH + qy * 14 + qx] = fmaxf(best, 0.f);
      C1[o * 196 + q] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int i = tid + NT * k;
    if (i < 2400) {
      const int o = i / 150, kk = i - 150 * o, c = kk / 25;
      const int t = kk - 25 * c, ky = t / 5;
      WT2[((o >> 1) * 6 + c) * WP_C + ky * WP_R + 2 * (t - 5 * ky) + (o & 1)] = lw2[k];
      WD[(c * 16 + o) * WD_LD + WD_CPAD * c + kk - 25 * c] = lw2[k];
    }
  }
  if (tid < 210) reinterpret_cast<f4*>(F3)[tid] = lf3;
  if constexpr (PERS) {  // (PERS: the fc2 weights go in now - their 12 registers would spill under conv2)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (tid + NT * k < 2520) reinterpret_cast<f4*>(F2)[tid + NT * k] = lf2[k];
  }
  lds_barrier();
  STAMP(2);

  // ============ phase C: conv2 (6->16, 5x5) + bias + ReLU + 2x2 maxpool =================
  // task = (input-channel half hh, channel pair pp, pool window w); the second half's partial
  // sums meet the first half's through LDS (fixed order: c 0-2, then + c 3-5)
  // fc1 rows of this wave (o = wave + 16 j): streamed from L2 ONCE, kept in registers through
  // the loss for the data gradient.  Issued now: the loads fly under conv2.
  // (the first 64 columns of the rows now, the remaining 36 after the conv2 products: register
  // budget)
  f4 r0[8], r1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r0[j] = mr.v4(OFF_F1W + 4 * (min(wave + 16 * j, 119) * 100 + lane));
  f2 cacc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
  // task c_r = (window c_w, channel pair c_pp), pair-minor: a 32-lane read group covers 4
  // windows x 8 pairs, so its 8-B image reads are 4 broadcast addresses and its 16-B weight reads
  // 8 distinct slots (bank model: 756 LDS cycles per sample, the window-minor order took 1458)
  const int c_hh = tid / 200, c_r = tid - 200 * c_hh, c_w = c_r >> 3, c_pp = c_r & 7;
  if (tid < 400) {
    const int wy = c_w / 5, wx = c_w - 5 * wy;
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) {
      const int c = 3 * c_hh + cc;
      float xs[6][6];
      const float* xr = P1 + c * P1_CH + (2 * wy) * 14 + 2 * wx;
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const f2 t = *reinterpret_cast<const f2*>(xr + r * 14 + 2 * j);
          xs[r][2 * j] = t.x;
          xs[r][2 * j + 1] = t.y;
        }
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        f2 wv[6];
        const f4* wr = reinterpret_cast<const f4*>(WT2 + (c_pp * 6 + c) * WP_C + ky * WP_R);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const f4 t = wr[j];
          wv[2 * j] = f2{t.x, t.y};
          wv[2 * j + 1] = f2{t.z, t.w};
        }
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) {
          const f2 w = wv[kx];
          cacc[0] += w * xs[ky][kx];
          cacc[1] += w * xs[ky][kx + 1];
          cacc[2] += w * xs[ky + 1][kx];
          cacc[3] += w * xs[ky + 1][kx + 1];
        }
      }
    }
    if (c_hh == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) reinterpret_cast<f2*>(PART)[c_r * 4 + i] = cacc[i];
    }
  }
  // the remaining 36 columns of the fc1 rows: issued as soon as the conv2 products are done
  // (their patch and weight registers are dead; waves 7-15 have no conv2 work and issue them
  // at once), so they land under the epilogue instead of at the start of phase D
#pragma unroll
  for (int j = 0; j < 8; ++j) r1[j] = mr.v4(OFF_F1W + 4 * (min(wave + 16 * j, 119) * 100 + 64 + min(lane, 35)));
  lds_barrier();
  STAMP(3);
  if (tid < 200) {
#pragma unroll
    for (int i = 0; i < 4; ++i) cacc[i] += reinterpret_cast<const f2*>(PART)[c_r * 4 + i];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = 2 * c_pp + h;
      const float bias = BIAS[B_C2 + o];
      float best = cacc[0][h] + bias;
      int arg = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        const float v = cacc[i][h] + bias;
        if (v > best) { best = v; arg = i; }
      }
      A0[o * 25 + c_w] = fmaxf(best, 0.f);  // torch.flatten order [16][5][5]
      C2[o * 25 + c_w] = best > 0.f ? (uint8_t)arg : (uint8_t)4;
    }
  }
  lds_barrier();
  STAMP(4);

  // ============ phase D: MLP forward + CrossEntropy =======================================
  {
    const f4 a0v = reinterpret_cast<const f4*>(A0)[lane];
    const f4 a1v = lane < 36 ? reinterpret_cast<const f4*>(A0)[64 + lane] : f4{0.f, 0.f, 0.f, 0.f};
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = r0[j].x * a0v.x;
      s = __builtin_fmaf(r0[j].y, a0v.y, s);
      s = __builtin_fmaf(r0[j].z, a0v.z, s);
      s = __builtin_fmaf(r0[j].w, a0v.w, s);
      s = __builtin_fmaf(r1[j].x, a1v.x, s);
      s = __builtin_fmaf(r1[j].y, a1v.y, s);
      s = __builtin_fmaf(r1[j].z, a1v.z, s);
      v[j] = __builtin_fmaf(r1[j].w, a1v.w, s);
    }
    // the wave's 8 row sums as a reduce-scatter: the xor 32 / 16 / 8 exchanges halve the rows
    // each lane carries (7 ds_bpermute, 3 deep - 8 separate wave sums were 48, 6 deep each),
    // then DPP finishes inside groups of 8 lanes; lane group (lane >> 3) holds row
    // j = 4 h5 + 2 h4 + h3 (a fixed summation tree: deterministic)
    const bool h5 = (lane & 32) != 0, h4 = (lane & 16) != 0, h3 = (lane & 8) != 0;
    float u[4], w2[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = (h5 ? v[k + 4] : v[k]) + __shfl_xor(h5 ? v[k] : v[k + 4], 32);
#pragma unroll
    for (int k = 0; k < 2; ++k) w2[k] = (h4 ? u[k + 2] : u[k]) + __shfl_xor(h4 ? u[k] : u[k + 2], 16);
    const float t = sum8((h3 ? w2[1] : w2[0]) + __shfl_xor(h3 ? w2[0] : w2[1], 8));
    const int o = wave + 16 * ((h5 ? 4 : 0) + (h4 ? 2 : 0) + (h3 ? 1 : 0));
    if ((lane & 7) == 0 && o < 120) H1[o] = fmaxf(t + BIAS[B_F1 + o], 0.f);
  }
  // fc1 waits on L2 and leaves the LDS idle: the fc2 weights (in registers since phase A)
  // and the zero padding of dY2 go in now
  if constexpr (!PERS) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (tid + NT * k < 2520) reinterpret_cast<f4*>(F2)[tid + NT * k] = lf2[k];
  }
  if (TRAIN)
    for (int i = tid; i < 16 * DY2_CH; i += NT) DY2[i] = 0.f;  // dY2 padding (phase E fills the argmaxes)
  lds_barrier();
  STAMP(5);
  if (tid < 672) {  // fc2: 84 outputs x 8 lanes (15 inputs each)
    const int o = tid >> 3, s = tid & 7;
    const float* row = F2 + o * 120 + 15 * s;
    const float* h = H1 + 15 * s;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 15; ++i) acc = __builtin_fmaf(row[i], h[i], acc);
    acc = sum8(acc);
    if (s == 0) H2[o] = fmaxf(acc + BIAS[B_F2 + o], 0.f);
  }
  lds_barrier();
  STAMP(6);
  int label = 0;
  if (wave == 0) {  // fc3 (10 x 84: 4 lanes per logit) + CrossEntropy + accuracy
    label = labels[sample];
    const int o = min(lane >> 2, 9), s = lane & 3;
    const float* row = F3 + o * 84 + 21 * s;
    const float* h = H2 + 21 * s;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 21; ++i) acc = __builtin_fmaf(row[i], h[i], acc);
    acc = sum4(acc);
    const float logit = __shfl(acc, 4 * min(lane, 9)) + BIAS[B_F3 + min(lane, 9)];
    const bool act = lane < 10;
    const float lg = act ? logit : -INFINITY;
    const float mx = max16(lg);
    const float e = act ? expf(lg - mx) : 0.f;
    const float sum = sum16(e);
    const int pred = min16((act && lg == mx) ? lane : 64);  // first max wins (torch.argmax)
    const float lse = mx + logf(sum);
    const float ll = __shfl(lg, label & 15, 16);
    if (lane == 0) {
      put_row(loss_out + b, lse - ll);
      put_row(reinterpret_cast<float*>(correct_out + b), __int_as_float(pred == label ? 1 : 0));
    }
    if (TRAIN && lane < 16) DZ3[lane] = act ? (e / sum - (lane == label ? 1.f : 0.f)) / (float)bvalid : 0.f;
  } else if (TRAIN && wave <= 6) {
    // meanwhile: the conv1 weight-gradient table of channel c - its active windows compacted in
    // window order (ballot prefix counts), each with the offset of its argmax pixel in XW
    const int c = wave - 1;
    int base = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = 64 * k + lane;
      const int code = q < 196 ? C1[c * 196 + q] : 4;
      const unsigned long long m = __ballot(code < 4);
      if (q < 196) {
        const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
        PS1[c * 196 + q] = code < 4 ? (uint8_t)pos : (uint8_t)255;
        if (code < 4) {
          const int qy = q / 14, qx = q - 14 * qy;
          T1[c * T1_LD + pos] = f2{0.f, __int_as_float((2 * qy + (code >> 1)) * XW_RS + 2 * qx + (code & 1))};
        }
      }
      base += __popcll(m);
    }
    float zf = 0.f;  // (PERS: an opaque zero - a hoisted 64-bit zero constant spilled across the step loop)
    if constexpr (PERS) asm volatile("" : "+v"(zf));
    if (lane < 2 * W1_PARTS) T1[c * T1_LD + base + lane] = f2{zf, zf};  // slices round up: zero pad
    if (lane == 0) NACT[c] = base;
  } else if (TRAIN && wave <= 14) {
    // and the conv2 table: channels o = 2 (wave - 7) + (lane >= 32), one per half wave
    const int h = lane >> 5, w = lane & 31, o = 2 * (wave - 7) + h;
    const int code = w < 25 ? C2[o * 25 + w] : 4;
    const unsigned int hm = (unsigned int)(__ballot(code < 4) >> (32 * h));
    if (w < 25) {
      const int pos = __popc(hm & ((1u << w) - 1u));
      PS2[o * 25 + w] = code < 4 ? (uint8_t)pos : (uint8_t)255;
      if (code < 4) {
        const int wy = w / 5, wx = w - 5 * wy;
        T2[o * 25 + pos] = f2{0.f, __int_as_float((2 * wy + (code >> 1)) * 14 + 2 * wx + (code & 1))};
      }
    }
    if (w == 0) NACT[6 + o] = __popc(hm);
  }
  if (!TRAIN) return;
  lds_barrier();
  STAMP(7);

  // ============ phase D': MLP data gradient ==============================================
  if (tid < 84) {  // dh2 = W3^T dz3, ReLU mask
    float d = 0.f;
#pragma unroll
    for (int o = 0; o < 10; ++o) d = __builtin_fmaf(F3[o * 84 + tid], DZ3[o], d);
    DZ2[tid] = H2[tid] > 0.f ? d : 0.f;
  }
  lds_barrier();
  STAMP(8);
  if (tid < 480) {  // dh1 = W2^T dz2 (120 x 84: 4 lanes per input), ReLU mask
    const int i = tid >> 2, s = tid & 3;
    float d = 0.f;
#pragma unroll
    for (int k = 0; k < 21; ++k) d = __builtin_fmaf(F2[(21 * s + k) * 120 + i], DZ2[21 * s + k], d);
    d = sum4(d);
    if (s == 0) DZ1[i] = H1[i] > 0.f ? d : 0.f;
  }
  lds_barrier();
  STAMP(9);
  {  // dA0 = W1^T dz1 from the fc1 rows still in registers: per-wave partials, then a fixed-order
     // sum over the 16 waves
    f4 p0 = {0.f, 0.f, 0.f, 0.f}, p1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = wave + 16 * j;
      const float dz = o < 120 ? DZ1[o] : 0.f;
      p0 += r0[j] * dz;
      p1 += r1[j] * dz;
    }
    reinterpret_cast<f4*>(PART + wave * 400)[lane] = p0;
    if (lane < 36) reinterpret_cast<f4*>(PART + wave * 400)[64 + lane] = p1;
  }
  lds_barrier();
  STAMP(10);
  if (tid < 400) {
    float d = PART[tid];
#pragma unroll
    for (int w = 1; w < 16; ++w) d += PART[w * 400 + tid];
    DA0[tid] = d;
    put_row(a0_out + (size_t)b * A0_LD + tid, A0[tid]);
    // pool2 / ReLU2 backward: dY2 at the argmax pixel (zero-padded copy for the data gradient)
    // and the value of the window's entry in the conv2 weight-gradient table
    const int o = tid / 25, w = tid - 25 * o, wy = w / 5, wx = w - 5 * wy;
    const int code = C2[tid];
    if (code < 4) {
      DY2[o * DY2_CH + (4 + 2 * wy + (code >> 1)) * DY2_LD + 4 + 2 * wx + (code & 1)] = d;
      reinterpret_cast<float*>(T2 + o * 25 + PS2[tid])[0] = d;
    }
  } else if (tid < 520) {
    put_row(h1_out + (size_t)b * H1_LD + tid - 400, H1[tid - 400]);
    put_row(z1_out + (size_t)b * Z1_LD + tid - 400, DZ1[tid - 400]);
  } else if (tid < 604) {
    put_row(h2_out + (size_t)b * H2_LD + tid - 520, H2[tid - 520]);
    put_row(z2_out + (size_t)b * Z2_LD + tid - 520, DZ2[tid - 520]);
  } else if (tid < 620) {
    put_row(z3_out + (size_t)b * Z3_LD + tid - 604, DZ3[tid - 604]);
  }
  // PERS: the MLP rows (and loss / correct) drained before this barrier, then wave 11 (its
  // phase-E work is the shortest) stores the arrival for the MLP workgroups - their reduction
  // overlaps the conv backward
  if constexpr (PERS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  if constexpr (PERS) {
    if (wave == 11) pf_arrive(pc, 1, b, g0 + (unsigned)s + 1u, lane);
    pst(2, tid == 704);
  }
  STAMP(11);

  // ============ phase E: conv2 backward ===================================================
  float* slab = slab_out + (size_t)b * SLAB;
  // conv2 data gradient: full correlation of the padded dY2 with the kernel.  A task owns a
  // 2 x 4 pixel block (yx: row pair yh = yx >> 2, column quad yx & 3) of one input channel c for
  // a quarter q of the output channels: per channel o one 6 x 8 dY2 window (12 aligned 16-B
  // reads) and 25 weights (7 16-B reads, broadcast over the lanes of the same c and o) feed 8
  // outputs; the quarters' partial sums meet through LDS in a fixed order.
  // Task -> lane map from the b128 bank model (tools/lds_banks.py rules): a 16-lane read group
  // of ds_read_b128 covers all 64 banks once only if its windows fall on 16 distinct 4-bank
  // slots, slot = (10 yh + (yx & 3)) mod 16 (+ a group-uniform shift).  The 16 blocks of even yh
  // have distinct slots, the 12 of odd yh too, and lanes of the same yx (other c) read the
  // same address (broadcast).  So each quarter fills 11 groups: 6 groups of one channel's even
  // blocks, then its 72 odd-yh tasks in channel order, 16 per group (44 groups = waves 0..10).
  // The plain tid order put 2 windows on one slot in most groups: 4416 vs 2112 LDS cycles.
  f2 dacc[2][2] = {{{0.f, 0.f}, {0.f, 0.f}}, {{0.f, 0.f}, {0.f, 0.f}}};
  bool d_on;
  int d_q, d_r, d_c, d_y0, d_x0;
  {
    const int l32 = lane & 31;
    const int gi = 4 * wave + 2 * (lane >> 5) + ((0xf00f0ff0u >> l32) & 1);  // read group of the wave
    const int pi = (int)(((l32 < 16 ? 0x7654765432103210ull : 0xfedcfedcba98ba98ull) >> (4 * (l32 & 15))) & 15);
    d_q = gi / 11;
    const int kg = gi - 11 * d_q, t = 16 * (kg - 6) + pi;
    int yx;
    if (kg < 6) {
      d_c = kg;
      yx = 8 * (pi >> 2) + (pi & 3);
    } else {
      d_c = t / 12;
      const int m = t - 12 * d_c;
      yx = 8 * (m >> 2) + 4 + (m & 3);
    }
    d_on = tid < 704 && (kg < 6 || t < 72);
    d_r = 28 * d_c + yx;
    d_y0 = 2 * (yx >> 2);
    d_x0 = 4 * (yx & 3);
  }
  if (d_on) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 4 * d_q + i;
      float D[6][8];
      const f4* dr = reinterpret_cast<const f4*>(DY2 + o * DY2_CH + d_y0 * DY2_LD + d_x0);
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f4 t = dr[r * (DY2_LD / 4) + j];
          D[r][4 * j] = t.x; D[r][4 * j + 1] = t.y; D[r][4 * j + 2] = t.z; D[r][4 * j + 3] = t.w;
        }
      float w[28];
      const f4* wr = reinterpret_cast<const f4*>(WD + (d_c * 16 + o) * WD_LD + WD_CPAD * d_c);
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const f4 t = wr[j];
        w[4 * j] = t.x; w[4 * j + 1] = t.y; w[4 * j + 2] = t.z; w[4 * j + 3] = t.w;
      }
#pragma unroll
      for (int ky = 0; ky < 5; ++ky)
#pragma unroll
        for (int kx = 0; kx < 5; ++kx)
#pragma unroll
          for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp)
              dacc[dy][pp] += w[ky * 5 + kx] * f2{D[dy - ky + 4][2 * pp + 4 - kx], D[dy - ky + 4][2 * pp + 5 - kx]};
    }
    f2* part = reinterpret_cast<f2*>(PART) + (d_q * 168 + d_r) * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) part[k] = dacc[k >> 1][k & 1];
    LANE_STAMP(16, 0);
  }
  // the conv2 weight gradient on the MATRIX cores, waves 11..15, concurrently with the data
  // gradient's VALU work on waves 0..10: dW2[o][n] = sum_k dY2[o][k] * im2col(P1)[k][n] with
  // n = (c, ky, kx) < 150 and k = (y, x) over the DENSE 10 x 10 unpooled dY2 (the zeros outside
  // the argmax pixels add exact zeros) - a 16 x 150 x 100 GEMM whose M = 16 output channels fill
  // the v_mfma_f32_16x16x4_f32 tile exactly.  Each wave owns two 16-column tiles, reads one dY2
  // fragment and two im2col fragments per K-step (no table, no dependent address), and runs two
  // interleaved accumulator chains of 25 MFMAs.  The sparse VALU form (tasks (o, c, ky) walking
  // the active-window table) took 5.5 us of LDS round trips after the data gradient's 2.1 us.
  if (wave >= 11) {
    const int wv = wave - 11, col = lane & 15, q = lane >> 4;
    const float* ab = DY2 + col * DY2_CH + 4 * DY2_LD + 4;  // A: dY2[o = col][k]
    int nb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {  // B: im2col column n = 32 wv + 16 t + col (clamped: n >= 150 unstored)
      const int n = min(32 * wv + 16 * t + col, 149), c = n / 25, r = n - 25 * c, ky = r / 5;
      nb[t] = c * P1_CH + ky * 14 + (r - 5 * ky);
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 25; ++s) {  // k = 4 s + q: (y, x) from the compile-time (4 s) / 10
      const int y0 = (4 * s) / 10, x0 = (4 * s) % 10;
      const int xs = x0 + q, wrap = xs >= 10 ? 1 : 0;
      const int y = y0 + wrap, x = xs - 10 * wrap;
      const float a = ab[y * DY2_LD + x];
      const float b0 = P1[nb[0] + y * 14 + x];
      const float b1 = P1[nb[1] + y * 14 + x];
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b1, acc1, 0, 0, 0);
    }
    // D[i = 4 q + r][j = col]: output channel o = 4 q + r, column n
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = 32 * wv + 16 * t + col;
      if (n < 150) {
#pragma unroll
        for (int r = 0; r < 4; ++r) put_row(slab + SLAB_C2W + (4 * q + r) * 150 + n, t ? acc1[r] : acc0[r]);
      }
    }
  }
  LANE_STAMP(17, 704);
  {
    if (tid >= 960 && tid < 976) {  // conv2 bias gradient (after wave 15's MFMA tiles)
      const int o = tid - 960;
      float sb = 0.f;
      const int n = NACT[6 + o];
#pragma unroll
      for (int w = 0; w < 25; ++w) sb += masked(T2[o * 25 + w].x, w < n);  // fixed trip: reads in flight
      put_row(slab + SLAB_C2B + o, sb);
    }
    if (tid < 704) {  // the re-strided image copy for the conv1 weight gradient: 3072 pixels over 704 lanes
      float* XW = reinterpret_cast<float*>(smem + L_F2);
      float v[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int i = min(tid + 704 * k, 3071), c = i >> 10, y = (i >> 5) & 31, x = i & 31;
        v[k] = X[c * X_CH + y * X_RS + x];
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int i = tid + 704 * k, c = i >> 10, y = (i >> 5) & 31, x = i & 31;
        if (i < 3072) XW[c * XW_CH + y * XW_RS + x] = v[k];
      }
    }
    LANE_STAMP(18, 128);
  }
  WAVE_STAMP(24);
  lds_barrier();
  STAMP(12);
  if (tid < 168) {  // lane = block d_r = 28 c + yx: the quarters' partials in the order 0, 1, 2, 3
    d_r = tid;
    d_c = tid / 28;
    d_y0 = 2 * ((tid - 28 * d_c) >> 2);
    d_x0 = 4 * ((tid - 28 * d_c) & 3);
    float db1 = 0.f;  // this lane's 8 windows' share of the conv1 bias gradient
    {
      const f2* part = reinterpret_cast<const f2*>(PART) + d_r * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) dacc[k >> 1][k & 1] = part[k];
    }
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const f2* part = reinterpret_cast<const f2*>(PART) + (q * 168 + d_r) * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) dacc[k >> 1][k & 1] += part[k];
    }
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int x = d_x0 + 2 * pp;
        if (x < 14) {
          // ReLU1 + pool1 backward: dP1 of an active window is the value of its entry in the
          // conv1 weight-gradient table (and part of the conv1 bias gradient)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int q = (d_y0 + dy) * 14 + x + e;
            const int pos = PS1[d_c * 196 + q];
            const float v = e ? dacc[dy][pp].y : dacc[dy][pp].x;
            if (pos != 255) {
              reinterpret_cast<float*>(T1 + d_c * T1_LD + pos)[0] = v;
              db1 += v;
            }
          }
        }
      }
    DY2[tid] = db1;  // (dY2 is dead after the data gradient) partials in a fixed order: lane d_r = 28 c + yx
  }
  lds_barrier();
  STAMP(13);

  // ============ phase F: conv1 weight + bias gradient =====================================
  static_assert(W1_PARTS * 90 <= 992 && 992 + 6 <= NT, "conv1 weight-gradient tasks + bias lanes fit the block");
  if (tid >= 992 && tid < 992 + 6) {  // conv1 bias gradient: the 28 epilogue partials of channel c
    const int c = tid - 992;
    const f4* pp = reinterpret_cast<const f4*>(DY2 + 28 * c);
    f4 t = pp[0];
#pragma unroll
    for (int i = 1; i < 7; ++i) t += pp[i];
    put_row(slab + SLAB_C1B + c, (t.x + t.y) + (t.z + t.w));
    LANE_STAMP(19, 992);
  }
  const float* XW = reinterpret_cast<const float*>(smem + L_F2);
  if (tid < W1_PARTS * 90) {
    // dW1 over the active argmax pixels (table T1) of channel o, in 11 slices of s windows (the
    // zero pad entries round the last slices up); lanes of one channel share a wave
    const int o = tid / (15 * W1_PARTS), r = tid - 15 * W1_PARTS * o, part = r / 15, ck = r - 15 * part;
    // slices of an even number of windows: the table is read two entries per 16-B read
    const int c = ck / 5, ky = ck - 5 * c, s2 = (NACT[o] + 2 * W1_PARTS - 1) / (2 * W1_PARTS);
    const f4* tb = reinterpret_cast<const f4*>(T1 + o * T1_LD) + s2 * part;
    const float* xb = XW + c * XW_CH + ky * XW_RS;
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
    for (int q = 0; q < s2; ++q) {  // unrolled: six windows' table + pixel reads in flight
      const f4 ee = tb[q];
      const float* xr0 = xb + __float_as_int(ee.y);
      const float* xr1 = xb + __float_as_int(ee.w);
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) acc[kx] = __builtin_fmaf(ee.x, xr0[kx], acc[kx]);
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) acc[kx] = __builtin_fmaf(ee.z, xr1[kx], acc[kx]);
    }
#pragma unroll
    for (int kx = 0; kx < 5; ++kx) PART[part * 450 + o * 75 + c * 25 + ky * 5 + kx] = acc[kx];
    LANE_STAMP(20, 0);
  }
  WAVE_STAMP(40);
  lds_barrier();
  STAMP(14);
  if (tid < 450) {
    float sum = PART[tid];
#pragma unroll
    for (int p = 1; p < W1_PARTS; ++p) sum += PART[p * 450 + tid];
    put_row(slab + SLAB_C1W + tid, sum);
  }
  if (stamp) {
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(15);
  }
  if constexpr (PERS) arrive(0);  // slab drained: the conv workgroups go
#undef STAMP
#undef LANE_STAMP
#undef WAVE_STAMP
}

template <bool TRAIN>
__global__ void __launch_bounds__(NT) lenet_f32_kernel(const F32Args A) {
  const int b = blockIdx.x;
  int sample, unused = 0;
  if constexpr (TRAIN) sample = A.order[b];
  else sample = A.base_index + b;
  f32_step<TRAIN, false>(A, PipeCtl{}, b, sample, 0, 0u, unused);
}

// The persistent launch: PF_WG reduction workgroups, then one workgroup per sample, every one
// looping over pc.nsteps steps (lenet_fused.hip PERS's protocol; the rows alternate parities).
// XNR: the per-step exchange inside the launch for groups of up to XNR ranks (0: none)
template <int XNR>
__global__ void __launch_bounds__(NT) lenet_f32_pers_kernel(const F32Args A, const ReduceArgs ra, const PipeCtl pc) {
  if ((int)blockIdx.x < PF_WG) {
    pers_reduce_f32<XNR>(ra, pc, blockIdx.x, A.stamps);
    return;
  }
  const int b = (int)blockIdx.x - PF_WG;
  const unsigned g0 = __builtin_amdgcn_readfirstlane(ld_tag(pc.gen + blockIdx.x));
  int sample = __builtin_amdgcn_readfirstlane(A.order[b]);  // step 0's (the published batch ids)
  for (int s = 0; s < pc.nsteps; ++s) {
    int next = -1;
    f32_step<true, true>(A, pc, b, sample, s, g0, next);
    sample = next;
  }
  if (threadIdx.x == 0) st_tag(pc.gen + blockIdx.x, g0 + (unsigned)pc.nsteps);
}

}  // namespace f32k

void init_kernels_f32() {
  static bool done = false;
  if (done) return;
  const void* kerns[] = {(const void*)f32k::lenet_f32_kernel<true>, (const void*)f32k::lenet_f32_kernel<false>,
                         (const void*)f32k::lenet_f32_pers_kernel<0>, (const void*)f32k::lenet_f32_pers_kernel<8>};
  for (const void* k : kerns)
    HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, f32k::LDS_TOTAL));
  done = true;
}

void launch_fused_train_f32(const uint8_t* images, const int32_t* labels, const int32_t* order, int order_len,
                            int batch, const int32_t* state, const float* master, float* a0, float* h1, float* h2,
                            float* z1, float* z2, float* z3, float* slab, float* loss, int32_t* correct,
                            hipStream_t stream, long long* stamps) {
  init_kernels_f32();
  const f32k::F32Args A{images, labels, order, order_len, batch, 0, state, master, a0, h1, h2, z1, z2, z3, slab,
                        loss, correct, stamps};
  hipLaunchKernelGGL(f32k::lenet_f32_kernel<true>, dim3(batch), dim3(f32k::NT), f32k::LDS_TOTAL, stream, A);
  HIP_CHECK(hipGetLastError());
}

void launch_fused_eval_f32(const uint8_t* images, const int32_t* labels, int n, int base, int count,
                           const float* master, float* loss, int32_t* correct, hipStream_t stream) {
  init_kernels_f32();
  if (count <= 0) return;
  const f32k::F32Args A{images, labels, nullptr, n, count, base, nullptr, master, nullptr, nullptr, nullptr,
                        nullptr, nullptr, nullptr, nullptr, loss, correct, nullptr};
  hipLaunchKernelGGL(f32k::lenet_f32_kernel<false>, dim3(count), dim3(f32k::NT), f32k::LDS_TOTAL, stream, A);
  HIP_CHECK(hipGetLastError());
}

// The fp32 persistent grid's co-residency (lenet_fused.hip persist_resident_workgroups' rule, for
// this kernel: one 1024-thread workgroup per CU) and the largest batch that keeps PERS_MARGIN_F32
// CUs free next to it.
constexpr int PERS_MARGIN_F32 = 8;
int persist_resident_workgroups_f32() {
  static int resident = -1;
  if (resident < 0) {
    init_kernels_f32();
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(f32k::lenet_f32_pers_kernel<0>), f32k::NT, f32k::LDS_TOTAL));
    int per_cu_x = 0;  // (the exchange instance: its own register count)
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu_x, reinterpret_cast<const void*>(f32k::lenet_f32_pers_kernel<8>), f32k::NT, f32k::LDS_TOTAL));
    resident = std::min(per_cu, per_cu_x) * cus;
  }
  return resident;
}
int persist_wg_f32() { return f32k::PF_WG; }
int persist_conv_wg_f32() { return f32k::PF_CONV_WG; }
int persist_ctl_bytes_f32(int batch) { return (int)(pers_arrive_off(batch) + (long)f32k::PF_WG * PERS_AROW * 4); }
int persist_max_batch_f32() {
  return std::max(0, std::min(persist_resident_workgroups_f32() - f32k::PF_WG - PERS_MARGIN_F32, PERS_AROW));
}

// The persistent kernel's parameter block (the kernarg segment of a direct AQL dispatch: the
// compiler lays kernel parameters out as this struct; aql_prepare checks its size against the
// loaded symbol's kernarg segment)
struct F32PersKernargs {
  f32k::F32Args A;
  ReduceArgs ra;
  PipeCtl pc;
};

int launch_fused_train_persist_f32(const uint8_t* images, const int32_t* labels, int order_len, int batch,
                                   const float* master, float* a0, float* h1, float* h2, float* z1, float* z2,
                                   float* z3, float* slab, float* loss, int32_t* correct, const ReduceArgs& red,
                                   const PipeCtl& pc_in, hipStream_t stream, long long* stamps, bool direct) {
  init_kernels_f32();
  // the shapes the kernel assumes (checked here: a mismatch would fault or hang on the device)
  if (batch < 1 || batch > persist_max_batch_f32() || f32k::PF_WG + batch > PERS_MAX_GRID)
    throw std::runtime_error("fused_train_persist_f32: batch must be 1.." + std::to_string(persist_max_batch_f32()) +
                             " (the whole grid co-resident)");
  if (pc_in.nsteps < 1 || pc_in.nsteps > (1 << 20))
    throw std::runtime_error("fused_train_persist_f32: nsteps out of range");
  if (pc_in.ctr == nullptr || pc_in.err == nullptr || !pc_in.bv_slot[0] || !pc_in.bv_slot[1] || !pc_in.nid_slot[0] ||
      !pc_in.nid_slot[1])
    throw std::runtime_error("fused_train_persist_f32: needs the control block, the error word and both slots");
  if (!red.bookkeeping || red.batch != batch || !red.fuse_sgd || red.lo != 0 || red.hi < ARENA ||
      red.batch_ids == nullptr || red.master != master)
    throw std::runtime_error("fused_train_persist_f32: a whole-arena fused-SGD reduction with bookkeeping");
  // the in-launch exchange: the serial one-launch exchange's arguments (fp32 granules, pull or
  // two-hop, grad_scale 1, counters set) - as lenet_fused.hip launch_fused_train_persist checks
  if (red.xp_nranks != 0 &&
      (red.xp_nranks < 1 || red.xp_nranks > XG_MAX_RANKS || (red.xp_mode & ~2) != 0 || red.grad_scale != 1.f ||
       red.xp_ctr == nullptr || red.xp_err == nullptr || red.xp_abort == nullptr || red.xp_rank < 0 ||
       red.xp_rank >= red.xp_nranks))
    throw std::runtime_error("fused_train_persist_f32: the in-launch exchange takes the whole-arena one-launch "
                             "exchange (fp32 granules, pull or two-hop, grad_scale 1, counters set)");
  if (red.a0 != a0 || red.h1 != h1 || red.h2 != h2 || red.z1 != z1 || red.z2 != z2 || red.z3 != z3 ||
      red.slab != slab || red.loss != loss || red.correct != correct)
    throw std::runtime_error("fused_train_persist_f32: the reduction reads the rows the samples write");
  PipeCtl pc = pc_in;  // control block layout (one uncached allocation of persist_ctl_bytes)
  unsigned char* base = reinterpret_cast<unsigned char*>(pc_in.ctr);
  pc.gen = reinterpret_cast<unsigned*>(base);
  pc.flg = reinterpret_cast<unsigned*>(base + PERS_FLG_OFF);
  pc.arrive = reinterpret_cast<unsigned*>(base + pers_arrive_off(batch));
  const f32k::F32Args A{images, labels, red.batch_ids, order_len, batch, 0, nullptr, master, a0, h1, h2, z1, z2, z3,
                        slab, loss, correct, stamps};
  auto* kern = red.xp_nranks == 0 ? &f32k::lenet_f32_pers_kernel<0> : &f32k::lenet_f32_pers_kernel<8>;
  if (direct) {  // prepare (not launch) the same kernel object for this process's AQL queue
    const F32PersKernargs ka{A, red, pc};
    const double bound_s = 10.0 + 2.0 * (double)pc.timeout_ticks * 1e-8 + 2e-3 * pc.nsteps;
    return aql_prepare(reinterpret_cast<const void*>(kern),
                       red.xp_nranks == 0 ? "lenet_f32_pers_kernelILi0E" : "lenet_f32_pers_kernelILi8E", &ka,
                       sizeof(ka), f32k::PF_WG + batch, f32k::NT, f32k::LDS_TOTAL, bound_s, stream);
  }
  hipLaunchKernelGGL(kern, dim3(f32k::PF_WG + batch), dim3(f32k::NT), f32k::LDS_TOTAL, stream, A, red, pc);
  HIP_CHECK(hipGetLastError());
  return -1;
}

}  // namespace dnn

// Host-side launch API of the gfx950 kernels (used by csrc/bindings.cpp).
#pragma once
#include "common.h"
#include "../comm/xgmi_layout.h"

namespace dnn {

struct ReduceArgs {
  const float* a0; const float* h1; const float* h2;
  const float* z1; const float* z2; const float* z3;
  const float* slab; const float* loss; const int32_t* correct;
  int batch;
  float* master; float* grad; float* mom; bf16* shadow;
  int32_t* state; double* stats;
  const int32_t* order; int order_len; int32_t* batch_ids;  // epoch order -> next step's sample ids
  float lr, momentum, grad_scale;
  int fuse_sgd;   // 1: apply SGD in place (local step); 0: write grads only
  int lo, hi;     // arena element range [lo, hi) handled by this launch (gradient bucket)
  int bookkeeping;  // 1: this launch also advances the cursor / epoch statistics
  long long* stamps = nullptr;  // diagnostic: per-block [start, end] s_memrealtime (grad_reduce)
  int32_t* next_ids = nullptr;  // bookkeeping: also publish the sample ids TWO steps ahead (-1: none),
                                // read by the fused kernel's image staging
  // one-launch xGMI all-reduce (xp_nranks > 0; region layout: comm/xgmi_layout.h): every
  // reduction block stores each reduced element into this rank's granule slot as ONE 8-byte
  // {value, step} word, reads the same element's granule from every peer until its tag shows
  // this step, sums the N values in rank order, scales by xp_scale and applies momentum SGD +
  // the bf16 images itself - the batch reduction and the all-reduce in ONE launch, with no
  // hand-off between blocks of this GPU and no flag (each block exchanges exactly the
  // elements it reduced; the tag travels in the same atomic word as the value).
  unsigned char* xp_region[XG_MAX_RANKS] = {};
  int xp_rank = 0, xp_nranks = 0;
  unsigned* xp_ctr = nullptr;          // [XP_MAX_BLOCKS] per-block step counters (local)
  unsigned* xp_err = nullptr;          // sticky error word (shared with the group's all-reduce kernel)
  const unsigned* xp_abort = nullptr;  // host-mapped abort word (fault watchdog)
  long long xp_timeout_ticks = 0;      // s_memrealtime ticks (100 MHz)
  long long xp_gslot_off = 0, xp_gslot_bytes = 0;
  float xp_scale = 1.f;                // 1 / N
  // xp_mode 0: pull one-shot (above).  xp_mode 2: two-hop pull (reduce-scatter + all-gather):
  // block k's elements are owned by rank k % N; the owner reads the peers' pull slots, sums in
  // rank order and publishes {sum, step} in its own ag slot, which the others read (every rank
  // writes only its own region).  Per-link bytes drop from E to 2 E / N granules.
  // + 4: bf16 granules - a lane's elements travel in pairs as {bf16 | bf16, step} words (half
  // the granules per link; every rank sums the same bf16-rounded values in fp32, rank order).
  int xp_mode = 0;
  long long xp_ag_off = 0;
  // diagnostic / accounting: per-step exchange wait (max over lanes, s_memrealtime ticks) as
  // {step << 32 | ticks} words in a ring of XP_WAIT_RING entries (one plain store per wave)
  unsigned long long* xp_wait = nullptr;
  // Bookkeeping slots (null: the serial layout - bvalid in state[ST_BVALID], ids in next_ids).
  // The pipelined step (lenet_fused.hip, PIPE) publishes one launch ahead into the other of
  // two {bvalid, next_ids} slots: bk_bv_in = bvalid of the step whose statistics this launch
  // adds (read before anything is published), bk_bv_out / next_ids = the slot published,
  // bk_adv = how far the cursor advances (1; 0 re-publishes the current step's slot: the
  // launch that ends a pipelined chunk), bk_stats = 0: publish only (no step was reduced).
  const int32_t* bk_bv_in = nullptr;
  int32_t* bk_bv_out = nullptr;
  int bk_adv = 1, bk_stats = 1;
};

// The pipelined step's per-launch control (lenet_fused.hip, PIPE): launch i of a chunk runs
// the batch reduction + SGD of step i - 1 (its rows in the other parity buffer set) in its
// first workgroups and the samples of step i in the rest; the samples wait for the reduction's
// ready flags (conv1, conv2, MLP groups) before they load the weights it writes.
struct PipeCtl {
  unsigned* ctr = nullptr;        // [2 parities][3 groups] arrival counters, 128 B apart, in uncached memory
  int par = 0;                    // this launch's parity (launch index & 1)
  int wait = 0;                   // 1: a reduction runs in this launch, wait for its flags
  int nred = 0;                   // reduction blocks of this launch (0, 1 = bookkeeping only, all)
  const int32_t* bvalid = nullptr;  // this launch's samples' valid count (its bookkeeping slot)
  unsigned* err = nullptr;          // sticky error word: a ready wait timed out (never a hang)
  unsigned* flg = nullptr;          // ready flags (uncached, [2][3][batch] x 128 B): see pipe_reduce
  long long timeout_ticks = 0;      // bound of one ready wait (s_memrealtime ticks, 100 MHz)
  int flags = 0;                    // & 1: no mid-phase-B fc1 stream (measurement)
  // Persistent launch (lenet_fused.hip PERS; nsteps > 0): ONE launch runs nsteps steps.  The
  // reduction workgroups loop over the steps (each waits for the samples' per-step arrival
  // flags), the sample workgroups loop too (each waits for the previous step's ready flags).
  // Ready / arrival words carry generation-relative step tags (never reset; lenet_fused.hip).
  int nsteps = 0;
  int32_t* bv_slot[2] = {nullptr, nullptr};   // bookkeeping slots {bvalid} (written in-launch)
  int32_t* nid_slot[2] = {nullptr, nullptr};  //   and {next_ids}
  unsigned* arrive = nullptr;                 // [reduction workgroup][PERS_AROW] per-sample arrival tags
  unsigned* gen = nullptr;                    // per-workgroup generation words (steps run so far)
};

void launch_fused_train(const uint8_t* images, const int32_t* labels, const int32_t* order, int order_len,
                        int batch, int32_t* state, const float* master, const bf16* shadow, float* a0,
                        float* h1, float* h2, float* z1, float* z2, float* z3, float* slab, float* loss,
                        int32_t* correct, long long* stamps, const int32_t* next_ids, unsigned char* stage,
                        hipStream_t stream, uint8_t* codes = nullptr);
// The pipelined step's merged launch: [reduction of the previous step (red, plain rows of the
// other parity)] + [samples of this step, writing this parity's rows]; see PipeCtl.
void launch_fused_train_pipe(const uint8_t* images, const int32_t* labels, int order_len, int batch,
                             const float* master, const bf16* shadow, float* a0, float* h1, float* h2, float* z1,
                             float* z2, float* z3, float* slab, float* loss, int32_t* correct, long long* stamps,
                             const int32_t* next_ids, unsigned char* stage, const ReduceArgs& red, const PipeCtl& pc,
                             hipStream_t stream);
// The persistent launch: pc.nsteps steps in one launch (rows: two parities, contiguous - parity
// 1 of each row kind right after parity 0); see PipeCtl.
// direct: do not launch; prepare the launch for this process's AQL queue (runtime/aql_dispatch.h)
// and return its handle for persist_direct_run (-1 otherwise)
int launch_fused_train_persist(const uint8_t* images, const int32_t* labels, int order_len, int batch,
                               const float* master, const bf16* shadow, float* a0, float* h1, float* h2, float* z1,
                               float* z2, float* z3, float* slab, float* loss, int32_t* correct, long long* stamps,
                               unsigned char* stage, const ReduceArgs& red, const PipeCtl& pc, hipStream_t stream,
                               bool direct = false);

int persist_max_batch();   // largest batch whose persistent grid is co-resident on this device
int persist_resident_workgroups();  // workgroups of the persistent kernel resident at once (occupancy x CUs)
int persist_ctl_bytes(int batch);  // control memory of a persistent launch (uncached)
int pipe_reduce_blocks();  // reduction blocks of a full PIPE launch (2 per workgroup)
int pipe_groups();         // ready groups (counters / flags per parity)
void launch_fused_eval(const uint8_t* images, const int32_t* labels, const int32_t* order, int n, int base,
                       int count, const float* master, const bf16* shadow, float* loss, int32_t* correct,
                       hipStream_t stream);


// fp32 fused kernel (lenet_f32.hip): same per-sample rows as launch_fused_train, fp32 weights
// straight from the master arena, no bf16 shadow / image staging
void launch_fused_train_f32(const uint8_t* images, const int32_t* labels, const int32_t* order, int order_len,
                            int batch, const int32_t* state, const float* master, float* a0, float* h1, float* h2,
                            float* z1, float* z2, float* z3, float* slab, float* loss, int32_t* correct,
                            hipStream_t stream, long long* stamps = nullptr);
void launch_fused_eval_f32(const uint8_t* images, const int32_t* labels, int n, int base, int count,
                           const float* master, float* loss, int32_t* correct, hipStream_t stream);
// its persistent launch (lenet_f32.hip PERS): pc.nsteps steps in one launch, the reduction
// (red: whole arena, fused SGD, bookkeeping) in its first persist_wg_f32() workgroups; rows and
// control block as launch_fused_train_persist's; red.batch_ids = step 0's sample ids
int launch_fused_train_persist_f32(const uint8_t* images, const int32_t* labels, int order_len, int batch,
                                    const float* master, float* a0, float* h1, float* h2, float* z1, float* z2,
                                    float* z3, float* slab, float* loss, int32_t* correct, const ReduceArgs& red,
                                    const PipeCtl& pc, hipStream_t stream, long long* stamps = nullptr, bool direct = false);
int persist_max_batch_f32();
int persist_resident_workgroups_f32();
int persist_wg_f32();
int persist_conv_wg_f32();
int persist_ctl_bytes_f32(int batch);

// one-time kernel attribute setup (must run before any hipGraph capture)
void init_kernels();
void init_kernels_f32();
void launch_grad_reduce(const ReduceArgs& args, hipStream_t stream);
int grad_reduce_blocks();  // grid of a whole-arena grad_reduce launch (with bookkeeping)
void launch_epoch_begin(const int32_t* staged, int32_t* order, int n, int32_t* state, int32_t* batch_ids, int batch,
                        const uint8_t* images, const int32_t* labels, int32_t* next_ids, unsigned char* stage,
                        hipStream_t stream);
void launch_sgd_apply(float* master, const float* grad, float* mom, bf16* shadow, int n, float lr, float momentum,
                      float grad_scale, int pack_only, hipStream_t stream);

// ---- generic layer kernels (layers.hip) --------------------------------------------------
void launch_ingest(const uint8_t* images, const int32_t* labels, const int32_t* ids, int batch, int per_img,
                   float* out, int32_t* lab_out, hipStream_t s);
void launch_relu_pool_fwd(const float* x, int BC, int H, int W, float* y, uint8_t* code, hipStream_t s);
void launch_relu_pool_bwd(const float* dy, const uint8_t* code, int BC, int H, int W, float* dx, hipStream_t s);
void launch_relu_fwd(const float* x, long n, float* y, hipStream_t s);
void launch_relu_bwd(const float* dy, const float* y, long n, float* dx, hipStream_t s);
int chan_parts(int B, int L);  // partitions per channel of the two-stage channel reductions
void launch_bn_fwd_train(const float* x, int B, int C, int L, const int32_t* state, const float* gamma,
                         const float* beta, float eps, float m, float* rmean, float* rvar, float* y, float* smean,
                         float* sinvstd, double* part, hipStream_t s);
void launch_bn_fwd_eval(const float* x, int B, int C, int L, const float* gamma, const float* beta, float eps,
                        const float* rmean, const float* rvar, float* y, hipStream_t s);
void launch_bn_bwd(const float* dy, const float* x, int B, int C, int L, const int32_t* state, const float* gamma,
                   const float* smean, const float* sinvstd, float* dx, float* dgamma, float* dbeta, double* part,
                   hipStream_t s);
// BatchNorm2d (training) fused with the activation that follows it: act 0 none, 1 ReLU,
// 2 ReLU + 2x2 max-pool (y is [B][C][H/2][W/2] + the 2-bit argmax code).  The backward
// takes the gradient of the ACTIVATION output (pooled for act 2).
void launch_bn_act_fwd_train(const float* x, int B, int C, int H, int W, const int32_t* state, const float* gamma,
                             const float* beta, float eps, float m, float* rmean, float* rvar, float* y, uint8_t* code,
                             float* smean, float* sinvstd, double* part, int act, hipStream_t s,
                             int ext_parts = 0);
void launch_bn_act_bwd(const float* dy, const float* x, int B, int C, int H, int W, const int32_t* state,
                       const float* gamma, const float* beta, const float* smean, const float* sinvstd,
                       const uint8_t* code, float* dx, float* dgamma, float* dbeta, double* part, int act,
                       hipStream_t s,
                       int ext_parts = 0);
void launch_chan_sum(const float* a, int B, int C, int L, float* out, double* part, hipStream_t s);
void launch_xent(const float* logits, const int32_t* labels, int B, int NC, const int32_t* state, float* loss,
                 int32_t* correct, float* dlogits, hipStream_t s);
void launch_layer_bookkeeping(const ReduceArgs& a, hipStream_t s);
// implicit-GEMM convolution (conv_igemm.hip)
size_t conv_fwd_workspace(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, int flip);
int conv_fwd_fast(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops);
void launch_conv_fwd(const float* x, const float* w, const float* bias, float* y, void* ws, int B, int C, int H, int W,
                     int M, int K, int pad, int bf16_ops, int flip, hipStream_t s);
void conv_wgrad_split(int B, int C, int H, int W, int M, int K, int pad, int* S, int* cps);
void launch_conv_wgrad(const float* x, const float* dy, float* part, float* dw, float* db, int B, int C, int H, int W,
                       int M, int K, int pad, int bf16_ops, hipStream_t s,
                       const uint8_t* pool_code = nullptr);
void launch_flip_weights(const float* w, int O, int C, int K, float* wf, hipStream_t s);
// Weight packing for the LDS-patch path, hoisted out of the convolutions: one launch packs
// the forward (flip = 0) and dgrad (flip = 1) images of every fast-path layer of a step
// (geometry = the launch_conv_fwd call the image is for); launch_conv_fwd_packed then
// skips its per-call pack kernel.
struct ConvPackJob {
  const float* w;
  void* dst;  // conv_fwd_workspace(B, C, H, W, M, K, pad, bf16_ops, flip) bytes
  int B, C, H, W, M, K, pad, bf16_ops, flip;
};
void launch_conv_pack_all(const ConvPackJob* jobs, int n, hipStream_t s);
void launch_conv_fwd_packed(const float* x, const void* wp, const float* bias, float* y, int B, int C, int H, int W,
                            int M, int K, int pad, int bf16_ops, hipStream_t s);
// conv + bias + ReLU + 2x2 max-pool in one launch (pooled y, argmax codes as relu_pool_fwd)
int conv_fwd_pool_ok(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops);
void launch_conv_fwd_packed_pool(const float* x, const void* wp, const float* bias, float* y, uint8_t* code, int B,
                                 int C, int H, int W, int M, int K, int pad, int bf16_ops, hipStream_t s);
// conv + bias with the following BatchNorm's batch-statistics partials in the epilogue
int conv_fwd_ingest_ok(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, int epi);
void launch_conv_fwd_packed_ingest(const uint8_t* images, const int32_t* ids, const int32_t* labels, float* x_out,
                                   int32_t* lab_out, const void* wp, const float* bias, float* y, uint8_t* code,
                                   double* stats, const int32_t* state, int B, int C, int H, int W, int M, int K,
                                   int pad, int bf16_ops, hipStream_t s);
int conv_fwd_unpool_ok(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops);
void launch_conv_fwd_packed_unpool(const float* x, const uint8_t* code, const void* wp, float* y, int B, int C, int H,
                                   int W, int M, int K, int pad, int bf16_ops, hipStream_t s);
int conv_fwd_stat_parts(int B, int C, int H, int W, int M, int K, int pad, int bf16_ops);
void launch_conv_fwd_packed_bnbwd(const float* x, const void* wp, float* y, double* stats, const int32_t* state,
                                  const float* bn_z, const float* bn_mean, const float* bn_invstd,
                                  const float* bn_gamma, const float* bn_beta, const uint8_t* bn_code, int zH, int zW,
                                  int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, hipStream_t s);
void launch_conv_fwd_packed_stats(const float* x, const void* wp, const float* bias, float* y, double* stats,
                                  const int32_t* state, int B, int C, int H, int W, int M, int K, int pad, int bf16_ops,
                                  hipStream_t s);
void launch_sgd_flat(float* p, const float* g, float* m, long n, float lr, float momentum, float grad_scale,
                     hipStream_t s);
// element map of a packed conv-weight image (the LDS-patch plan of the job's layer)
void conv_pack_geometry(const ConvPackJob& job, int* M, int* C, int* K, int* Mp, int* Cp);
// conv-weight images the SGD tail refreshes (weight offset in the arena, packed destination)
struct PackScatter {
  static constexpr int kMax = 16;
  struct Item {
    long off, len;
    void* dst;
    int M, C, K, Mp, Cp, flip, bf;
  } it[kMax];
  int n;
};
// deferred conv weight-gradient slice sums (launch_conv_wgrad with dw == nullptr): part rows are
// [S][M][Kd + 1]; element e = m (Kd + 1) + j of their sum is dW[m][j] (j < Kd) or db[m] (j == Kd)
struct SliceJob {
  const float* part;
  int S, M, Kd;
  long dw_off, db_off;  // arena offsets of dW (M x Kd) and db (M)
};
struct SliceSet {
  static constexpr int kMax = 8;
  SliceJob it[kMax];
  int start[kMax + 1];  // prefix sums of the jobs' 16-element groups
  int n;
};
// SGD + packed conv-weight images (jobs: conv_pack_all's list; arena: the parameter arena the
// jobs' weights live in) + the step bookkeeping (book != nullptr) in one launch; slices: conv
// gradients still in slice partials - their elements are summed, stored to g and updated here
void launch_sgd_tail(float* p, float* g, float* m, long n, float lr, float momentum, float grad_scale,
                     const ConvPackJob* jobs, int njobs, const float* arena, const SliceJob* slices, int nslices,
                     const ReduceArgs* book, hipStream_t s);
// Linear layers on MFMA (linear.hip): y = act(x W^T + b); dx = dz W; dW = dz^T x, db = sum_b dz,
// dz = dy masked by y > 0 when y != nullptr (fused ReLU)
void launch_linear_fwd(const float* x, const float* w, const float* b, float* y, int B, int K, int N, int relu,
                       hipStream_t s);
int linear_splitk_splits(int B, int K, int N);
void launch_linear_fwd_splitk(const float* x, const float* w, const float* b, float* y, float* part, int S, int B,
                              int K, int N, int relu, hipStream_t s);
void launch_linear_dgrad(const float* dy, const float* y, const float* w, float* dx, int B, int K, int N,
                         hipStream_t s);
void launch_linear_wgrad(const float* dy, const float* y, const float* x, float* dw, float* db, int B, int K, int N,
                         hipStream_t s);
void launch_linear_fwd_xent(const float* x, const float* w, const float* b, float* y, const int32_t* labels,
                            const int32_t* state, float* loss, int32_t* correct, float* dlogits, int B, int K, int N,
                            hipStream_t s);
void launch_linear_bwd(const float* dy, const float* y, const float* w, const float* x, float* dx, float* dw,
                       float* db, int B, int K, int N, hipStream_t s);

}  // namespace dnn

// Host-side launch API of the gfx950 kernels (used by csrc/bindings.cpp).
#pragma once
#include "common.h"

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
};

void launch_fused_train(const uint8_t* images, const int32_t* labels, const int32_t* order, int order_len,
                        int batch, int32_t* state, const float* master, const bf16* shadow, float* a0,
                        float* h1, float* h2, float* z1, float* z2, float* z3, float* slab, float* loss,
                        int32_t* correct, long long* stamps, const ReduceArgs* ra, unsigned* sync,
                        hipStream_t stream);
void launch_fused_eval(const uint8_t* images, const int32_t* labels, const int32_t* order, int n, int base,
                       int count, const float* master, const bf16* shadow, float* loss, int32_t* correct,
                       hipStream_t stream);


// one-time kernel attribute setup (must run before any hipGraph capture)
void init_kernels();
void launch_grad_reduce(const ReduceArgs& args, hipStream_t stream);
void launch_sgd_apply(float* master, const float* grad, float* mom, bf16* shadow, int n, float lr, float momentum,
                      float grad_scale, int pack_only, hipStream_t stream);

}  // namespace dnn

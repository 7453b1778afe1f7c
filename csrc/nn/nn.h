// Non-GEMM NN kernels (softmax + cross-entropy, bias-gradient column sums).
#pragma once
#include "bfp/bfp_format.h"

namespace fan {

// Writes per-row loss (lse - x[label]) and dlogits = (softmax - onehot) * grad_scale.
void launch_softmax_xent(int in_dtype, const void* logits, int64_t ld, const int32_t* labels, int out_dtype,
                         void* dlogits, int64_t ldd, float* loss_rows, int M, int C, float grad_scale,
                         hipStream_t s);

// The same with the logits given as the classifier GEMM's unreduced split-K slabs ws[k][M][C] (k < sk) + bias
// (bf16): logits = the slabs' sum in split order + bias (written to `logits`, bit-identical to the GEMM's reduce).
bool softmax_xent_slabs_supported(int C);
void launch_softmax_xent_slabs(const float* ws, int sk, const bf16_t* bias, float* logits, int64_t ld,
                               const int32_t* labels, int out_dtype, void* dlogits, int64_t ldd, float* loss_rows,
                               int M, int C, float grad_scale, hipStream_t s);

size_t col_sum_workspace_floats(int M, int N);
// out[n] (+)= scale * sum_m x[m][n]
void launch_col_sum(int in_dtype, const void* x, int64_t ld, int M, int N, int out_dtype, void* out, float scale,
                    bool accumulate, float* workspace, hipStream_t s);

}  // namespace fan

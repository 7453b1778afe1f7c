// Layer-chain GEMM: the GEMMs of one MLP pass as one persistent launch (see the layer-chain comment in
// gemm_bf16_kernel.h and gemm_chain.hip).
#pragma once
#include "gemm/gemm.h"

namespace fan {

enum GemmChainKind : int {
  // forward: stages 0 .. n-2 bias+ReLU bf16 (A K-contiguous X / H, B MN-contiguous W), 256x256 tiles; the last stage
  // either the same or bias-only f32 logits on 256x128 tiles
  kChainFwd = 0,
  // backward data: every stage ReLU-mask bf16 (A K-contiguous dZ, B K-contiguous W), 256x256 tiles
  kChainBwdData = 1,
};

int gemm_chain_max_stages();
// a[0..n-1]: the stages' GEMM args; stage s + 1's A must be stage s's C (same pointer, lda == ldc, K == N of s).
bool gemm_chain_supported(const GemmArgs* a, int n, int kind);
// counters: a zero-initialised block of gemm_chain_counter_words(n, M) uint32 (one per call site and stream; the
// kernel leaves it zeroed again); returns nothing, errors raise.
int gemm_chain_counter_words(int n, int M);
void launch_gemm_chain(const GemmArgs* a, int n, int kind, unsigned* counters, hipStream_t stream);

}  // namespace fan

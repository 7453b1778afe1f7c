// Grouped GEMM launch: up to kGroupMax bwd-weight GEMMs of one configuration in one dispatch. See gemm_group.hip.
#pragma once
#include "gemm/gemm.h"

namespace fan {

// n <= kGroupMax bwd-weight GEMMs dW_i = X_i^T . dY_i (A and B MN-contiguous, f32 out, no accumulate), each with its
// fused bias gradient (colsum) and either the BFP wire epilogue (all of them) or none; 256x128 tiles, one per
// workgroup, no split-K: M_i % 256 == 0, N_i % 128 == 0, K_i % 64 == 0. a[i].workspace: f32 scratch of
// gemm_wgrad_group_ws(a[i]) elements (the bias-gradient partials, one slab per 256-row tile row).
constexpr int kGroupMax = 8;
bool gemm_wgrad_group_supported(const GemmArgs* a, int n);
int64_t gemm_wgrad_group_ws(const GemmArgs& a);
void launch_gemm_wgrad_group(const GemmArgs* a, int n, hipStream_t stream);

}  // namespace fan

// Grouped backward GEMMs of one layer (bwd-data + bwd-weight in one dispatch). See gemm_pair.hip.
#pragma once
#include "gemm/gemm.h"

namespace fan {

// bd: bwd-data args (A dZ K-contiguous, B W K-contiguous, ReLU-mask epilogue, bf16 out); bw: bwd-weight args (A X and
// B dZ MN-contiguous, f32 out, tile_bn 128 or 256). grid0 / grid1: workgroups of each (multiples of the XCD count).
bool gemm_bwd_pair_supported(const GemmArgs& bd, const GemmArgs& bw, int grid0, int grid1);
void launch_gemm_bwd_pair(const GemmArgs& bd, const GemmArgs& bw, int grid0, int grid1, hipStream_t stream);

}  // namespace fan

// Grouped backward of one MLP layer: bwd-data and bwd-weight in ONE dispatch (gemm_group2_kernel), each on its own
// share of the CUs. Reference: libxsmm's PASS_BWD computes dX and dW of a layer in one fc_bwd_exec call
// (sw/mlp_mpi_example_f32.cpp:741-742).
#include "gemm/gemm_bf16_kernel.h"
#include "gemm/gemm_pair.h"

namespace fan {

using namespace gemm_detail;

namespace {

template <typename TC>
PlProblem<TC> problem_of(const GemmArgs& a, const WireOut& wo) {
  return PlProblem<TC>{(const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb, (TC*)a.C, a.ldc, (const bf16_t*)a.bias,
                       (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, 1, (float*)a.workspace, a.colsum, wo};
}

template <class P0, class P1>
void launch_group(const GemmArgs& a0, const GemmArgs& a1, int grid0, int grid1, hipStream_t s) {
  constexpr int lds = P0::kLds > P1::kLds ? P0::kLds : P1::kLds;
  auto k = gemm_group2_kernel<P0, P1>;
  FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const WireOut none{};
  hipLaunchKernelGGL(k, grid0 + grid1, 256, lds, s, problem_of<typename P0::TC>(a0, none),
                     problem_of<typename P1::TC>(a1, none), grid0);
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace

bool gemm_bwd_pair_supported(const GemmArgs& bd, const GemmArgs& bw, int grid0, int grid1) {
  if (grid0 <= 0 || grid1 <= 0 || grid0 % kNumXCD || grid1 % kNumXCD || grid0 + grid1 > 4 * kNumCU) return false;
  // bwd-data: dX = dZ . W^T (both operands K-contiguous), ReLU-mask epilogue, bf16 out, 256x256 tiles
  if (!bd.a_kcontig || !bd.b_kcontig || bd.epilogue != kEpiReluMask || !bd.c_bf16 || bd.accumulate || !bd.aux)
    return false;
  if (bd.M % 256 || bd.N % 256 || bd.K % 64) return false;
  // bwd-weight: dW = X^T . dZ (both operands MN-contiguous), plain f32 out, 256x256 or 256x128 tiles, no split-K
  if (bw.a_kcontig || bw.b_kcontig || bw.epilogue != kEpiNone || bw.c_bf16 || bw.accumulate || bw.colsum) return false;
  if (bw.tile_bn != 128 && bw.tile_bn != 256) return false;
  if (bw.M % 256 || bw.N % bw.tile_bn || bw.K % 64) return false;
  if (((uintptr_t)bd.C | (uintptr_t)bd.aux) & 15 || bd.ldc % 8 || bd.ldaux % 8) return false;
  return true;
}

void launch_gemm_bwd_pair(const GemmArgs& bd, const GemmArgs& bw, int grid0, int grid1, hipStream_t s) {
  FAN_CHECK(gemm_bwd_pair_supported(bd, bw, grid0, grid1), "gemm_bwd_pair: unsupported shapes / layouts / grids");
  using P0 = PlCfg<true, true, kEpiReluMask, bf16_t, false, false, false, 256, 256>;
  if (bw.tile_bn == 128) launch_group<P0, PlCfg<false, false, kEpiNone, float, false, false, false, 128, 256>>(bd, bw, grid0, grid1, s);
  else launch_group<P0, PlCfg<false, false, kEpiNone, float, false, false, false, 256, 256>>(bd, bw, grid0, grid1, s);
}

}  // namespace fan

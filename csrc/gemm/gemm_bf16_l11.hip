// bf16 GEMM instantiations for A K-contiguous, B K-contiguous: the 128-wide tiles (the 256x256 tiles, by far the
// largest instantiation set, compile in parallel in gemm_bf16_l11_t256.hip).
#include "gemm/gemm_bf16_launch.h"

namespace fan {
namespace gemm_detail {
extern template void launch_epi<256, 256, 2, 4, true, true>(const GemmArgs&, int, hipStream_t);
template void launch_tile<true, true>(const GemmArgs&, int, int, int, int, hipStream_t);
}  // namespace gemm_detail
}  // namespace fan

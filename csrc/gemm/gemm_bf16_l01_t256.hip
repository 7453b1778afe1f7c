// bf16 GEMM instantiations for A MN-contiguous, B K-contiguous: 256x256 tiles (one-role, pipelined 8-wave and 4-wave
// main loops).
#include "gemm/gemm_bf16_launch.h"

namespace fan {
namespace gemm_detail {
template void launch_epi<256, 256, 2, 4, false, true>(const GemmArgs&, int, hipStream_t);
}  // namespace gemm_detail
}  // namespace fan

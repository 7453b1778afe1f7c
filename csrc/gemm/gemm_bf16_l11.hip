// bf16 GEMM instantiations for A K-contiguous, B K-contiguous.
#include "gemm/gemm_bf16_kernel.h"

namespace fan {
namespace gemm_detail {
template void launch_tile<true, true>(const GemmArgs&, int, int, int, int, hipStream_t);
}  // namespace gemm_detail
}  // namespace fan

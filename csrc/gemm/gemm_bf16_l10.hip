// bf16 GEMM instantiations for A K-contiguous, B MN-contiguous.
#include "gemm/gemm_bf16_kernel.h"

namespace fan {
namespace gemm_detail {
template void launch_tile<true, false>(const GemmArgs&, int, int, int, int, hipStream_t);
}  // namespace gemm_detail
}  // namespace fan

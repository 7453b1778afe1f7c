// Multi-segment copy: one launch moves every segment of a P2P round (one per peer), so all xGMI links carry
// traffic at once instead of one hipMemcpyAsync after another. Each workgroup walks 16-B chunks of the
// concatenated segments (grid-stride); stores to IPC-mapped peer pointers travel over xGMI.
#include "bfp/bfp_format.h"
#include "comm/p2p_comm.h"

namespace fan {

namespace {

constexpr int kMaxSeg = 16;

struct Segs {
  const uint8_t* src[kMaxSeg];
  uint8_t* dst[kMaxSeg];
  uint64_t end[kMaxSeg];  // exclusive prefix sums of the segment sizes (bytes, multiples of 16)
  int n;
};

__global__ void __launch_bounds__(256) multi_copy_kernel(Segs s, int rel) {
  const uint64_t total = s.end[s.n - 1] >> 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  int seg = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint64_t b = i << 4;
    while (b >= s.end[seg]) ++seg;  // i only grows: the segment index only moves forward
    const uint64_t off = b - (seg ? s.end[seg - 1] : 0);
    const uint4 v = *reinterpret_cast<const uint4*>(s.src[seg] + off);
    *reinterpret_cast<uint4*>(s.dst[seg] + off) = v;
  }
  // peer stores are posted over xGMI: make them visible system-wide before the kernel retires, i.e. before
  // the stream-ordered flag write that tells the peer to read them (bfp_format.h p2p_release)
  p2p_release(rel);
}

}  // namespace

void launch_multi_copy(const std::vector<P2PCopy>& segs, hipStream_t stream) {
  for (size_t first = 0; first < segs.size(); first += kMaxSeg) {
    Segs s{};
    uint64_t acc = 0;
    s.n = 0;
    for (size_t k = first; k < segs.size() && s.n < kMaxSeg; ++k) {
      const P2PCopy& c = segs[k];
      if (c.bytes == 0) continue;
      FAN_CHECK(c.bytes % 16 == 0 && ((uintptr_t)c.src & 15) == 0 && ((uintptr_t)c.dst & 15) == 0,
                "multi_copy: 16-B aligned segments expected");
      s.src[s.n] = static_cast<const uint8_t*>(c.src);
      s.dst[s.n] = static_cast<uint8_t*>(c.dst);
      acc += c.bytes;
      s.end[s.n] = acc;
      ++s.n;
    }
    if (s.n == 0) continue;
    const int grid = stream_grid(acc / 16, 256, p2p_grid_cap());
    hipLaunchKernelGGL(multi_copy_kernel, grid, 256, 0, stream, s, p2p_release_mode());
    FAN_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace fan

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

namespace {

constexpr int kMaxFlags = 16;
constexpr uint32_t kFlagSpinLimit = 1u << 22;  // s_sleep 2 + an uncached (remote) load per trip: several seconds
struct FlagOps {
  uint64_t* p[kMaxFlags];
  uint64_t v[kMaxFlags];
  int n;
};

// lane i publishes word i: a system-scope release (this kernel follows the round's payload kernels in stream order;
// in release modes block / thread they released their peer stores themselves, in mode cp the release event does) and
// a system-coherent store, so the peer's spin or command processor sees the value once the payload is visible
__global__ void __launch_bounds__(64) flag_write_kernel(FlagOps f) {
  const int i = threadIdx.x;
  if (i < f.n) __hip_atomic_store(f.p[i], f.v[i], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// lane i spins on word i (relaxed system-scope loads of this rank's uncached flag block, s_sleep between), then the
// wave acquires at system scope: the next kernel of the stream, which reads the arena slot, starts after this one
__global__ void __launch_bounds__(64) flag_wait_kernel(FlagOps f, unsigned* err) {
  const int i = threadIdx.x;
  if (i < f.n) {
    for (uint32_t spins = 0; __hip_atomic_load(f.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < f.v[i];) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > kFlagSpinLimit) {  // a dead or aborted peer that nobody poisoned: give up (error), no hang
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

template <class K, class... X>
void launch_flag_batches(K kernel, const std::vector<std::pair<uint64_t*, uint64_t>>& w, hipStream_t stream,
                         X... extra) {
  for (size_t first = 0; first < w.size(); first += kMaxFlags) {
    FlagOps f{};
    f.n = 0;
    for (size_t k = first; k < w.size() && f.n < kMaxFlags; ++k) {
      f.p[f.n] = w[k].first;
      f.v[f.n] = w[k].second;
      ++f.n;
    }
    hipLaunchKernelGGL(kernel, 1, 64, 0, stream, f, extra...);
    FAN_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace

void launch_flag_write(const std::vector<std::pair<uint64_t*, uint64_t>>& w, hipStream_t stream) {
  launch_flag_batches(flag_write_kernel, w, stream);
}

void launch_flag_wait(const std::vector<std::pair<uint64_t*, uint64_t>>& w, unsigned* err, hipStream_t stream) {
  launch_flag_batches(flag_wait_kernel, w, stream, err);
}

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

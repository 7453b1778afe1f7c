// Message tags / verification / fault-injection kernels. See verify.h.
#include "comm/verify.h"

#include <chrono>
#include <sstream>
#include <thread>

namespace fan {

namespace {

// grid (blocks per row, rows): each block folds its 16-B chunks of one row into (s1, s2) and adds them to the row's
// tag (uint32 wrap-around sums are associative, so the block order does not matter).
__global__ void __launch_bounds__(256) msg_sum_kernel(const uint8_t* __restrict__ rows, size_t row_bytes,
                                                      size_t row_stride, uint32_t* __restrict__ tags) {
  const int r = blockIdx.y;
  const uint4* p = reinterpret_cast<const uint4*>(rows + (size_t)r * row_stride);
  const size_t chunks = row_bytes / 16;
  uint32_t s1 = 0, s2 = 0;
  for (size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[c];
    const uint32_t i = (uint32_t)(c * 4);
    s1 += v.x + v.y + v.z + v.w;
    s2 += (i + 1) * v.x + (i + 2) * v.y + (i + 3) * v.z + (i + 4) * v.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += (uint32_t)__shfl_xor((int)s1, o);
    s2 += (uint32_t)__shfl_xor((int)s2, o);
  }
  __shared__ uint32_t red[2][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0, b = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
      a += red[0][k];
      b += red[1][k];
    }
    atomicAdd(&tags[r * 4 + 0], a);
    atomicAdd(&tags[r * 4 + 1], b);
  }
}

__global__ void msg_seal_kernel(uint32_t* __restrict__ tags, int nrows, uint32_t seq, uint32_t row_bytes) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < nrows) {
    tags[r * 4 + 2] = seq;
    tags[r * 4 + 3] = row_bytes;
  }
}

__global__ void msg_compare_kernel(const uint32_t* __restrict__ got, const uint32_t* __restrict__ exp, int nrows,
                                   uint32_t expect_seq, VerifyError* __restrict__ err, uint32_t site,
                                   uint32_t row_base) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  const uint32_t* e = exp + r * 4;
  const uint32_t* g = got + r * 4;
  uint32_t kind = 0;
  if (e[2] != expect_seq) kind = 2;
  else if (e[0] != g[0] || e[1] != g[1] || e[3] != g[3]) kind = 1;
  if (kind && atomicCAS(&err->flag, 0u, 1u) == 0u) {
    err->kind = kind;
    err->site = site;
    err->row = row_base + (uint32_t)r;
    err->exp_s1 = e[0];
    err->got_s1 = g[0];
    err->exp_seq = expect_seq;
    err->got_seq = e[2];
  }
}

__global__ void fault_byte_kernel(uint8_t* p, size_t bytes, int kind) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (kind == 0) p[0] ^= 0xFF;
    else p[bytes - 1] = 0xFF;
  }
}

void tags_into(const uint8_t* rows, size_t row_bytes, size_t row_stride, int nrows, uint32_t seq, uint32_t* tags,
               hipStream_t s) {
  FAN_CHECK(row_bytes % 16 == 0 && row_stride % 16 == 0, "message rows must be 16-B multiples");
  FAN_HIP_CHECK(hipMemsetAsync(tags, 0, (size_t)nrows * 16, s));
  const size_t chunks = row_bytes / 16;
  const int bx = (int)std::min<size_t>(64, std::max<size_t>(1, (chunks + 255) / 256));
  hipLaunchKernelGGL(msg_sum_kernel, dim3(bx, nrows), 256, 0, s, rows, row_bytes, row_stride, tags);
  hipLaunchKernelGGL(msg_seal_kernel, (nrows + 63) / 64, 64, 0, s, tags, nrows, seq, (uint32_t)row_bytes);
}

}  // namespace

void launch_msg_tags(const uint8_t* rows, size_t row_bytes, size_t row_stride, int nrows, uint32_t seq, uint32_t* tags,
                     hipStream_t s) {
  tags_into(rows, row_bytes, row_stride, nrows, seq, tags, s);
  FAN_HIP_CHECK(hipGetLastError());
}

void launch_msg_verify(const uint8_t* rows, size_t row_bytes, size_t row_stride, int nrows, const uint32_t* recv_tags,
                       uint32_t expect_seq, uint32_t* scratch, VerifyError* err, uint32_t site, uint32_t row_base,
                       hipStream_t s) {
  tags_into(rows, row_bytes, row_stride, nrows, expect_seq, scratch, s);
  hipLaunchKernelGGL(msg_compare_kernel, (nrows + 63) / 64, 64, 0, s, scratch, recv_tags, nrows, expect_seq, err, site,
                     row_base);
  FAN_HIP_CHECK(hipGetLastError());
}

void launch_fault_byte(uint8_t* p, size_t bytes, int kind, hipStream_t s) {
  hipLaunchKernelGGL(fault_byte_kernel, 1, 64, 0, s, p, bytes, kind);
  FAN_HIP_CHECK(hipGetLastError());
}

FaultInjector::FaultInjector() {
  if (const char* e = std::getenv("FAN_FAULT")) *this = FaultInjector(e);
}

FaultInjector::FaultInjector(const std::string& spec) : rules_(parse_fault_spec(spec)) {}

void FaultInjector::maybe_corrupt(const std::string& site, uint8_t* buf, size_t bytes, hipStream_t s) {
  if (rules_.empty()) return;
  const int64_t k = counts_[site]++;
  for (const FaultRule& r : rules_) {
    if (r.site != site || r.index != k) continue;
    if (r.kind == "flip") launch_fault_byte(buf, bytes, 0, s);
    else if (r.kind == "nan") launch_fault_byte(buf, bytes, 1, s);
    else if (r.kind == "delay_ms") {  // the request's producer-side progress stalls (what a slow link looks like)
      FAN_HIP_CHECK(hipStreamSynchronize(s));
      std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(r.delay_ms * 1000.0)));
    }
  }
}

bool FaultInjector::maybe_drop(const std::string& site) {
  if (rules_.empty()) return false;
  const int64_t k = counts_[site]++;
  for (const FaultRule& r : rules_)
    if (r.site == site && r.index == k && r.kind == "drop") return true;
  return false;
}

}  // namespace fan

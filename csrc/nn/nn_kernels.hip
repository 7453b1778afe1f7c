// Non-GEMM training kernels for the MLP (gfx950):
//   softmax_xent : fused softmax + cross-entropy forward AND backward (one wave per row, online
//                  max/sum in one read, gradient written in a second pass over the L1/L2-resident row).
//                  Reference: libxsmm smax fwd/bwd with loss_weight (sw/mlp_mpi_example_f32.cpp:525-531,
//                  718-728).
//   col_sum      : bias gradient db[n] = sum_m dZ[m][n], two-pass deterministic (row-chunk partials in a
//                  workspace, then an ordered sum). Reference: libxsmm fc bwd dbias (sw:741-742).
#include "nn/nn.h"

namespace fan {
namespace {

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float v[8]);
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float v[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float v[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float v[8]);
template <>
__device__ __forceinline__ void st8<float>(float* p, const float v[8]) {
  reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}
template <>
__device__ __forceinline__ void st8<bf16_t>(bf16_t* p, const float v[8]) {
  uint4 u;
  u.x = pack_bf16x2(v[0], v[1]);
  u.y = pack_bf16x2(v[2], v[3]);
  u.z = pack_bf16x2(v[4], v[5]);
  u.w = pack_bf16x2(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = u;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <typename T>
__device__ __forceinline__ float ld1(const T* p) {
  if constexpr (sizeof(T) == 4) return *reinterpret_cast<const float*>(p);
  else return bf16_to_f32(*reinterpret_cast<const bf16_t*>(p));
}
template <typename T>
__device__ __forceinline__ void st1(T* p, float v) {
  if constexpr (sizeof(T) == 4) *reinterpret_cast<float*>(p) = v;
  else *reinterpret_cast<bf16_t*>(p) = f32_to_bf16(v);
}

// Rows of up to NCH * 512 classes (C, ld, ldd % 8 == 0): the row stays in registers (8 * NCH values per lane), so
// the logits are read from memory once, every chunk's load is in flight before the first max, and each exp is
// computed once (the flagship's 8192 x 1024 f32 logits: one 32 MB read + the 16 MB dlogits write).
template <typename TIN, typename TOUT, int NCH>
__global__ void __launch_bounds__(256)
    softmax_xent_reg_kernel(const TIN* __restrict__ logits, int64_t ld, const int32_t* __restrict__ labels,
                            TOUT* __restrict__ dlogits, int64_t ldd, float* __restrict__ loss_rows, int M, int C,
                            float grad_scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const TIN* x = logits + (int64_t)row * ld;
  const int lab = labels[row];
  float v[NCH][8];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
      ld8<TIN>(x + c, v[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = -INFINITY;
    }
  }
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, v[k][j]);
  const float gm = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[k][j] = __expf(v[k][j] - gm);  // -inf padding -> 0
      s += v[k][j];
    }
  s = wave_sum(s);
  const float inv = 1.f / s;
  if (lane == 0) {
    const float xl = sizeof(TIN) == 4 ? reinterpret_cast<const float*>(x)[lab]
                                      : bf16_to_f32(reinterpret_cast<const bf16_t*>(x)[lab]);
    loss_rows[row] = gm + __logf(s) - xl;
  }
  TOUT* d = dlogits + (int64_t)row * ldd;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c >= C) continue;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[k][j] * inv - (c + j == lab ? 1.f : 0.f)) * grad_scale;
    st8<TOUT>(d + c, o);
  }
}

// The classifier GEMM's split-K partial slabs folded in (ws[k][M][C], k < sk; the GEMM ran with defer_reduce): each
// logit is the slabs' sum in split order plus the bias — the arithmetic of the GEMM's own slab reduce
// (splitk_reduce_kernel with the bias epilogue), so the logits (also written out) are bit-identical and the reduce
// launch disappears. Then as softmax_xent_reg_kernel.
template <typename TOUT, int NCH, int SK>
__global__ void __launch_bounds__(256)
    softmax_xent_slab_kernel(const float* __restrict__ ws, int sk, const bf16_t* __restrict__ bias,
                             float* __restrict__ logits, int64_t ld, const int32_t* __restrict__ labels,
                             TOUT* __restrict__ dlogits, int64_t ldd, float* __restrict__ loss_rows, int M, int C,
                             float grad_scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int64_t slab = (int64_t)M * C;
  const float* x = ws + (int64_t)row * C;
  const int lab = labels[row];
  float v[NCH][8];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
      // (SK > 0: the split count at compile time, so every slab's load is in flight before the first add)
      float t[SK > 1 ? SK - 1 : 1][8];
      ld8<float>(x + c, v[k]);
#pragma unroll
      for (int q = 1; q < (SK > 0 ? SK : sk); ++q) ld8<float>(x + q * slab + c, t[SK > 0 ? q - 1 : 0]);
#pragma unroll
      for (int q = 1; q < (SK > 0 ? SK : sk); ++q) {
        if constexpr (SK == 0) ld8<float>(x + q * slab + c, t[0]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += t[SK > 0 ? q - 1 : 0][j];
      }
      float b[8];
      ld8<bf16_t>(bias + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] += b[j];
      st8<float>(logits + (int64_t)row * ld + c, v[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = -INFINITY;
    }
  }
  // the label's logit from the registers: lane (lab / 8) % 64 of chunk lab / 512 holds it
  float xl = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if ((k * 64 + lane) * 8 + j == lab) xl = v[k][j];
  xl = wave_sum(xl);
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, v[k][j]);
  const float gm = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[k][j] = __expf(v[k][j] - gm);
      s += v[k][j];
    }
  s = wave_sum(s);
  const float inv = 1.f / s;
  if (lane == 0) loss_rows[row] = gm + __logf(s) - xl;
  TOUT* d = dlogits + (int64_t)row * ldd;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c >= C) continue;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[k][j] * inv - (c + j == lab ? 1.f : 0.f)) * grad_scale;
    st8<TOUT>(d + c, o);
  }
}

// One wave per row; 4 waves per block. VEC: 8 values per lane access (C, ld, ldd % 8 == 0); otherwise one value
// per lane access (any class count, e.g. a 10-class head).
template <typename TIN, typename TOUT, bool VEC>
__global__ void __launch_bounds__(256)
    softmax_xent_kernel(const TIN* __restrict__ logits, int64_t ld, const int32_t* __restrict__ labels,
                        TOUT* __restrict__ dlogits, int64_t ldd, float* __restrict__ loss_rows, int M, int C,
                        float grad_scale) {
  constexpr int V = VEC ? 8 : 1;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const TIN* x = logits + (int64_t)row * ld;
  float m = -INFINITY, s = 0.f;
  for (int c = lane * V; c < C; c += 64 * V) {
    float v[V];
    if constexpr (VEC) ld8<TIN>(x + c, v);
    else v[0] = ld1<TIN>(x + c);
    float cm = v[0];
#pragma unroll
    for (int j = 1; j < V; ++j) cm = fmaxf(cm, v[j]);
    const float nm = fmaxf(m, cm);
    float cs = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) cs += __expf(v[j] - nm);
    s = s * __expf(m - nm) + cs;
    m = nm;
  }
  const float gm = wave_max(m);
  s = wave_sum(s * __expf(m - gm));
  const float inv = 1.f / s;
  const float lse = gm + __logf(s);
  const int lab = labels[row];
  if (lane == 0) {
    float xl = 0.f;
    if (sizeof(TIN) == 4) xl = reinterpret_cast<const float*>(x)[lab];
    else xl = bf16_to_f32(reinterpret_cast<const bf16_t*>(x)[lab]);
    loss_rows[row] = lse - xl;
  }
  TOUT* d = dlogits + (int64_t)row * ldd;
  for (int c = lane * V; c < C; c += 64 * V) {
    float v[V];
    if constexpr (VEC) ld8<TIN>(x + c, v);
    else v[0] = ld1<TIN>(x + c);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float p = __expf(v[j] - gm) * inv;
      v[j] = (p - (c + j == lab ? 1.f : 0.f)) * grad_scale;
    }
    if constexpr (VEC) st8<TOUT>(d + c, v);
    else st1<TOUT>(d + c, v[0]);
  }
}

// Partial column sums over a chunk of rows: block = 256 threads covers 64 columns (16 thr x 4 cols)
// and 16 row lanes; grid = (ceil(N/64), chunks). VEC: 4-column vector loads (N % 4 == 0, ld % 4 == 0); the
// scalar form takes any width.
template <typename T, bool VEC>
__global__ void __launch_bounds__(256)
    col_sum_partial_kernel(const T* __restrict__ x, int64_t ld, int M, int N, int rows_per_chunk,
                           float* __restrict__ part) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + tx * 4;
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = min(M, r0 + rows_per_chunk);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = r0 + ty; r < r1 && col < N; r += 16) {
    const T* p = x + (int64_t)r * ld + col;
    if (!VEC) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (col + u < N) acc[u] += ld1<T>(p + u);
    } else if (sizeof(T) == 4) {
      const float4 v = *reinterpret_cast<const float4*>(p);
      acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
    } else {
      const uint2 u = *reinterpret_cast<const uint2*>(p);
      acc[0] += __uint_as_float(u.x << 16);
      acc[1] += __uint_as_float(u.x & 0xFFFF0000u);
      acc[2] += __uint_as_float(u.y << 16);
      acc[3] += __uint_as_float(u.y & 0xFFFF0000u);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) red[ty][tx * 4 + u] = acc[u];
  __syncthreads();
  if (threadIdx.x < 64 && blockIdx.x * 64 + threadIdx.x < N) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][threadIdx.x];
    part[(int64_t)blockIdx.y * N + blockIdx.x * 64 + threadIdx.x] = s;
  }
}

template <typename TO>
__global__ void __launch_bounds__(256)
    col_sum_final_kernel(const float* __restrict__ part, int chunks, int N, TO* __restrict__ out, float scale,
                         int accumulate) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[(int64_t)c * N + n];
  s *= scale;
  if (sizeof(TO) == 4) {
    float* o = reinterpret_cast<float*>(out) + n;
    *o = accumulate ? *o + s : s;
  } else {
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + n;
    *o = f32_to_bf16(accumulate ? bf16_to_f32(*o) + s : s);
  }
}

}  // namespace

void launch_softmax_xent(int in_dtype, const void* logits, int64_t ld, const int32_t* labels, int out_dtype,
                         void* dlogits, int64_t ldd, float* loss_rows, int M, int C, float grad_scale,
                         hipStream_t s) {
  FAN_CHECK(C > 0, "softmax_xent needs C > 0");
  const int grid = (M + 3) / 4;
  const bool vec = C % 8 == 0 && ld % 8 == 0 && ldd % 8 == 0;
  const int nch = vec ? (C + 511) / 512 : 0;
#define FAN_SMX(TI, TO)                                                                                         \
  if (nch >= 1 && nch <= 4) {                                                                                   \
    auto k = nch == 1 ? softmax_xent_reg_kernel<TI, TO, 1> : nch == 2 ? softmax_xent_reg_kernel<TI, TO, 2>      \
           : nch == 3 ? softmax_xent_reg_kernel<TI, TO, 3> : softmax_xent_reg_kernel<TI, TO, 4>;                \
    hipLaunchKernelGGL(k, grid, 256, 0, s, (const TI*)logits, ld, labels, (TO*)dlogits, ldd, loss_rows, M, C,   \
                       grad_scale);                                                                             \
  } else if (vec)                                                                                               \
    hipLaunchKernelGGL((softmax_xent_kernel<TI, TO, true>), grid, 256, 0, s, (const TI*)logits, ld, labels,     \
                       (TO*)dlogits, ldd, loss_rows, M, C, grad_scale);                                          \
  else                                                                                                          \
    hipLaunchKernelGGL((softmax_xent_kernel<TI, TO, false>), grid, 256, 0, s, (const TI*)logits, ld, labels,    \
                       (TO*)dlogits, ldd, loss_rows, M, C, grad_scale);
  if (in_dtype == kF32 && out_dtype == kF32) {
    FAN_SMX(float, float)
  } else if (in_dtype == kF32 && out_dtype == kBF16) {
    FAN_SMX(float, bf16_t)
  } else if (in_dtype == kBF16 && out_dtype == kBF16) {
    FAN_SMX(bf16_t, bf16_t)
  } else {
    FAN_SMX(bf16_t, float)
  }
#undef FAN_SMX
  FAN_HIP_CHECK(hipGetLastError());
}

bool softmax_xent_slabs_supported(int C) { return C % 8 == 0 && C <= 2048; }

void launch_softmax_xent_slabs(const float* ws, int sk, const bf16_t* bias, float* logits, int64_t ld,
                               const int32_t* labels, int out_dtype, void* dlogits, int64_t ldd, float* loss_rows,
                               int M, int C, float grad_scale, hipStream_t s) {
  FAN_CHECK(softmax_xent_slabs_supported(C) && ld % 8 == 0 && ldd % 8 == 0 && sk >= 1,
            "softmax_xent over split-K slabs: C % 8 == 0, C <= 2048, ld / ldd % 8 == 0");
  const int grid = (M + 3) / 4;
  const int nch = (C + 511) / 512;
#define FAN_SMS_K(TO, SKC)                                                                                     \
  {                                                                                                            \
    auto k = nch == 1 ? softmax_xent_slab_kernel<TO, 1, SKC> : nch == 2 ? softmax_xent_slab_kernel<TO, 2, SKC> \
           : nch == 3 ? softmax_xent_slab_kernel<TO, 3, SKC> : softmax_xent_slab_kernel<TO, 4, SKC>;           \
    hipLaunchKernelGGL(k, grid, 256, 0, s, ws, sk, bias, logits, ld, labels, (TO*)dlogits, ldd, loss_rows, M, C, \
                       grad_scale);                                                                            \
  }
#define FAN_SMS(TO)                \
  if (sk == 2) FAN_SMS_K(TO, 2)    \
  else if (sk == 4) FAN_SMS_K(TO, 4) \
  else FAN_SMS_K(TO, 0)
  if (out_dtype == kBF16) {
    FAN_SMS(bf16_t)
  } else {
    FAN_SMS(float)
  }
#undef FAN_SMS
#undef FAN_SMS_K
  FAN_HIP_CHECK(hipGetLastError());
}

size_t col_sum_workspace_floats(int M, int N) {
  const int chunks = (M + 255) / 256;
  return (size_t)chunks * N;
}

void launch_col_sum(int in_dtype, const void* x, int64_t ld, int M, int N, int out_dtype, void* out, float scale,
                    bool accumulate, float* workspace, hipStream_t s) {
  FAN_CHECK(N > 0, "col_sum needs N > 0");
  const int rows_per_chunk = 256;
  const int chunks = (M + rows_per_chunk - 1) / rows_per_chunk;
  dim3 grid((N + 63) / 64, chunks);
  const bool vec = N % 4 == 0 && ld % 4 == 0;
  if (in_dtype == kF32 && vec)
    hipLaunchKernelGGL((col_sum_partial_kernel<float, true>), grid, 256, 0, s, (const float*)x, ld, M, N,
                       rows_per_chunk, workspace);
  else if (in_dtype == kF32)
    hipLaunchKernelGGL((col_sum_partial_kernel<float, false>), grid, 256, 0, s, (const float*)x, ld, M, N,
                       rows_per_chunk, workspace);
  else if (vec)
    hipLaunchKernelGGL((col_sum_partial_kernel<bf16_t, true>), grid, 256, 0, s, (const bf16_t*)x, ld, M, N,
                       rows_per_chunk, workspace);
  else
    hipLaunchKernelGGL((col_sum_partial_kernel<bf16_t, false>), grid, 256, 0, s, (const bf16_t*)x, ld, M, N,
                       rows_per_chunk, workspace);
  if (out_dtype == kF32)
    hipLaunchKernelGGL((col_sum_final_kernel<float>), (N + 255) / 256, 256, 0, s, workspace, chunks, N, (float*)out,
                       scale, accumulate ? 1 : 0);
  else
    hipLaunchKernelGGL((col_sum_final_kernel<bf16_t>), (N + 255) / 256, 256, 0, s, workspace, chunks, N,
                       (bf16_t*)out, scale, accumulate ? 1 : 0);
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace fan

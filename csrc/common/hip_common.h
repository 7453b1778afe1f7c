// Common HIP helpers for the fpga_ai_nic_amd native runtime (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

#define FAN_HIP_CHECK(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);      \
    }                                                                                        \
  } while (0)

#define FAN_CHECK(cond, msg)                                                                 \
  do {                                                                                       \
    if (!(cond)) throw std::runtime_error(std::string("fpga_ai_nic_amd: ") + (msg));        \
  } while (0)

namespace fan {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)
constexpr int kNumCU = 256;
constexpr int kNumXCD = 8;

typedef uint16_t bf16_t;  // raw bf16 storage

__device__ __forceinline__ float bf16_to_f32(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// RNE f32 -> bf16, NaN preserving (lowers to v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// Grid size for a grid-stride memory-bound kernel: enough waves to fill 256 CUs, capped.
inline int stream_grid(size_t work_items, int block = 256, int max_blocks = 2048) {
  size_t b = (work_items + block - 1) / block;
  if (b < 1) b = 1;
  if (b > (size_t)max_blocks) b = max_blocks;
  return (int)b;
}

}  // namespace fan

// Wire-codec kernels of the compressed all-reduce engine (gfx950).
//
// All kernels are HBM-streaming: each lane owns one 16-element BFP group (32-B loads of bf16, 64-B of f32; one
// 16-B mantissa store, and the group exponents of 16 consecutive lanes leave as one 16-B store, bfp_format.h
// WireLane16) — except wire_pack_range (the short bias / padding tails at any 16-element offset), where a lane
// PAIR owns a group. Grids are capped at 2048 blocks and grid-stride over every shard, so each lane runs the same
// number of iterations per shard and 16-lane segments never split (group counts are multiples of 16).
//
// Reference parity:
//   wire_pack    = bfp_adapter TX (hw/bfp_adapter.sv:100-154, 279-379)
//   wire_unpack  = bfp_adapter RX (hw/bfp_adapter.sv:489-699)
//   wire_reduce  = the ring engine's 8-lane fadd stage + re-encode (hw/all_reduce.sv:1090-1183)
//   wire_sgd     = weight_update FFMA w' = fma(-lr, g, w) (hw/weight_update.sv:433-452), fused
//                  into the all-gather epilogue so weights never take an extra HBM round trip.
#include "bfp/bfp_format.h"

#include <algorithm>
#include <atomic>
#include <cstring>

namespace fan {

static int wire_max_blocks();

// The lane-contiguous (4 values per lane) BFP reduce kernels pay off where the dense f32 operands dominate the bytes
// (the local gradient, the master / momentum planes) and cost where the 1-byte wire slots do — one group per lane
// already reads a slot's mantissas 1 KiB per wave instruction, 4 values per lane 256 B: C.wire_reduce of 8 slots
// measured 38.1 vs 33.6 us, of 2 slots 17.0 vs 17.1 (tools/probes/wire_reduce4_probe.py). So they run for at most two
// slots (world 1 through the multi-rank path, 2 ranks); FAN_WIRE_REDUCE4=0 turns them off.
static bool wire_reduce4_for(int n_slots) { return n_slots <= 2 && wire_reduce4() != 0; }

static std::atomic<int>& release_mode_flag() {
  static std::atomic<int> m{[] {
    const char* e = getenv("FAN_P2P_RELEASE");
    if (!e) return 3;
    if (!strcmp(e, "thread")) return 2;
    if (!strcmp(e, "none")) return 0;
    if (!strcmp(e, "block")) return 1;
    return 3;
  }()};
  return m;
}
int p2p_release_mode() { return release_mode_flag().load(std::memory_order_relaxed); }
void set_p2p_release_mode(int mode) { release_mode_flag().store(mode < 0 ? 0 : mode > 3 ? 3 : mode); }

// Grid cap of the kernels that store into peers' receive arenas (FAN_P2P_GRID; 0 = auto): with the in-kernel
// release forms every workgroup ends with one system-scope release, so fewer, longer-lived workgroups pay fewer of
// them — "block" (the cross-device default) 128: 2 ranks, 2.27 ms/step at 64-128 workgroups vs 2.36 at 256, 2.49 at
// 512, 2.63 at 1024, 2.83 at 2048, i.e. the whole cost of the in-kernel release over "cp" (2.27)
// (profiles/r4_p2p_block_grid_sweep.jsonl); "thread" 512; with the command-processor release nothing is paid per
// workgroup and the cap is the ordinary one (profiles/r3_wire_store_bw.jsonl: 18.95 us at 512 vs 17.39 at 2048).
static std::atomic<int>& p2p_grid_flag() {
  static std::atomic<int> g{[] {
    const char* e = getenv("FAN_P2P_GRID");
    return e ? atoi(e) : 0;
  }()};
  return g;
}
int p2p_grid_cap() {
  const int g = p2p_grid_flag().load(std::memory_order_relaxed);
  if (g > 0) return g;
  const int m = p2p_release_mode();
  return m == 1 ? 128 : m == 2 ? 512 : wire_max_blocks();
}
void set_p2p_grid_cap(int blocks) { p2p_grid_flag().store(blocks > 0 ? blocks : 0); }

// Upper bound on the workgroups of one wire kernel (env FAN_WIRE_MAX_BLOCKS, default 2048): these memory-bound
// kernels run on the comm stream beside the GEMMs at world > 1, and every CU they occupy cannot host a GEMM
// workgroup (profiles/r1_gemm_cu_contention_probe.txt), so the footprint is a tunable. Measured at world 1 through
// the multi-rank path: capping it at 512 / 128 / 64 made the step 0.4 / 4 / 11 % slower
// (profiles/r1_wire_grid_cap_ab.txt) — the kernels are on the critical path more than they crowd the GEMMs.
static int wire_max_blocks() {
  static const int v = [] {
    const char* e = getenv("FAN_WIRE_MAX_BLOCKS");
    const int x = e ? atoi(e) : 0;
    return x > 0 ? x : 2048;
  }();
  return v;
}

namespace {

constexpr int kBlock = 256;

template <typename TIN, int C>
__global__ void __launch_bounds__(kBlock) wire_pack_kernel(const TIN* __restrict__ in, uint8_t* __restrict__ out,
                                                          size_t n_s, int n_shards) {
  const size_t tasks = n_s >> 4;  // one 16-value group per lane (WireLane16)
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t sb = wire_shard_bytes(C, n_s);
  for (int s = 0; s < n_shards; ++s) {
    const TIN* src = in + (size_t)s * n_s;
    uint8_t* dst = out + (size_t)s * sb;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
      float v[16];
      DenseLane16<TIN>::load16(src, t << 4, v);
      WireLane16<C>::store16(dst, n_s, t << 4, v);
    }
  }
}

// Pack flat elements [begin, end) (multiples of 16) of a bucket into its shard layout (shards of n_s elements):
// the part of a bucket the producing GEMM did not encode itself (bias gradient + padding).
template <typename TIN, int C>
__global__ void __launch_bounds__(kBlock) wire_pack_range_kernel(const TIN* __restrict__ in, uint8_t* __restrict__ out,
                                                                size_t n_s, size_t begin, size_t end) {
  const size_t tasks = (end - begin) >> 3;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t sb = wire_shard_bytes(C, n_s);
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
    const size_t f = begin + (t << 3);
    const size_t sh = f / n_s;
    float v[8];
    DenseLane<TIN>::load8(in, f, v);
    WireLane<C>::store8(out + sh * sb, n_s, f - sh * n_s, v);
  }
}

template <typename TOUT, int C>
__global__ void __launch_bounds__(kBlock) wire_unpack_kernel(const uint8_t* __restrict__ in, TOUT* __restrict__ out,
                                                            size_t n_s, int n_shards) {
  const size_t tasks = n_s >> 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t sb = wire_shard_bytes(C, n_s);
  for (int s = 0; s < n_shards; ++s) {
    const uint8_t* src = in + (size_t)s * sb;
    TOUT* dst = out + (size_t)s * n_s;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
      float v[16];
      WireLane16<C>::load16(src, n_s, t << 4, v);
      DenseLane16<TOUT>::store16(dst, t << 4, v);
    }
  }
}

template <typename TL, int C, bool HAS_LOCAL, bool OUT_WIRE, bool OUT_F32>
__global__ void __launch_bounds__(kBlock)
    wire_reduce_kernel(const uint8_t* __restrict__ slots, size_t slot_stride, int n_slots, int self_pos,
                       const TL* __restrict__ local, uint8_t* __restrict__ out_wire, float* __restrict__ out_f32,
                       size_t n_s) {
  const size_t tasks = n_s >> 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
    const size_t le = t << 4;
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
    for (int r = 0; r < n_slots; ++r) {
      float v[16];
      if (HAS_LOCAL && r == self_pos) {
        DenseLane16<TL>::load16(local, le, v);
      } else {
        WireLane16<C>::load16(slots + (size_t)r * slot_stride, n_s, le, v);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] += v[j];
    }
    if (OUT_F32) DenseLane16<float>::store16(out_f32, le, acc);
    if (OUT_WIRE) WireLane16<C>::store16(out_wire, n_s, le, acc);
  }
}

// wire_reduce_kernel for the BFP codecs, lane-contiguous (as wire_reduce_to4_kernel): 4 values per lane, the group
// exponent from quad xor shuffles; bit-identical (FAN_WIRE_REDUCE4).
template <typename TL, int C, bool HAS_LOCAL, bool OUT_WIRE, bool OUT_F32>
__global__ void __launch_bounds__(kBlock)
    wire_reduce4_kernel(const uint8_t* __restrict__ slots, size_t slot_stride, int n_slots, int self_pos,
                        const TL* __restrict__ local, uint8_t* __restrict__ out_wire, float* __restrict__ out_f32,
                        size_t n_s) {
  static_assert(C == kBfpTrunc || C == kBfpRne, "BFP codecs");
  const size_t tasks = n_s >> 2;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
    const size_t le = t << 2;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < n_slots; ++r) {
      float v[4];
      if (HAS_LOCAL && r == self_pos) {
        if constexpr (sizeof(TL) == 4) {
          const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(local) + le);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        } else {
          const uint2 a = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(local) + le);
          v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xFFFF0000u);
          v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xFFFF0000u);
        }
      } else {
        const uint8_t* sh = slots + (size_t)r * slot_stride;
        const uint32_t m = *reinterpret_cast<const uint32_t*>(sh + le);
        const uint32_t E = sh[n_s + (le >> 4)];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int32_t q = (int32_t)(int8_t)(uint8_t)(m >> (8 * j));
          v[j] = (C == kBfpTrunc) ? bfp_decode_trunc(q, E) : bfp_decode_rne(q, E);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += v[j];
    }
    if (OUT_F32) *reinterpret_cast<float4*>(out_f32 + le) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    if (OUT_WIRE) {
      uint32_t mx = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) mx = max(mx, __float_as_uint(acc[j]) & 0x7FFFFFFFu);
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, 1));
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, 2));
      const uint32_t E = mx >> 23;
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t q =
            (C == kBfpTrunc) ? bfp_encode_trunc(__float_as_uint(acc[j]), E) : bfp_encode_rne(acc[j], E);
        w |= ((uint32_t)q & 0xFFu) << (8 * j);
      }
      *reinterpret_cast<uint32_t*>(out_wire + le) = w;
      if ((le & 15) == 0) out_wire[n_s + (le >> 4)] = (uint8_t)E;
    }
  }
}

// Direct-transport variants: pack / reduce store their encoded output into a table of destinations (peers'
// receive slots over xGMI), then release at system scope before the kernel retires.
template <typename TIN, int C>
__global__ void __launch_bounds__(kBlock) wire_pack_to_kernel(const TIN* __restrict__ in, WirePtrs dst, size_t n_s,
                                                             int n_shards, int rel) {
  const size_t tasks = n_s >> 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (int s = 0; s < n_shards; ++s) {
    uint8_t* d = dst.p[s];
    if (d == nullptr) continue;
    const TIN* src = in + (size_t)s * n_s;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
      float v[16];
      DenseLane16<TIN>::load16(src, t << 4, v);
      WireLane16<C>::store16(d, n_s, t << 4, v);
    }
  }
  p2p_release(rel);
}

template <typename TL, int C>
__global__ void __launch_bounds__(kBlock)
    wire_reduce_to_kernel(const uint8_t* __restrict__ slots, size_t slot_stride, int n_slots, int self_pos,
                          const TL* __restrict__ local, WirePtrs dst, int n_dst, size_t n_s, int rel) {
  const size_t tasks = n_s >> 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
    const size_t le = t << 4;
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
    for (int r = 0; r < n_slots; ++r) {
      float v[16];
      if (r == self_pos) DenseLane16<TL>::load16(local, le, v);
      else WireLane16<C>::load16(slots + (size_t)r * slot_stride, n_s, le, v);
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] += v[j];
    }
    for (int i = 0; i < n_dst; ++i)  // wave-uniform condition: every lane of a 16-lane segment stores
      if (dst.p[i] != nullptr) WireLane16<C>::store16(dst.p[i], n_s, le, acc);
  }
  p2p_release(rel);
}

// wire_reduce_to_kernel for the BFP codecs, lane-contiguous (as wire_reduce_sgd4_kernel below): 4 values per lane, 4
// lanes a group, the group exponent from quad xor shuffles; each destination gets the lane's 4 mantissa bytes as one
// dword and the group's exponent byte from its first lane. The same sums in slot order and the same encoding:
// bit-identical (FAN_WIRE_REDUCE4).
template <typename TL, int C>
__global__ void __launch_bounds__(kBlock)
    wire_reduce_to4_kernel(const uint8_t* __restrict__ slots, size_t slot_stride, int n_slots, int self_pos,
                           const TL* __restrict__ local, WirePtrs dst, int n_dst, size_t n_s, int rel) {
  static_assert(C == kBfpTrunc || C == kBfpRne, "BFP codecs");
  const size_t tasks = n_s >> 2;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
    const size_t le = t << 2;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < n_slots; ++r) {
      float v[4];
      if (r == self_pos) {
        if constexpr (sizeof(TL) == 4) {
          const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(local) + le);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        } else {
          const uint2 a = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(local) + le);
          v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xFFFF0000u);
          v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xFFFF0000u);
        }
      } else {
        const uint8_t* sh = slots + (size_t)r * slot_stride;
        const uint32_t m = *reinterpret_cast<const uint32_t*>(sh + le);
        const uint32_t E = sh[n_s + (le >> 4)];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int32_t q = (int32_t)(int8_t)(uint8_t)(m >> (8 * j));
          v[j] = (C == kBfpTrunc) ? bfp_decode_trunc(q, E) : bfp_decode_rne(q, E);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += v[j];
    }
    uint32_t mx = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) mx = max(mx, __float_as_uint(acc[j]) & 0x7FFFFFFFu);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, 1));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, 2));
    const uint32_t E = mx >> 23;
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t q = (C == kBfpTrunc) ? bfp_encode_trunc(__float_as_uint(acc[j]), E) : bfp_encode_rne(acc[j], E);
      w |= ((uint32_t)q & 0xFFu) << (8 * j);
    }
    for (int i = 0; i < n_dst; ++i) {  // wave-uniform condition
      uint8_t* d = dst.p[i];
      if (d == nullptr) continue;
      *reinterpret_cast<uint32_t*>(d + le) = w;
      if ((le & 15) == 0) d[n_s + (le >> 4)] = (uint8_t)E;
    }
  }
  p2p_release(rel);
}

// The value a rank decodes after the owner re-encodes `v` (one 16-value group) with codec C.
template <int C>
__device__ __forceinline__ void codec_roundtrip16(float v[16]) {
  if constexpr (C == kBfpTrunc || C == kBfpRne) {
    uint32_t mx = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) mx = max(mx, __float_as_uint(v[j]) & 0x7FFFFFFFu);
    const uint32_t E = mx >> 23;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int32_t q = (C == kBfpTrunc) ? bfp_encode_trunc(__float_as_uint(v[j]), E) : bfp_encode_rne(v[j], E);
      const int32_t q8 = (int32_t)(int8_t)(uint8_t)((uint32_t)q & 0xFFu);  // the stored byte, as the decoder reads it
      v[j] = (C == kBfpTrunc) ? bfp_decode_trunc(q8, E) : bfp_decode_rne(q8, E);
    }
  } else if constexpr (C == kRawBf16) {
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const uint32_t u = pack_bf16x2(v[j], v[j + 1]);
      v[j] = __uint_as_float(u << 16);
      v[j + 1] = __uint_as_float(u & 0xFFFF0000u);
    }
  }
}

template <typename TL, int C, bool HAS_MOM>
__global__ void __launch_bounds__(kBlock)
    wire_reduce_sgd_kernel(const uint8_t* __restrict__ slots, size_t slot_stride, int n_slots, int self_pos,
                           const TL* __restrict__ local, float* __restrict__ master, float* __restrict__ mom,
                           SgdParams p, size_t n_valid, WirePtrs dst, int n_dst, size_t n_s, int rel) {
  const size_t tasks = n_s >> 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
    const size_t le = t << 4;
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
    for (int r = 0; r < n_slots; ++r) {
      float v[16];
      if (r == self_pos) DenseLane16<TL>::load16(local, le, v);
      else WireLane16<C>::load16(slots + (size_t)r * slot_stride, n_s, le, v);
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] += v[j];
    }
    codec_roundtrip16<C>(acc);
    float w[16], m[16];
    DenseLane16<float>::load16(master, le, w);
    if (HAS_MOM) DenseLane16<float>::load16(mom, le, m);
#pragma unroll
    for (int j = 0; j < 16; ++j) {  // wire_sgd_kernel's operations, in its order
      if (le + j >= n_valid) continue;
      float gj = acc[j] * p.grad_scale;
      if (p.weight_decay != 0.0f) gj = fmaf(p.weight_decay, w[j], gj);
      if (HAS_MOM) {
        m[j] = fmaf(p.momentum, m[j], gj);
        gj = p.nesterov ? fmaf(p.momentum, m[j], gj) : m[j];
      }
      w[j] = fmaf(-p.lr, gj, w[j]);
    }
    if (le < n_valid) {
      DenseLane16<float>::store16(master, le, w);
      if (HAS_MOM) DenseLane16<float>::store16(mom, le, m);
    }
    for (int i = 0; i < n_dst; ++i)
      if (dst.p[i] != nullptr) DenseLane16<bf16_t>::store16(reinterpret_cast<bf16_t*>(dst.p[i]), le, w);
  }
  if (rel >= 0) p2p_release(rel);
}

// wire_reduce_sgd_kernel for the BFP codecs, lane-contiguous: 4 consecutive values per lane, 4 lanes a 16-value group
// (the group's exponent for the codec round trip from quad xor shuffles: exact), so every load and store of a wave
// covers contiguous bytes instead of striding a group per lane — the same sums in slot order, the same round trip and
// SGD per value: bit-identical (FAN_WIRE_REDUCE4, default on). n_s is a multiple of 16 and the grid's thread count a
// multiple of 4, so a quad's lanes are always all in or all out of range.
template <typename TL, int C, bool HAS_MOM>
__global__ void __launch_bounds__(kBlock)
    wire_reduce_sgd4_kernel(const uint8_t* __restrict__ slots, size_t slot_stride, int n_slots, int self_pos,
                            const TL* __restrict__ local, float* __restrict__ master, float* __restrict__ mom,
                            SgdParams p, size_t n_valid, WirePtrs dst, int n_dst, size_t n_s, int rel) {
  static_assert(C == kBfpTrunc || C == kBfpRne, "BFP codecs");
  const size_t tasks = n_s >> 2;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
    const size_t le = t << 2;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < n_slots; ++r) {
      float v[4];
      if (r == self_pos) {
        if constexpr (sizeof(TL) == 4) {
          const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(local) + le);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        } else {
          const uint2 a = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(local) + le);
          v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xFFFF0000u);
          v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xFFFF0000u);
        }
      } else {
        const uint8_t* sh = slots + (size_t)r * slot_stride;
        const uint32_t m = *reinterpret_cast<const uint32_t*>(sh + le);
        const uint32_t E = sh[n_s + (le >> 4)];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int32_t q = (int32_t)(int8_t)(uint8_t)(m >> (8 * j));
          v[j] = (C == kBfpTrunc) ? bfp_decode_trunc(q, E) : bfp_decode_rne(q, E);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += v[j];
    }
    // codec_roundtrip16 on the quad's group
    uint32_t mx = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) mx = max(mx, __float_as_uint(acc[j]) & 0x7FFFFFFFu);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, 1));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, 2));
    const uint32_t E = mx >> 23;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t q = (C == kBfpTrunc) ? bfp_encode_trunc(__float_as_uint(acc[j]), E) : bfp_encode_rne(acc[j], E);
      const int32_t q8 = (int32_t)(int8_t)(uint8_t)((uint32_t)q & 0xFFu);
      acc[j] = (C == kBfpTrunc) ? bfp_decode_trunc(q8, E) : bfp_decode_rne(q8, E);
    }
    float4 wv = *reinterpret_cast<const float4*>(master + le);
    float w[4] = {wv.x, wv.y, wv.z, wv.w}, m[4] = {0.f, 0.f, 0.f, 0.f};
    if (HAS_MOM) {
      const float4 mv = *reinterpret_cast<const float4*>(mom + le);
      m[0] = mv.x; m[1] = mv.y; m[2] = mv.z; m[3] = mv.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // wire_sgd_kernel's operations, in its order
      if (le + j >= n_valid) continue;
      float gj = acc[j] * p.grad_scale;
      if (p.weight_decay != 0.0f) gj = fmaf(p.weight_decay, w[j], gj);
      if (HAS_MOM) {
        m[j] = fmaf(p.momentum, m[j], gj);
        gj = p.nesterov ? fmaf(p.momentum, m[j], gj) : m[j];
      }
      w[j] = fmaf(-p.lr, gj, w[j]);
    }
    if (le < n_valid) {
      *reinterpret_cast<float4*>(master + le) = make_float4(w[0], w[1], w[2], w[3]);
      if (HAS_MOM) *reinterpret_cast<float4*>(mom + le) = make_float4(m[0], m[1], m[2], m[3]);
    }
    const uint2 lp = make_uint2(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]));
    for (int i = 0; i < n_dst; ++i)
      if (dst.p[i] != nullptr) *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(dst.p[i]) + le) = lp;
  }
  if (rel >= 0) p2p_release(rel);
}

template <typename TOUT, int C>
__global__ void __launch_bounds__(kBlock) wire_unpack_strided_kernel(const uint8_t* __restrict__ in,
                                                                    size_t shard_stride, TOUT* __restrict__ out,
                                                                    size_t n_s, int n_shards) {
  const size_t tasks = n_s >> 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (int s = 0; s < n_shards; ++s) {
    const uint8_t* src = in + (size_t)s * shard_stride;
    TOUT* dst = out + (size_t)s * n_s;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
      float v[16];
      WireLane16<C>::load16(src, n_s, t << 4, v);
      DenseLane16<TOUT>::store16(dst, t << 4, v);
    }
  }
}

template <int C, bool HAS_LP, bool HAS_MOM>
__global__ void __launch_bounds__(kBlock)
    wire_sgd_kernel(const uint8_t* __restrict__ wire, size_t n_s, int n_shards, int skip_shard, int skip_period,
                    float* __restrict__ master, bf16_t* __restrict__ lp, float* __restrict__ mom, SgdParams p,
                    size_t n_valid, size_t sb) {
  // 8 elements per lane here (a read-only wire: the 16-per-lane store layout buys nothing, and the smaller
  // register footprint streams master / lp faster: 33.5 vs 42.5 us on a 16.8 M bucket in the flagship step)
  const size_t tasks = n_s >> 3;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (int s = 0; s < n_shards; ++s) {
    if (skip_shard >= 0 && (s % skip_period) == skip_shard) continue;
    const uint8_t* src = wire + (size_t)s * sb;
    const size_t base = (size_t)s * n_s;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tasks; t += stride) {
      const size_t e = base + (t << 3);
      if (e >= n_valid) continue;
      float g[8], w[8];
      WireLane<C>::load8(src, n_s, t << 3, g);
      DenseLane<float>::load8(master, e, w);
      float m[8];
      if (HAS_MOM) DenseLane<float>::load8(mom, e, m);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float gj = g[j] * p.grad_scale;
        if (p.weight_decay != 0.0f) gj = fmaf(p.weight_decay, w[j], gj);
        if (HAS_MOM) {
          m[j] = fmaf(p.momentum, m[j], gj);
          gj = p.nesterov ? fmaf(p.momentum, m[j], gj) : m[j];
        }
        w[j] = fmaf(-p.lr, gj, w[j]);
      }
      const bool full = e + 8 <= n_valid;
      if (full) {
        DenseLane<float>::store8(master, e, w);
        if (HAS_MOM) DenseLane<float>::store8(mom, e, m);
        if (HAS_LP) DenseLane<bf16_t>::store8(lp, e, w);
      } else {
        for (int j = 0; j < 8 && e + j < n_valid; ++j) {
          master[e + j] = w[j];
          if (HAS_MOM) mom[e + j] = m[j];
          if (HAS_LP) lp[e + j] = f32_to_bf16(w[j]);
        }
      }
    }
  }
}

}  // namespace

#define FAN_CODEC_SWITCH(codec, ...)                         \
  switch (codec) {                                           \
    case kBfpTrunc: { constexpr int C = kBfpTrunc; __VA_ARGS__; break; } \
    case kBfpRne: { constexpr int C = kBfpRne; __VA_ARGS__; break; }     \
    case kRawF32: { constexpr int C = kRawF32; __VA_ARGS__; break; }     \
    case kRawBf16: { constexpr int C = kRawBf16; __VA_ARGS__; break; }   \
    default: FAN_CHECK(false, "unknown codec");              \
  }

static void check_ns(size_t n_s) {
  FAN_CHECK(n_s % 256 == 0, "shard element count must be a multiple of 256");
}

void launch_wire_pack(int codec, int in_dtype, const void* in, void* out, size_t n_s, int n_shards,
                      hipStream_t stream) {
  check_ns(n_s);
  if (n_s == 0 || n_shards == 0) return;
  const int grid = stream_grid(n_s / 16, kBlock, wire_max_blocks());
  FAN_CODEC_SWITCH(codec, {
    if (in_dtype == kF32)
      hipLaunchKernelGGL((wire_pack_kernel<float, C>), grid, kBlock, 0, stream, (const float*)in, (uint8_t*)out,
                         n_s, n_shards);
    else
      hipLaunchKernelGGL((wire_pack_kernel<bf16_t, C>), grid, kBlock, 0, stream, (const bf16_t*)in,
                         (uint8_t*)out, n_s, n_shards);
  });
  FAN_HIP_CHECK(hipGetLastError());
}

void launch_wire_pack_range(int codec, int in_dtype, const void* in, void* out, size_t n_s, size_t begin,
                            size_t end, hipStream_t stream) {
  check_ns(n_s);
  FAN_CHECK(begin % 16 == 0 && end % 16 == 0 && begin <= end, "pack_range: bounds must be multiples of 16");
  if (end == begin) return;
  const int grid = stream_grid((end - begin) / 8, kBlock, wire_max_blocks());
  FAN_CODEC_SWITCH(codec, {
    if (in_dtype == kF32)
      hipLaunchKernelGGL((wire_pack_range_kernel<float, C>), grid, kBlock, 0, stream, (const float*)in,
                         (uint8_t*)out, n_s, begin, end);
    else
      hipLaunchKernelGGL((wire_pack_range_kernel<bf16_t, C>), grid, kBlock, 0, stream, (const bf16_t*)in,
                         (uint8_t*)out, n_s, begin, end);
  });
  FAN_HIP_CHECK(hipGetLastError());
}

void launch_wire_unpack(int codec, int out_dtype, const void* in, void* out, size_t n_s, int n_shards,
                        hipStream_t stream) {
  check_ns(n_s);
  if (n_s == 0 || n_shards == 0) return;
  const int grid = stream_grid(n_s / 16, kBlock, wire_max_blocks());
  FAN_CODEC_SWITCH(codec, {
    if (out_dtype == kF32)
      hipLaunchKernelGGL((wire_unpack_kernel<float, C>), grid, kBlock, 0, stream, (const uint8_t*)in, (float*)out,
                         n_s, n_shards);
    else
      hipLaunchKernelGGL((wire_unpack_kernel<bf16_t, C>), grid, kBlock, 0, stream, (const uint8_t*)in,
                         (bf16_t*)out, n_s, n_shards);
  });
  FAN_HIP_CHECK(hipGetLastError());
}

template <typename TL, int C>
static void reduce_dispatch(const void* slots, size_t slot_stride, int n_slots, int self_pos, const void* local,
                            void* out_wire, float* out_f32, size_t n_s, hipStream_t stream) {
  const bool q4 = (C == kBfpTrunc || C == kBfpRne) && wire_reduce4_for(n_slots);
  const int grid = stream_grid(q4 ? n_s / 4 : n_s / 16, kBlock, wire_max_blocks());
  const uint8_t* sl = (const uint8_t*)slots;
  const TL* lo = (const TL*)local;
  uint8_t* ow = (uint8_t*)out_wire;
#define FAN_RED(HL, OW, OF)                                                                                    \
  do {                                                                                                         \
    if constexpr (C == kBfpTrunc || C == kBfpRne) {                                                            \
      if (q4) {                                                                                                \
        hipLaunchKernelGGL((wire_reduce4_kernel<TL, C, HL, OW, OF>), grid, kBlock, 0, stream, sl, slot_stride, \
                           n_slots, self_pos, lo, ow, out_f32, n_s);                                           \
        break;                                                                                                 \
      }                                                                                                        \
    }                                                                                                          \
    hipLaunchKernelGGL((wire_reduce_kernel<TL, C, HL, OW, OF>), grid, kBlock, 0, stream, sl, slot_stride,      \
                       n_slots, self_pos, lo, ow, out_f32, n_s);                                               \
  } while (0)
  const bool hl = local != nullptr, w = out_wire != nullptr, f = out_f32 != nullptr;
  FAN_CHECK(w || f, "wire_reduce needs an output");
  if (hl) {
    if (w && f) FAN_RED(true, true, true);
    else if (w) FAN_RED(true, true, false);
    else FAN_RED(true, false, true);
  } else {
    if (w && f) FAN_RED(false, true, true);
    else if (w) FAN_RED(false, true, false);
    else FAN_RED(false, false, true);
  }
#undef FAN_RED
}

void launch_wire_reduce(int codec, int local_dtype, const void* slots, size_t slot_stride, int n_slots,
                        int self_pos, const void* local, void* out_wire, float* out_f32, size_t n_s,
                        hipStream_t stream) {
  check_ns(n_s);
  if (n_s == 0) return;
  FAN_CODEC_SWITCH(codec, {
    if (local_dtype == kF32)
      reduce_dispatch<float, C>(slots, slot_stride, n_slots, self_pos, local, out_wire, out_f32, n_s, stream);
    else
      reduce_dispatch<bf16_t, C>(slots, slot_stride, n_slots, self_pos, local, out_wire, out_f32, n_s, stream);
  });
  FAN_HIP_CHECK(hipGetLastError());
}

void launch_wire_sgd(int codec, const void* wire, size_t n_s, int n_shards, int skip_shard, int skip_period,
                     float* master, bf16_t* lp, float* mom, SgdParams p, size_t n_valid, hipStream_t stream,
                     size_t shard_stride) {
  if (skip_period < 1) skip_period = 1 << 30;
  check_ns(n_s);
  if (n_s == 0 || n_shards == 0) return;
  const int grid = stream_grid(n_s / 8, kBlock, wire_max_blocks());
  const uint8_t* w = (const uint8_t*)wire;
  FAN_CODEC_SWITCH(codec, {
    const size_t sb = shard_stride ? shard_stride : wire_shard_bytes(C, n_s);
    if (lp && mom)
      hipLaunchKernelGGL((wire_sgd_kernel<C, true, true>), grid, kBlock, 0, stream, w, n_s, n_shards, skip_shard, skip_period,
                         master, lp, mom, p, n_valid, sb);
    else if (lp)
      hipLaunchKernelGGL((wire_sgd_kernel<C, true, false>), grid, kBlock, 0, stream, w, n_s, n_shards,
                         skip_shard, skip_period, master, lp, mom, p, n_valid, sb);
    else if (mom)
      hipLaunchKernelGGL((wire_sgd_kernel<C, false, true>), grid, kBlock, 0, stream, w, n_s, n_shards,
                         skip_shard, skip_period, master, lp, mom, p, n_valid, sb);
    else
      hipLaunchKernelGGL((wire_sgd_kernel<C, false, false>), grid, kBlock, 0, stream, w, n_s, n_shards,
                         skip_shard, skip_period, master, lp, mom, p, n_valid, sb);
  });
  FAN_HIP_CHECK(hipGetLastError());
}

void launch_wire_unpack_strided(int codec, int out_dtype, const void* in, size_t shard_stride, void* out, size_t n_s,
                                int n_shards, hipStream_t stream) {
  check_ns(n_s);
  if (n_s == 0 || n_shards == 0) return;
  const int grid = stream_grid(n_s / 16, kBlock, wire_max_blocks());
  FAN_CODEC_SWITCH(codec, {
    if (out_dtype == kF32)
      hipLaunchKernelGGL((wire_unpack_strided_kernel<float, C>), grid, kBlock, 0, stream, (const uint8_t*)in,
                         shard_stride, (float*)out, n_s, n_shards);
    else
      hipLaunchKernelGGL((wire_unpack_strided_kernel<bf16_t, C>), grid, kBlock, 0, stream, (const uint8_t*)in,
                         shard_stride, (bf16_t*)out, n_s, n_shards);
  });
  FAN_HIP_CHECK(hipGetLastError());
}

void launch_wire_pack_to(int codec, int in_dtype, const void* in, const WirePtrs& dst, size_t n_s, int n_shards,
                         hipStream_t stream) {
  check_ns(n_s);
  FAN_CHECK(n_shards <= kMaxPeers, "pack_to: at most 16 destinations");
  if (n_s == 0 || n_shards == 0) return;
  const int grid = stream_grid(n_s / 16, kBlock, std::min(wire_max_blocks(), p2p_grid_cap()));
  FAN_CODEC_SWITCH(codec, {
    if (in_dtype == kF32)
      hipLaunchKernelGGL((wire_pack_to_kernel<float, C>), grid, kBlock, 0, stream, (const float*)in, dst, n_s,
                         n_shards, p2p_release_mode());
    else
      hipLaunchKernelGGL((wire_pack_to_kernel<bf16_t, C>), grid, kBlock, 0, stream, (const bf16_t*)in, dst, n_s,
                         n_shards, p2p_release_mode());
  });
  FAN_HIP_CHECK(hipGetLastError());
}

// the lane-contiguous reduce-to-peers kernel for the BFP codecs (false: not launched — another codec, or the flag off)
template <int C>
static bool reduce_to4_dispatch(int grid4, int local_dtype, const void* slots, size_t slot_stride, int n_slots,
                                int self_pos, const void* local, const WirePtrs& dst, int n_dst, size_t n_s,
                                hipStream_t stream) {
  if constexpr (C == kBfpTrunc || C == kBfpRne) {
    if (grid4 <= 0) return false;
    if (local_dtype == kF32)
      hipLaunchKernelGGL((wire_reduce_to4_kernel<float, C>), grid4, kBlock, 0, stream, (const uint8_t*)slots,
                         slot_stride, n_slots, self_pos, (const float*)local, dst, n_dst, n_s, p2p_release_mode());
    else
      hipLaunchKernelGGL((wire_reduce_to4_kernel<bf16_t, C>), grid4, kBlock, 0, stream, (const uint8_t*)slots,
                         slot_stride, n_slots, self_pos, (const bf16_t*)local, dst, n_dst, n_s, p2p_release_mode());
    return true;
  } else {
    return false;
  }
}

void launch_wire_reduce_to(int codec, int local_dtype, const void* slots, size_t slot_stride, int n_slots, int self_pos,
                           const void* local, const WirePtrs& dst, int n_dst, size_t n_s, hipStream_t stream) {
  check_ns(n_s);
  FAN_CHECK(n_dst <= kMaxPeers && local != nullptr, "reduce_to: local operand and at most 16 destinations");
  if (n_s == 0) return;
  const int grid = stream_grid(n_s / 16, kBlock, std::min(wire_max_blocks(), p2p_grid_cap()));
  const int grid4 =
      wire_reduce4_for(n_slots) ? stream_grid(n_s / 4, kBlock, std::min(wire_max_blocks(), p2p_grid_cap())) : 0;
  FAN_CODEC_SWITCH(codec, {
    if (reduce_to4_dispatch<C>(grid4, local_dtype, slots, slot_stride, n_slots, self_pos, local, dst, n_dst, n_s,
                               stream)) {
      FAN_HIP_CHECK(hipGetLastError());
      return;
    }
    if (local_dtype == kF32)
      hipLaunchKernelGGL((wire_reduce_to_kernel<float, C>), grid, kBlock, 0, stream, (const uint8_t*)slots,
                         slot_stride, n_slots, self_pos, (const float*)local, dst, n_dst, n_s, p2p_release_mode());
    else
      hipLaunchKernelGGL((wire_reduce_to_kernel<bf16_t, C>), grid, kBlock, 0, stream, (const uint8_t*)slots,
                         slot_stride, n_slots, self_pos, (const bf16_t*)local, dst, n_dst, n_s, p2p_release_mode());
  });
  FAN_HIP_CHECK(hipGetLastError());
}

static std::atomic<int>& reduce4_flag() {
  static std::atomic<int> f{[] {
    const char* e = getenv("FAN_WIRE_REDUCE4");
    return e && e[0] == '0' ? 0 : 1;
  }()};
  return f;
}
void set_wire_reduce4(int on) { reduce4_flag().store(on); }
int wire_reduce4() { return reduce4_flag().load(std::memory_order_relaxed); }

template <int C>
static void reduce_sgd_dispatch(int local_dtype, int grid, const void* slots, size_t slot_stride, int n_slots,
                                int self_pos, const void* local, float* master, float* mom, SgdParams p,
                                size_t n_valid, const WirePtrs& dst, int n_dst, size_t n_s, int rel,
                                hipStream_t stream, int grid4) {
  const uint8_t* sl = (const uint8_t*)slots;
  if constexpr (C == kBfpTrunc || C == kBfpRne) {
    if (grid4 > 0) {
      if (local_dtype == kF32) {
        if (mom)
          hipLaunchKernelGGL((wire_reduce_sgd4_kernel<float, C, true>), grid4, kBlock, 0, stream, sl, slot_stride,
                             n_slots, self_pos, (const float*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
        else
          hipLaunchKernelGGL((wire_reduce_sgd4_kernel<float, C, false>), grid4, kBlock, 0, stream, sl, slot_stride,
                             n_slots, self_pos, (const float*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
      } else {
        if (mom)
          hipLaunchKernelGGL((wire_reduce_sgd4_kernel<bf16_t, C, true>), grid4, kBlock, 0, stream, sl, slot_stride,
                             n_slots, self_pos, (const bf16_t*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
        else
          hipLaunchKernelGGL((wire_reduce_sgd4_kernel<bf16_t, C, false>), grid4, kBlock, 0, stream, sl, slot_stride,
                             n_slots, self_pos, (const bf16_t*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
      }
      return;
    }
  }
  if (local_dtype == kF32) {
    if (mom)
      hipLaunchKernelGGL((wire_reduce_sgd_kernel<float, C, true>), grid, kBlock, 0, stream, sl, slot_stride, n_slots,
                         self_pos, (const float*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
    else
      hipLaunchKernelGGL((wire_reduce_sgd_kernel<float, C, false>), grid, kBlock, 0, stream, sl, slot_stride, n_slots,
                         self_pos, (const float*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
  } else {
    if (mom)
      hipLaunchKernelGGL((wire_reduce_sgd_kernel<bf16_t, C, true>), grid, kBlock, 0, stream, sl, slot_stride, n_slots,
                         self_pos, (const bf16_t*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
    else
      hipLaunchKernelGGL((wire_reduce_sgd_kernel<bf16_t, C, false>), grid, kBlock, 0, stream, sl, slot_stride,
                         n_slots, self_pos, (const bf16_t*)local, master, mom, p, n_valid, dst, n_dst, n_s, rel);
  }
}

void launch_wire_reduce_sgd(int codec, int local_dtype, const void* slots, size_t slot_stride, int n_slots,
                            int self_pos, const void* local, float* master, float* mom, SgdParams p, size_t n_valid,
                            const WirePtrs& dst, int n_dst, size_t n_s, bool peers, hipStream_t stream) {
  check_ns(n_s);
  FAN_CHECK(n_dst <= kMaxPeers && local != nullptr && master != nullptr,
            "reduce_sgd: local operand, master shard and at most 16 destinations");
  if (n_s == 0) return;
  const int cap = peers ? std::min(wire_max_blocks(), p2p_grid_cap()) : wire_max_blocks();
  const int grid = stream_grid(n_s / 16, kBlock, cap);
  const int grid4 = wire_reduce4_for(n_slots) ? stream_grid(n_s / 4, kBlock, cap) : 0;
  const int rel = peers ? p2p_release_mode() : -1;
  FAN_CODEC_SWITCH(codec, reduce_sgd_dispatch<C>(local_dtype, grid, slots, slot_stride, n_slots, self_pos, local,
                                                 master, mom, p, n_valid, dst, n_dst, n_s, rel, stream, grid4));
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace fan

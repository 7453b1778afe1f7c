// Block-floating-point (BFP) wire format and the other wire codecs of the all-reduce engine.
//
// Behavioural spec (derived from the reference RTL):
//   encode  hw/bf16_to_bfp_core.sv:97-126 (shared exp = max, right barrel shift of the 24-bit
//           mantissa with forced hidden 1, 25-bit two's complement, keep [24:1]),
//           hw/bfp_adapter.sv:145-154 (truncate to the top MANT_SIZE=8 bits -> floor),
//           hw/barrel_shifter.sv:44-51 (shift >= 32 clears).
//   decode  hw/bfp_to_bf16_core.sv:55-117 (|q| << 16, exp = E + 1 - lzc, normalise, bit0 = 0).
//
// CDNA4 mapping: one group of 16 values is handled by a PAIR of lanes (8 values each, 16-byte
// loads of bf16 / 2x16-byte of f32); the shared exponent is one v_max_u32 tree per lane plus a
// single DPP/swizzle exchange (__shfl_xor 1). No LDS round trip, no cross-wave traffic.
//
// Packed layout of one shard of n_s elements (n_s % 256 == 0): [int8 mant[n_s]][uint8 exp[n_s/16]]
// (the SoA analogue of the reference's 16 mantissa flits + 1 exponent flit per 32 groups,
// hw/bfp_adapter.sv:279-379). A multi-shard buffer is shards back to back.
#pragma once
#include "common/hip_common.h"

namespace fan {

enum Codec : int {
  kBfpTrunc = 0,  // bit-exact reference numerics (floor truncation, reference decode quirks)
  kBfpRne = 1,    // framework default: round-to-nearest-even, exact decode q * 2^(E-133)
  kRawF32 = 2,    // uncompressed fp32 on the wire
  kRawBf16 = 3,   // uncompressed bf16 on the wire
};

enum DType : int { kF32 = 0, kBF16 = 1 };

struct SgdParams {
  float lr;
  float grad_scale;
  float weight_decay;
  float momentum;
  int nesterov;
};

__host__ __device__ inline size_t wire_shard_bytes(int codec, size_t n_s) {
  switch (codec) {
    case kBfpTrunc:
    case kBfpRne: return n_s + n_s / 16;
    case kRawF32: return n_s * 4;
    default: return n_s * 2;
  }
}

// ---------------------------------------------------------------- scalar BFP primitives
// Reference (trunc) encode of one value given the group's shared exponent E.
__device__ __forceinline__ int32_t bfp_encode_trunc(uint32_t bits, uint32_t E) {
  const uint32_t e = (bits >> 23) & 0xFFu;
  const uint32_t m = (bits & 0x7FFFFFu) | 0x800000u;  // hidden 1 forced, even for 0/denormals
  const uint32_t d = E - e;
  const uint32_t a = d >= 32u ? 0u : (m >> d);         // VALU shifts are mod 32: clear explicitly
  const int32_t t = (bits >> 31) ? -(int32_t)a : (int32_t)a;
  return t >> 17;  // keep t[24:17] of the 25-bit two's complement: floor
}

// Reference decode (bit-level: q==0 -> 2^(E-150), |-128| = 128, exponent field wraps mod 256).
__device__ __forceinline__ float bfp_decode_trunc(int32_t q, uint32_t E) {
  const uint32_t sign = q < 0 ? 1u : 0u;
  const uint32_t M = (uint32_t)(q < 0 ? -q : q) << 16;  // 24-bit magnitude
  const uint32_t zc = __clz(M) - 8u;                     // 24-bit leading-zero count (24 for 0)
  const uint32_t ex = (E + 1u - zc) & 0xFFu;
  const uint32_t frac = (M << zc) & 0x7FFFFEu;           // bit 0 forced to 0
  return __uint_as_float((sign << 31) | (ex << 23) | frac);
}

// Framework encode: q = clamp(rne(x * 2^(133-E)), -127, 127).
__device__ __forceinline__ int32_t bfp_encode_rne(float x, uint32_t E) {
  float s = rintf(ldexpf(x, 133 - (int)E));
  s = fminf(fmaxf(s, -127.0f), 127.0f);
  return (int32_t)s;
}

__device__ __forceinline__ float bfp_decode_rne(int32_t q, uint32_t E) {
  return E == 255u ? __uint_as_float(0x7FC00000u) : ldexpf((float)q, (int)E - 133);
}

// ---------------------------------------------------------------- 8-value lane codecs
template <int C>
struct WireLane;

template <int C>
struct BfpLane {
  __device__ static __forceinline__ void load8(const uint8_t* shard, size_t n_s, size_t le, float v[8]) {
    const uint2 m = *reinterpret_cast<const uint2*>(shard + le);
    const uint32_t E = shard[n_s + (le >> 4)];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t w = j < 4 ? m.x : m.y;
      const int32_t q = (int32_t)(int8_t)(uint8_t)(w >> (8 * (j & 3)));
      v[j] = (C == kBfpTrunc) ? bfp_decode_trunc(q, E) : bfp_decode_rne(q, E);
    }
  }
  // Both lanes of the pair (lane, lane^1) must be active: they hold the two halves of a group.
  __device__ static __forceinline__ void store8(uint8_t* shard, size_t n_s, size_t le, const float v[8]) {
    uint32_t mx = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = max(mx, __float_as_uint(v[j]) & 0x7FFFFFFFu);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, 1));
    const uint32_t E = mx >> 23;
    uint32_t w[2] = {0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int32_t q = (C == kBfpTrunc) ? bfp_encode_trunc(__float_as_uint(v[j]), E) : bfp_encode_rne(v[j], E);
      w[j >> 2] |= ((uint32_t)q & 0xFFu) << (8 * (j & 3));
    }
    *reinterpret_cast<uint2*>(shard + le) = make_uint2(w[0], w[1]);
    if ((le & 15) == 0) shard[n_s + (le >> 4)] = (uint8_t)E;
  }
};

template <>
struct WireLane<kBfpTrunc> : BfpLane<kBfpTrunc> {};
template <>
struct WireLane<kBfpRne> : BfpLane<kBfpRne> {};

template <>
struct WireLane<kRawF32> {
  __device__ static __forceinline__ void load8(const uint8_t* shard, size_t, size_t le, float v[8]) {
    const float4* p = reinterpret_cast<const float4*>(shard) + (le >> 2);
    const float4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ static __forceinline__ void store8(uint8_t* shard, size_t, size_t le, const float v[8]) {
    float4* p = reinterpret_cast<float4*>(shard) + (le >> 2);
    p[0] = make_float4(v[0], v[1], v[2], v[3]);
    p[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <>
struct WireLane<kRawBf16> {
  __device__ static __forceinline__ void load8(const uint8_t* shard, size_t, size_t le, float v[8]) {
    const uint4 u = *(reinterpret_cast<const uint4*>(shard) + (le >> 3));
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
    }
  }
  __device__ static __forceinline__ void store8(uint8_t* shard, size_t, size_t le, const float v[8]) {
    uint4 u;
    u.x = pack_bf16x2(v[0], v[1]);
    u.y = pack_bf16x2(v[2], v[3]);
    u.z = pack_bf16x2(v[4], v[5]);
    u.w = pack_bf16x2(v[6], v[7]);
    *(reinterpret_cast<uint4*>(shard) + (le >> 3)) = u;
  }
};

// ---------------------------------------------------------------- 16-value lane codecs (one BFP group per lane)
// The streaming kernels give each lane a whole 16-value group: the shared exponent needs no cross-lane exchange,
// the mantissas leave as ONE 16-B store, and the 16 exponents of 16 consecutive lanes are gathered into ONE 16-B
// store by the group's first lane (the NIC ships the 32 exponents of a frame as one 256-bit flit,
// hw/bfp_adapter.sv:279-379). Every store of a wire shard is then a full 16-B vector store, which is what a store
// into a peer's uncached receive arena over xGMI needs (a byte store there is one fabric write per byte).
// Requirements: the 16 lanes 16k..16k+15 of a wave handle 16 consecutive groups starting at a multiple of 16
// (grid-stride loops over group indices with block and stride multiples of 16; n_s % 256 == 0, so a 16-lane
// segment is either entirely inside the shard or entirely past its end), and they are all active at the store.
template <int C>
struct WireLane16 {
  __device__ static __forceinline__ void load16(const uint8_t* shard, size_t n_s, size_t le, float v[16]) {
    WireLane<C>::load8(shard, n_s, le, v);
    WireLane<C>::load8(shard, n_s, le + 8, v + 8);
  }
  __device__ static __forceinline__ void store16(uint8_t* shard, size_t n_s, size_t le, const float v[16]) {
    WireLane<C>::store8(shard, n_s, le, v);
    WireLane<C>::store8(shard, n_s, le + 8, v + 8);
  }
};

template <int C>
struct BfpLane16 {
  __device__ static __forceinline__ void load16(const uint8_t* shard, size_t n_s, size_t le, float v[16]) {
    const uint4 m = *reinterpret_cast<const uint4*>(shard + le);
    const uint32_t E = shard[n_s + (le >> 4)];
    const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int32_t q = (int32_t)(int8_t)(uint8_t)(w[j >> 2] >> (8 * (j & 3)));
      v[j] = (C == kBfpTrunc) ? bfp_decode_trunc(q, E) : bfp_decode_rne(q, E);
    }
  }
  __device__ static __forceinline__ void store16(uint8_t* shard, size_t n_s, size_t le, const float v[16]) {
    uint32_t mx = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) mx = max(mx, __float_as_uint(v[j]) & 0x7FFFFFFFu);
    const uint32_t E = mx >> 23;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int32_t q = (C == kBfpTrunc) ? bfp_encode_trunc(__float_as_uint(v[j]), E) : bfp_encode_rne(v[j], E);
      w[j >> 2] |= ((uint32_t)q & 0xFFu) << (8 * (j & 3));
    }
    *reinterpret_cast<uint4*>(shard + le) = make_uint4(w[0], w[1], w[2], w[3]);
    // exponent plane: 4 lanes -> one dword, 4 dwords -> one 16-B store by lane 16k
    uint32_t e4 = E | ((uint32_t)__shfl_down((int)E, 1) << 8) | ((uint32_t)__shfl_down((int)E, 2) << 16) |
                  ((uint32_t)__shfl_down((int)E, 3) << 24);
    const uint32_t e4b = (uint32_t)__shfl_down((int)e4, 4), e4c = (uint32_t)__shfl_down((int)e4, 8),
                   e4d = (uint32_t)__shfl_down((int)e4, 12);
    if ((threadIdx.x & 15) == 0) *reinterpret_cast<uint4*>(shard + n_s + (le >> 4)) = make_uint4(e4, e4b, e4c, e4d);
  }
};

template <>
struct WireLane16<kBfpTrunc> : BfpLane16<kBfpTrunc> {};
template <>
struct WireLane16<kBfpRne> : BfpLane16<kBfpRne> {};

// Dense (local) operand loads: f32 or bf16 arrays.
template <typename T>
struct DenseLane;
template <>
struct DenseLane<float> {
  __device__ static __forceinline__ void load8(const float* p, size_t e, float v[8]) {
    WireLane<kRawF32>::load8(reinterpret_cast<const uint8_t*>(p), 0, e, v);
  }
  __device__ static __forceinline__ void store8(float* p, size_t e, const float v[8]) {
    WireLane<kRawF32>::store8(reinterpret_cast<uint8_t*>(p), 0, e, v);
  }
};
template <>
struct DenseLane<bf16_t> {
  __device__ static __forceinline__ void load8(const bf16_t* p, size_t e, float v[8]) {
    WireLane<kRawBf16>::load8(reinterpret_cast<const uint8_t*>(p), 0, e, v);
  }
  __device__ static __forceinline__ void store8(bf16_t* p, size_t e, const float v[8]) {
    WireLane<kRawBf16>::store8(reinterpret_cast<uint8_t*>(p), 0, e, v);
  }
};
template <typename T>
struct DenseLane16 {
  __device__ static __forceinline__ void load16(const T* p, size_t e, float v[16]) {
    DenseLane<T>::load8(p, e, v);
    DenseLane<T>::load8(p, e + 8, v + 8);
  }
  __device__ static __forceinline__ void store16(T* p, size_t e, const float v[16]) {
    DenseLane<T>::store8(p, e, v);
    DenseLane<T>::store8(p, e + 8, v + 8);
  }
};

// ---------------------------------------------------------------- release of stores into peer memory
// A kernel that stores into peers' receive arenas (direct P2P transport) must have every store performed before the
// stream-ordered flag write that tells the peer to read them (p2p_comm.h, memory ordering). Modes (FAN_P2P_RELEASE,
// settable at run time for A/B: p2p_release_mode()):
//   3 cp (default): nothing in the kernel; the transport records a system-scope release event
//     (hipEventReleaseToSystem) on the stream right before it writes the flags: ONE command-processor release
//     per round, ordered after every kernel of the round (2-rank flagship 2.25 vs 2.59 ms/step with "block",
//     profiles/r3_p2p_release_ab.txt);
//   1 block: every wave drains its own stores (s_waitcnt vmcnt(0)), the workgroup meets at a barrier,
//     then ONE lane issues the system-scope release (the valid form of MI355X_MICROARCH.md §Workgroup dispatch);
//   2 thread: every wave issues __threadfence_system() (the round-2 form: one system fence per wave, 4.9 ms/step);
//   0 none: rely on the end-of-kernel release alone (diagnostic only).
int p2p_release_mode();
void set_p2p_release_mode(int mode);
int p2p_grid_cap();  // workgroup cap of the peer-storing kernels (FAN_P2P_GRID)
void set_p2p_grid_cap(int blocks);

__device__ __forceinline__ void p2p_release(int mode) {
  if (mode == 2) {
    __threadfence_system();
  } else if (mode == 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep the wait after the write-back (compiler hazard)
    }
  }
}

// ---------------------------------------------------------------- host launchers
// Destination table of a kernel that stores its output straight into several buffers (the direct peer-to-peer
// transport: one entry per rank, each an IPC-mapped slot of that peer's receive arena; nullptr entries skipped).
constexpr int kMaxPeers = 16;
struct WirePtrs {
  uint8_t* p[kMaxPeers];
};

void launch_wire_pack(int codec, int in_dtype, const void* in, void* out, size_t n_s, int n_shards,
                      hipStream_t stream);
void launch_wire_unpack(int codec, int out_dtype, const void* in, void* out, size_t n_s, int n_shards,
                        hipStream_t stream);
// Pack flat elements [begin, end) (multiples of 16) into the shard layout (shards of n_s elements).
void launch_wire_pack_range(int codec, int in_dtype, const void* in, void* out, size_t n_s, size_t begin,
                            size_t end, hipStream_t stream);
// out = sum over slots (slot self_pos replaced by the dense local operand when given).
void launch_wire_reduce(int codec, int local_dtype, const void* slots, size_t slot_stride, int n_slots,
                        int self_pos, const void* local, void* out_wire, float* out_f32, size_t n_s,
                        hipStream_t stream);
// Fused all-gather epilogue: decode + SGD in place (master f32, optional bf16 copy, optional momentum).
// Shards s with (s % skip_period) == skip_shard are left untouched (skip_shard < 0: none).
// shard_stride: bytes between consecutive shards of `wire` (0: packed, wire_shard_bytes(codec, n_s)) — a gathered
// wire read in place from a receive arena has its shards one arena slot pair apart.
void launch_wire_sgd(int codec, const void* wire, size_t n_s, int n_shards, int skip_shard, int skip_period,
                     float* master, bf16_t* lp, float* mom, SgdParams p, size_t n_valid, hipStream_t stream,
                     size_t shard_stride = 0);
// Decode to f32/bf16 from a strided wire (as launch_wire_sgd's shard_stride).
void launch_wire_unpack_strided(int codec, int out_dtype, const void* in, size_t shard_stride, void* out, size_t n_s,
                                int n_shards, hipStream_t stream);
// Pack shards 0..n_shards-1 of `in`, shard s stored at dst.p[s] (skipped when nullptr); ends with a system-scope
// release so a peer may read the stores once the (stream-ordered) ready flag is set.
void launch_wire_pack_to(int codec, int in_dtype, const void* in, const WirePtrs& dst, size_t n_s, int n_shards,
                         hipStream_t stream);
// launch_wire_reduce whose encoded output is stored to every non-null dst.p[i] (i < n_dst), with a system-scope
// release at the end (the owner's reduced shard goes straight into every peer's receive slot).
void launch_wire_reduce_to(int codec, int local_dtype, const void* slots, size_t slot_stride, int n_slots, int self_pos,
                           const void* local, const WirePtrs& dst, int n_dst, size_t n_s, hipStream_t stream);
// Sharded update of the owner's shard (engine shard_update mode, ZeRO-1 style): sum the N received wire shards
// (slot self_pos replaced by the dense local operand), take the sum through the wire codec's round trip in registers
// (exactly the values every rank would decode from the re-encoded owner shard in the unsharded schedule), apply SGD to
// `master` / `mom` (this shard's planes; elements at or past n_valid keep their values) and write the updated
// weights in bf16 to every non-null dst.p[i] (i < n_dst: this rank's own copy and, on the direct P2P transport,
// every peer's receive slot), ending with the P2P release of `rel` (-1: none, a local output). Same arithmetic in
// the same order as wire_reduce (re-encode) + wire_sgd, so the weights are bit-identical to the unsharded schedule.
void launch_wire_reduce_sgd(int codec, int local_dtype, const void* slots, size_t slot_stride, int n_slots,
                            int self_pos, const void* local, float* master, float* mom, SgdParams p, size_t n_valid,
                            const WirePtrs& dst, int n_dst, size_t n_s, bool peers, hipStream_t stream);
// BFP codecs: the lane-contiguous form of that kernel, 4 values per lane (1, default) or one 16-value group per lane
// (0) (FAN_WIRE_REDUCE4); bit-identical either way
void set_wire_reduce4(int on);
int wire_reduce4();

}  // namespace fan

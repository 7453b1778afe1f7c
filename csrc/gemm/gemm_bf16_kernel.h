// bf16 MFMA GEMM for gfx950 (v_mfma_f32_16x16x32_bf16), LDS-tiled, global_load_lds staged.
//
// Structure (one workgroup = 8 waves = 512 threads; tile BM x BN x 64):
//   * operand tiles are staged global->LDS by global_load_lds_dwordx4 (no VGPR round trip) into an
//     S-deep LDS ring (S = 3 when it fits in 160 KiB, else 2). Each K-tile iteration does
//         s_waitcnt vmcnt(G*(S-2)) ; s_barrier ; issue stage kt+S-1 ; ds_read + MFMA on stage kt
//     i.e. ONE raw barrier per K-tile and a counted vmcnt that keeps the next stage's DMA in flight
//     across the barrier (never __syncthreads() in the loop: it would drain vmcnt to 0).
//   * K-contiguous operand image: [rows][64 k] (128-B rows), 16-B chunk c of row r at c ^ ((r>>1)&7):
//     ds_read_b128 fragment reads are bank-conflict-free.
//   * MN-contiguous operand image: 128-column halves, each [64 k][128] (256-B rows), 32-B block b of
//     row k at b ^ ((k&3) | ((k>>3)&1)<<2): ds_read_b64_tr_b16 (hardware transpose) reads are conflict-free.
//     glds writes LDS linearly, so every swizzle is applied to the per-lane GLOBAL source address and
//     mirrored on the read (one involution on both sides).
//   * waves are arranged WM x WN; each owns a (BM/WM) x (BN/WN) sub-tile of 16x16 MFMA tiles; MFMA
//     clusters run at s_setprio 1.
//   * workgroup -> tile map is XCD-aware (bijective): each of the 8 round-robin XCD groups gets a
//     contiguous run of tiles so neighbouring tiles share A rows in one L2.
//   * epilogue: accumulators are staged through LDS per 16-row block and written as coalesced 16-B
//     (f32) / 8-B (bf16) row segments, with bias / ReLU / ReLU-mask (bwd-data) / accumulate fused.
//   * split-K: K is split over workgroups, f32 partial slabs + an ordered (deterministic) reduce kernel
//     that applies the same epilogue.
//   * any M, N, K that are multiples of 8 (reference: libxsmm falls back to the whole dimension when MB or C does
//     not divide the blocking, sw/mlp_mpi_example_f32.cpp:498-506): tiles are ceil-divided; a workgroup whose
//     tile crosses an operand edge (a uniform flag) stages every out-of-range 16-B chunk from a zero page
//     (global_load_lds has no predicate, so the lane reads zeros instead), so the MFMAs accumulate exact zeros
//     there, and its epilogue stores only in-range elements. Interior tiles run the unpredicated path.
#pragma once
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "bfp/bfp_format.h"
#include "gemm/gemm.h"
#include "gemm/glds.h"

namespace fan {
namespace gemm_detail {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;

constexpr int BK = 64;
constexpr int kDefaultWaves = 8;

#ifdef FAN_GEMM_STAMPS
// Diagnostic build only (FAN_EXTRA_CFLAGS=-DFAN_GEMM_STAMPS): s_memtime stamps of the one-role loop for the first
// kStampWG workgroups, [wg][wave][kt][point]. One-role loop: 0 loop top, 1 after vmcnt, 2 after barrier, 3 after the
// DMA issue, 4 after the fragment reads are issued. Pipelined loop: 0 K-tile top, 1 k-step-0 block issued, 2 after
// the vmcnt/lgkmcnt wait, 3 after the barrier, 4 k-step-1 block issued. Never in a production build.
constexpr int kStampWG = 8, kStampKT = 64, kStampPts = 5;
#define FAN_STAMP(pt)                                                                                        \
  if (wo.stamps && blockIdx.x < kStampWG && kt < kStampKT && lane == 0)                                       \
  wo.stamps[(((size_t)blockIdx.x * 8 + wave) * kStampKT + kt) * kStampPts + (pt)] = __builtin_amdgcn_s_memtime()
#else
#define FAN_STAMP(pt)
#endif

__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// Zero page for the edge tiles' out-of-range operand chunks (one per code object; zero-initialised).
static __device__ __attribute__((aligned(256))) uint4 g_gemm_zero16[16];

__host__ __device__ constexpr int cdiv_i(int a, int b) { return (a + b - 1) / b; }

template <int OUTER, int NT>
struct OpTile {
  static constexpr int BYTES = OUTER * BK * 2;
  static constexpr int IB = NT * 16;              // bytes written by one block-wide glds instruction
  static constexpr int GLDS = BYTES / IB;         // glds instructions per thread per stage
  static constexpr int PER_HALF = (64 * 256) / IB;  // MN-contig: instructions per 128-column half
};

// Issue glds instruction i (of OpTile::GLDS) of one operand tile (outer extent OUTER from o0, k extent 64 from
// k0) with NT threads: this wave's 1 KiB piece of it. EDGE: chunks at outer >= o_lim or k >= k_lim (both
// multiples of 8, so a 16-B chunk is wholly in or out) load the zero page instead.
template <bool KCONTIG, int OUTER, int NT, bool EDGE = false>
__device__ __forceinline__ void stage_one(const bf16_t* __restrict__ g, int64_t ld, int o0, int k0, char* lds,
                                          int wave, int lane, int i, int o_lim = 0, int k_lim = 0) {
  using T = OpTile<OUTER, NT>;
  const int t = wave * 64 + lane;
  const bf16_t* src;
  bool out = false;
  if (KCONTIG) {
    const int row = i * (T::IB / 128) + (t >> 3);  // rows of 128 B
    const int c = (t & 7) ^ ((row >> 1) & 7);
    src = g + (int64_t)(o0 + row) * ld + k0 + c * 8;
    if (EDGE) out = o0 + row >= o_lim || k0 + c * 8 >= k_lim;
  } else {
    const int half = i / T::PER_HALF;                               // 128-column half
    const int krow = (i % T::PER_HALF) * (T::IB / 256) + (t >> 4);  // k-rows of 256 B
    const int cs = t & 15;
    const int blk = (cs >> 1) ^ mn_swz(krow);
    const int col = o0 + half * 128 + blk * 16 + (cs & 1) * 8;
    src = g + (int64_t)(k0 + krow) * ld + col;
    if (EDGE) out = k0 + krow >= k_lim || col >= o_lim;
  }
  if (EDGE && out) src = reinterpret_cast<const bf16_t*>(g_gemm_zero16);
  glds16((const void*)src, __builtin_amdgcn_readfirstlane(lds_addr_of(lds + i * T::IB + wave * 1024)));
}

// Stage one whole operand tile.
template <bool KCONTIG, int OUTER, int NT, bool EDGE = false>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ g, int64_t ld, int o0, int k0, char* lds,
                                           int wave, int lane, int o_lim = 0, int k_lim = 0) {
#pragma unroll
  for (int i = 0; i < OpTile<OUTER, NT>::GLDS; ++i)
    stage_one<KCONTIG, OUTER, NT, EDGE>(g, ld, o0, k0, lds, wave, lane, i, o_lim, k_lim);
}

template <bool KCONTIG>
__device__ __forceinline__ s16x8 read_frag(const char* lds, int o, int ks, int lane) {
  if (KCONTIG) {
    const int row = o + (lane & 15);
    const int chunk = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const s16x8*>(lds + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
  } else {
    const char* h = lds + (o >> 7) * (64 * 256);
    const int oo = o & 127;
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int kb = ks * 32 + 8 * (lane >> 4) + q;
    const int blk = oo >> 4;
    const int off0 = kb * 256 + ((blk ^ mn_swz(kb)) << 5) + 8 * p;
    const int off1 = (kb + 4) * 256 + ((blk ^ mn_swz(kb + 4)) << 5) + 8 * p;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(h + off0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(h + off1));
    s16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

// Sum of the 8 bf16 values of a fragment: 4 v_dot2c_f32_bf16 against (1, 1) (products exact, f32 accumulate)
// instead of 8 conversions + 8 adds — the fused bias gradient's VALU cost beside the MFMAs.
__device__ __forceinline__ float frag_sum(const s16x8& f) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const s16x2 p = {f[2 * e], f[2 * e + 1]};
    s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, p), one, s, false);
  }
  return s;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % kNumXCD;
  const int q = nwg / kNumXCD, r = nwg % kNumXCD;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / kNumXCD;
}

template <typename TC>
struct Out;
template <>
struct Out<float> {
  __device__ static __forceinline__ void load4(const float* p, float v[4]) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  __device__ static __forceinline__ void store4(float* p, const float v[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <>
struct Out<bf16_t> {
  __device__ static __forceinline__ void load4(const bf16_t* p, float v[4]) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xFFFF0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xFFFF0000u);
  }
  __device__ static __forceinline__ void store4(bf16_t* p, const float v[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  }
};

template <int EPI, typename TC, bool ACCUM>
__device__ __forceinline__ void epi4(float v[4], TC* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ bias,
                                     const TC* __restrict__ aux, int64_t ldaux, int row, int col) {
  if (EPI == kEpiBias || EPI == kEpiBiasRelu) {
    const uint2 u = *reinterpret_cast<const uint2*>(bias + col);
    v[0] += __uint_as_float(u.x << 16); v[1] += __uint_as_float(u.x & 0xFFFF0000u);
    v[2] += __uint_as_float(u.y << 16); v[3] += __uint_as_float(u.y & 0xFFFF0000u);
  }
  if (EPI == kEpiBiasRelu) {
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = fmaxf(v[u], 0.f);
  }
  if (EPI == kEpiReluMask) {
    float m[4];
    Out<TC>::load4(aux + (int64_t)row * ldaux + col, m);
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = m[u] > 0.f ? v[u] : 0.f;
  }
  TC* p = C + (int64_t)row * ldc + col;
  if (ACCUM) {
    float o[4];
    Out<TC>::load4(p, o);
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] += o[u];
  }
  Out<TC>::store4(p, v);
}

// epi4 for 8 bf16 outputs C(row, col..col+7): one 16-B store per lane (and 16-B bias / activation loads). The
// epilogue of a 256x256 bf16 tile is store-ISSUE-bound (MI355X_MICROARCH.md per-instruction table: a dwordx2 store
// tail runs at about half the rate of dwordx4), so the bf16 outputs are written 8 columns per lane. Same
// arithmetic, element for element, as epi4.
// 16-B store that writes through the XCD's L2 (sc1): the bytes are in memory once the storing wave's vmcnt reaches
// zero, so a workgroup on another XCD can read them after a counter hand-off with no release fence (the layer-chain
// GEMM's producer stages; MI355X_MICROARCH.md § visibility, publish-large: write-through beats plain stores + a
// release fence for tens of KB per workgroup). Not tracked by the compiler: every wait on it is an explicit vmcnt.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_wt16(void* p, const uint4& o) {
  const u32x4_t v = {o.x, o.y, o.z, o.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int EPI, bool ACCUM, bool WT = false>
__device__ __forceinline__ void epi8_bf16(float v[8], bf16_t* __restrict__ C, int64_t ldc,
                                          const bf16_t* __restrict__ bias, const uint4* mask, int row, int col) {
  auto lo = [](uint32_t u) { return __uint_as_float(u << 16); };
  auto hi = [](uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); };
  if (EPI == kEpiBias || EPI == kEpiBiasRelu) {
    const uint4 u = *reinterpret_cast<const uint4*>(bias + col);
    v[0] += lo(u.x); v[1] += hi(u.x); v[2] += lo(u.y); v[3] += hi(u.y);
    v[4] += lo(u.z); v[5] += hi(u.z); v[6] += lo(u.w); v[7] += hi(u.w);
  }
  if (EPI == kEpiBiasRelu) {
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = fmaxf(v[u], 0.f);
  }
  if (EPI == kEpiReluMask) {
    const uint4 m = *mask;
    const float mv[8] = {lo(m.x), hi(m.x), lo(m.y), hi(m.y), lo(m.z), hi(m.z), lo(m.w), hi(m.w)};
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = mv[u] > 0.f ? v[u] : 0.f;
  }
  bf16_t* p = C + (int64_t)row * ldc + col;
  if (ACCUM) {
    const uint4 o = *reinterpret_cast<const uint4*>(p);
    v[0] += lo(o.x); v[1] += hi(o.x); v[2] += lo(o.y); v[3] += hi(o.y);
    v[4] += lo(o.z); v[5] += hi(o.z); v[6] += lo(o.w); v[7] += hi(o.w);
  }
  const uint4 o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                             pack_bf16x2(v[6], v[7]));
  if constexpr (WT) store_wt16(p, o);
  else *reinterpret_cast<uint4*>(p) = o;
}

// kEpiWire target (GemmArgs::wire*): passed by value as one kernel argument.
struct WireOut {
  uint8_t* p;
  int64_t shard;  // elements per shard (multiple of 256)
  int own;        // shard also written to C in f32 (-1: none; kWireOwnAll: every shard, e.g. the ring's inputs)
  int period;     // > 0: shards s with s % period == own are all written (chunked buckets: one owner shard per chunk)
  int codec;      // kBfpTrunc / kBfpRne
  float inv_shard;  // 1 / shard (shard index without a 64-bit integer division)
  int bias_off;     // > 0: flat offset of the bias segment, encoded from the fused column sum
  // Fused local update (single-rank engine: the all-reduce of one rank is the identity): um != nullptr replaces the
  // wire stores by the SGD update of the bucket in place — each 16-value group takes its BFP round trip in registers
  // (encode -> decode: exactly the values the one-rank all-reduce hands its decode + SGD epilogue) and updates
  // master (f32), lp (bf16 copy) and mom at the same flat indices. The NIC's weight-update unit consumes the
  // all-reduce output stream the same way, without a round trip through host memory (hw/weight_update.sv:433-452).
  float* um;
  bf16_t* ulp;
  float* umom;
  SgdParams up;
#ifdef FAN_GEMM_STAMPS
  unsigned long long* stamps;  // diagnostic builds: s_memtime stamp buffer (see FAN_STAMP)
#endif
  // flat bucket index of C(0, 0) (GemmArgs::wire_off): a weight matrix that is not the first tensor of its bucket
  // (a transformer layer's bucket holds several; bench/bert_overlap.py). bias_off is absolute (includes it).
  uint32_t off;
  // > 0: the 4-wave persistent loops run their waves at this s_setprio level (gemm_prio_flag): a kernel of another
  // stream sharing the CU (the all-reduce's copy / reduce / SGD kernels) then issues only in the GEMM wave's stalls
  int prio;
};

// flat index -> (shard, position); f < 2^31, shard >= 256: the float estimate is off by at most one
__device__ __forceinline__ int wire_shard_of(uint32_t f, const WireOut& wo) {
  int sh = (int)((float)f * wo.inv_shard);
  const uint32_t sz = (uint32_t)wo.shard;
  if ((uint32_t)sh * sz > f) --sh;
  else if ((uint32_t)(sh + 1) * sz <= f) ++sh;
  return sh;
}

__device__ __forceinline__ uint8_t* wire_shard_base(int sh, const WireOut& wo) {
  return wo.p + (int64_t)sh * (wo.shard + wo.shard / 16);
}

__device__ __forceinline__ int32_t wire_encode(float x, uint32_t E, int codec) {
  return codec == kBfpTrunc ? bfp_encode_trunc(__float_as_uint(x), E) : bfp_encode_rne(x, E);
}

// BFP round trip of one value of a group with shared exponent E, as the single-rank all-reduce delivers it to its
// decode + SGD epilogue (framework codec only: the fused update is built for rne — with both codecs' branches the
// epilogue grows past the unroller's limit and the accumulator array lands in scratch memory).
__device__ __forceinline__ float wire_roundtrip_rne(float x, uint32_t E) {
  return bfp_decode_rne(bfp_encode_rne(x, E), E);  // |q| <= 127: the stored byte decodes to q
}

// One element of the fused update: the same operations, in the same order, as wire_sgd_kernel (bfp_kernels.hip), so
// the fused and the unfused single-rank step produce bit-identical weights.
__device__ __forceinline__ float sgd_apply(float g, float& w, float& m, bool has_mom, const SgdParams& p) {
  float gj = g * p.grad_scale;
  if (p.weight_decay != 0.0f) gj = fmaf(p.weight_decay, w, gj);
  if (has_mom) {
    m = fmaf(p.momentum, m, gj);
    gj = p.nesterov ? fmaf(p.momentum, m, gj) : m;
  }
  w = fmaf(-p.lr, gj, w);
  return w;
}

// Fused update of the 16-value group at flat index f (shared exponent E already computed): 16-B master / mom
// loads and stores, one 32-B bf16 store.
// (PRE: the group's master values w[] were loaded ahead by the caller)
template <bool PRE = false>
__device__ __forceinline__ void local_update16(const float v[16], uint32_t E, uint32_t f, const WireOut& wo,
                                               float (&w)[16]) {
  float m[16];
  if constexpr (!PRE) {
#pragma unroll
    for (int u = 0; u < 16; u += 4) {
      const float4 a = *reinterpret_cast<const float4*>(wo.um + f + u);
      w[u] = a.x; w[u + 1] = a.y; w[u + 2] = a.z; w[u + 3] = a.w;
    }
  }
  const bool hm = wo.umom != nullptr;
  if (hm) {
#pragma unroll
    for (int u = 0; u < 16; u += 4) {
      const float4 a = *reinterpret_cast<const float4*>(wo.umom + f + u);
      m[u] = a.x; m[u + 1] = a.y; m[u + 2] = a.z; m[u + 3] = a.w;
    }
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) sgd_apply(wire_roundtrip_rne(v[u], E), w[u], m[u], hm, wo.up);
#pragma unroll
  for (int u = 0; u < 16; u += 4) {
    *reinterpret_cast<float4*>(wo.um + f + u) = make_float4(w[u], w[u + 1], w[u + 2], w[u + 3]);
    if (hm) *reinterpret_cast<float4*>(wo.umom + f + u) = make_float4(m[u], m[u + 1], m[u + 2], m[u + 3]);
  }
  if (wo.ulp) {
    uint4* d = reinterpret_cast<uint4*>(wo.ulp + f);
    d[0] = make_uint4(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]), pack_bf16x2(w[4], w[5]),
                      pack_bf16x2(w[6], w[7]));
    d[1] = make_uint4(pack_bf16x2(w[8], w[9]), pack_bf16x2(w[10], w[11]), pack_bf16x2(w[12], w[13]),
                      pack_bf16x2(w[14], w[15]));
  }
}

// Encode the 16-value group at flat bucket index f (f % 16 == 0) held by this lane: 16-B mantissa store +
// 1 exponent byte (or, with the fused local update, the update of the group in place). Returns the shard it
// landed in (-1: updated in place).
template <bool UPD = false, bool PRE = false>
__device__ __forceinline__ int wire_store16(const float v[16], uint32_t f, const WireOut& wo, float (&wm)[16]) {
  uint32_t mx = 0;
#pragma unroll
  for (int u = 0; u < 16; ++u) mx = max(mx, __float_as_uint(v[u]) & 0x7FFFFFFFu);
  const uint32_t E = mx >> 23;
  if constexpr (UPD) {
    local_update16<PRE>(v, E, f, wo, wm);
    return -1;
  }
  const int sh = wire_shard_of(f, wo);
  const uint32_t pos = f - (uint32_t)sh * (uint32_t)wo.shard;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int u = 0; u < 16; ++u) w[u >> 2] |= ((uint32_t)wire_encode(v[u], E, wo.codec) & 0xFFu) << (8 * (u & 3));
  uint8_t* base = wire_shard_base(sh, wo);
  *reinterpret_cast<uint4*>(base + pos) = make_uint4(w[0], w[1], w[2], w[3]);
  base[wo.shard + pos / 16] = (uint8_t)E;
  return sh;
}

template <bool UPD = false>
__device__ __forceinline__ int wire_store16(const float v[16], uint32_t f, const WireOut& wo) {
  float wm[16];
  return wire_store16<UPD, false>(v, f, wo, wm);
}

// Encode one whole 16-column group of C(row, col..col+15); the owner shard is also written to C in f32.
template <bool UPD = false, bool PRE = false>
__device__ __forceinline__ void wire_epi16(const float v[16], float* __restrict__ C, int64_t ldc, const WireOut& wo,
                                           int row, int col, float (&w)[16]) {
  const uint32_t loc = (uint32_t)row * (uint32_t)ldc + (uint32_t)col;
  const int sh = wire_store16<UPD, PRE>(v, wo.off + loc, wo, w);
  if (sh >= 0 && (wo.own == kWireOwnAll || (wo.period > 0 ? sh % wo.period : sh) == wo.own)) {
#pragma unroll
    for (int u = 0; u < 16; u += 4)
      *reinterpret_cast<float4*>(C + loc + u) = make_float4(v[u], v[u + 1], v[u + 2], v[u + 3]);
  }
}

template <bool UPD = false>
__device__ __forceinline__ void wire_epi16(const float v[16], float* __restrict__ C, int64_t ldc, const WireOut& wo,
                                           int row, int col) {
  float w[16];
  wire_epi16<UPD, false>(v, C, ldc, wo, row, col, w);
}

// Fused bias gradient tail: lanes l, l^16, l^32, l^48 hold the same column over different k rows. Writes
// out[col0 + j*16 + lane] (the column sums, or this K-split's partial sums); with kEpiWire and no split-K also
// encodes the bias segment of the [W | b] bucket (its 16-column group is lanes 0..15).
template <int NJ, int WTN, int EPI, bool SPLIT>
__device__ __forceinline__ void colsum_finish(float (&cs)[NJ], int lane, int col0, float* __restrict__ out,
                                              const WireOut& wo, int N) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float v = cs[j];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    const int col = col0 + j * 16 + (lane & 15);
    if (lane < 16 && col < N) out[col] = v;
    if constexpr (is_wire_epi(EPI) && !SPLIT) {
      if (wo.bias_off > 0 && col0 + j * 16 < N) {  // N % 16 == 0: the 16-column group is wholly in range
        uint32_t mx = __float_as_uint(v) & 0x7FFFFFFFu;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        const uint32_t E = mx >> 23;
        const uint32_t f = (uint32_t)wo.bias_off + (uint32_t)col;
        if constexpr (EPI == kEpiWireUpd) {  // fused local update of the bias segment, one element per lane
          if (lane < 16) {
            float w = wo.um[f], m = wo.umom ? wo.umom[f] : 0.f;
            sgd_apply(wire_roundtrip_rne(v, E), w, m, wo.umom != nullptr, wo.up);
            wo.um[f] = w;
            if (wo.umom) wo.umom[f] = m;
            if (wo.ulp) wo.ulp[f] = f32_to_bf16(w);
          }
          continue;
        }
        const int sh = wire_shard_of(f, wo);
        const uint32_t pos = f - (uint32_t)sh * (uint32_t)wo.shard;
        uint8_t* base = wire_shard_base(sh, wo);
        if (lane < 16) base[pos] = (uint8_t)(wire_encode(v, E, wo.codec) & 0xFF);
        if (lane == 0) base[wo.shard + pos / 16] = (uint8_t)E;
      }
    }
  }
}

// Epilogue of one wave's (MI*16) x WTN accumulator tile at C(row0, col0), staged through a wave-private LDS
// region one 16-row block at a time and written as coalesced row segments (f32 16 B / bf16 8 B per lane), with
// the fused epilogue; SPLIT writes the f32 partial slab of K-split ksplit; kEpiWire encodes whole 16-column
// groups (one lane per group: 16-B mantissa store + exponent byte). Caller: all LDS operand reads retired.
// SW (bf16 8-column path only): staged columns per pass over a 16-row block — WTN, or 64 (two halves: 17 KiB of
// staging for 4 waves instead of 33, beside the operand stages of the overlapped persistent loop).
template <int MI, int NJ, int WTN, int EPI, typename TC, bool ACCUM, bool SPLIT, int SW = WTN, bool WT = false>
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[MI][NJ], char* smem, int wave, int lane, int row0,
                                           int col0, TC* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ bias,
                                           const TC* __restrict__ aux, int64_t ldaux, int M, int N, int ksplit,
                                           float* __restrict__ ws, const WireOut& wo, bool mn_edge = false) {
  static_assert(SW == WTN || (SW == 64 && WTN % 64 == 0 && sizeof(TC) == 2 && !SPLIT && !is_wire_epi(EPI)),
                "64-column staging: bf16 8-column path only");
  static_assert(!WT || (sizeof(TC) == 2 && !SPLIT && !is_wire_epi(EPI)), "write-through stores: the bf16 8-column path");
  constexpr int EW = SW + 4;  // staged row stride in floats (16-B aligned, breaks bank aliasing)
  float* stg = reinterpret_cast<float*>(smem) + wave * (16 * EW);
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
  constexpr int C4 = WTN / 4;   // float4 chunks per staged row
  constexpr int RPI = 64 / C4;  // rows covered per pass by the wave
  // ReLU-mask epilogue: the activation reads are latency-bound (64 MB over a 190 us GEMM is no bandwidth), so the
  // loads of 16-row block i + kPf are issued before block i is staged and stored; each lane keeps kPf + 1 blocks
  // of 4-element activation chunks in registers (bwd-data 8192x4096: 19 us of exposed load latency otherwise).
  // bf16 outputs: 8 columns (16 B) per lane and store (epi8_bf16). C, bias and the activation must be 16-B aligned
  // with ldc, ldaux % 8 == 0 (launch_gemm_bf16 checks; ops/gemm.py stages misaligned operands through aligned
  // copies). One path only: keeping the 8-B path beside it as a run-time fallback spilled 20-33 VGPRs in the
  // persistent kernels.
  if constexpr (sizeof(TC) == 2 && !SPLIT && !is_wire_epi(EPI)) {
    {
      constexpr int C8 = SW / 8;    // 16-B chunks per staged row
      constexpr int RP8 = 64 / C8;  // rows per pass
      constexpr int NP8 = 16 / RP8;
      constexpr int HV = WTN / SW;  // staged column halves
      static_assert(WTN % 8 == 0 && RP8 <= 16 && 16 % RP8 == 0, "8-column chunks of whole 16-row blocks");
      constexpr bool kPf8 = EPI == kEpiReluMask;
      constexpr int kPfd = 2;
      uint4 aq8[kPf8 ? MI : 1][kPf8 ? HV * NP8 : 1];
      auto aux_load8 = [&](int i) __attribute__((always_inline)) {
#pragma unroll
        for (int hv = 0; hv < HV; ++hv)
#pragma unroll
          for (int pass = 0; pass < NP8; ++pass) {
            const int row = row0 + i * 16 + pass * RP8 + lane / C8;
            const int col = col0 + hv * SW + (lane % C8) * 8;
            if (!mn_edge || (row < M && col < N))
              aq8[i][hv * NP8 + pass] = *reinterpret_cast<const uint4*>(aux + (int64_t)row * ldaux + col);
          }
      };
      if constexpr (kPf8) {
#pragma unroll
        for (int i = 0; i < kPfd && i < MI; ++i) aux_load8(i);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr (kPf8) {
          if (i + kPfd < MI) aux_load8(i + kPfd);
        }
#pragma unroll
        for (int hv = 0; hv < HV; ++hv) {
#pragma unroll
        for (int j = 0; j < SW / 16; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) stg[(row_l + r) * EW + j * 16 + col_l] = acc[i][hv * (SW / 16) + j][r];
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own LDS writes landed (wave-private region)
#pragma unroll
        for (int pass = 0; pass < NP8; ++pass) {
          const int rr = pass * RP8 + lane / C8;
          const int cc = (lane % C8) * 8;
          const float4 q0 = *reinterpret_cast<const float4*>(stg + rr * EW + cc);
          const float4 q1 = *reinterpret_cast<const float4*>(stg + rr * EW + cc + 4);
          float v[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
          const int row = row0 + i * 16 + rr;
          const int col = col0 + hv * SW + cc;
          if (mn_edge && (row >= M || col >= N)) continue;  // N % 8 == 0: an 8-column chunk is wholly in or out
          const uint4* mk = nullptr;
          if constexpr (kPf8) mk = &aq8[i][hv * NP8 + pass];
          epi8_bf16<EPI, ACCUM, WT>(v, reinterpret_cast<bf16_t*>(C), ldc, bias, mk, row, col);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // the staged rows are read before the next half / block rewrites them
        }
      }
      return;
    }
  }
  constexpr bool kPfAux = EPI == kEpiReluMask && !SPLIT && sizeof(TC) == 2;  // (f32 chunks: too many registers)
  constexpr int kPf = 2;
  constexpr int NP = 16 / RPI;
  using AuxV = typename std::conditional<sizeof(TC) == 2, uint2, uint4>::type;
  AuxV aq[kPfAux ? MI : 1][kPfAux ? NP : 1];
  auto aux_load = [&](int i) __attribute__((always_inline)) {
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
      const int row = row0 + i * 16 + pass * RPI + lane / C4;
      const int col = col0 + (lane % C4) * 4;
      if (!mn_edge || (row < M && col < N))
        aq[i][pass] = *reinterpret_cast<const AuxV*>(aux + (int64_t)row * ldaux + col);
    }
  };
  if constexpr (kPfAux) {
#pragma unroll
    for (int i = 0; i < kPf && i < MI; ++i) aux_load(i);
  }
  // fused local update (unsplit wire epilogue): the master values of 16-row block i + kUpf's groups are loaded while
  // block i is encoded and updated, instead of one dependent load round trip per block (all CUs run this epilogue
  // at the same moment, so each round trip is a loaded-HBM latency)
  constexpr bool kPfUpd = EPI == kEpiWireUpd && !SPLIT;
  constexpr int UG16 = WTN / 16, URPG = 64 / UG16, UPASS = URPG >= 16 ? 1 : 16 / URPG;
#ifndef FAN_GEMM_UPD_PF
// row blocks of master weights loaded ahead of the one being updated (2: profiles/r6_upd_prefetch_depth_ab.txt)
#define FAN_GEMM_UPD_PF 2
#endif
  constexpr int kUpf = FAN_GEMM_UPD_PF, US = kPfUpd ? kUpf + 1 : 1;
  float um_pf[US][kPfUpd ? UPASS : 1][16];
  auto upd_load = [&](int i, int slot) __attribute__((always_inline)) {
    if constexpr (kPfUpd) {
#pragma unroll
      for (int pass = 0; pass < UPASS; ++pass) {
        const int rr = pass * URPG + lane / UG16;
        const int row = row0 + i * 16 + rr, col = col0 + (lane % UG16) * 16;
        if ((URPG <= 16 || rr < 16) && (!mn_edge || (row < M && col < N))) {
          const float* q = wo.um + wo.off + (uint32_t)row * (uint32_t)ldc + (uint32_t)col;
#pragma unroll
          for (int u = 0; u < 16; u += 4) {
            const float4 a = *reinterpret_cast<const float4*>(q + u);
            um_pf[slot][pass][u] = a.x; um_pf[slot][pass][u + 1] = a.y;
            um_pf[slot][pass][u + 2] = a.z; um_pf[slot][pass][u + 3] = a.w;
          }
        }
      }
    }
  };
  if constexpr (kPfUpd) {
#pragma unroll
    for (int d = 0; d < kUpf && d < MI; ++d) upd_load(d, d % US);
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    if constexpr (kPfAux) {
      if (i + kPf < MI) aux_load(i + kPf);
    }
    if constexpr (kPfUpd) {
      if (i + kUpf < MI) upd_load(i + kUpf, (i + kUpf) % US);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) stg[(row_l + r) * EW + j * 16 + col_l] = acc[i][j][r];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own LDS writes landed (wave-private region)
    if constexpr (is_wire_epi(EPI) && !SPLIT) {
      constexpr int G16 = WTN / 16;  // groups per staged row
      constexpr int RPG = 64 / G16;  // rows per pass (lanes beyond 16 rows idle)
      constexpr int PASSES = RPG >= 16 ? 1 : 16 / RPG;
#pragma unroll
      for (int pass = 0; pass < PASSES; ++pass) {
        const int rr = pass * RPG + lane / G16;
        if (RPG <= 16 || rr < 16) {
          const int cc = (lane % G16) * 16;
          float v[16];
#pragma unroll
          for (int u = 0; u < 16; u += 4) {
            const float4 q = *reinterpret_cast<const float4*>(stg + rr * EW + cc + u);
            v[u] = q.x; v[u + 1] = q.y; v[u + 2] = q.z; v[u + 3] = q.w;
          }
          if (!mn_edge || (row0 + i * 16 + rr < M && col0 + cc < N))
            wire_epi16<EPI == kEpiWireUpd, kPfUpd>(v, reinterpret_cast<float*>(C), ldc, wo, row0 + i * 16 + rr,
                                                   col0 + cc, um_pf[kPfUpd ? i % US : 0][kPfUpd ? pass : 0]);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      continue;
    }
#pragma unroll
    for (int pass = 0; pass < 16 / RPI; ++pass) {
      const int rr = pass * RPI + lane / C4;
      const int cc = (lane % C4) * 4;
      const float4 q = *reinterpret_cast<const float4*>(stg + rr * EW + cc);
      float v[4] = {q.x, q.y, q.z, q.w};
      const int row = row0 + i * 16 + rr;
      const int col = col0 + cc;
      if (mn_edge && (row >= M || col >= N)) continue;  // N % 8 == 0: a 4-column chunk is wholly in or out
      if (SPLIT) {
        float* slab = ws + (int64_t)ksplit * M * N;
        *reinterpret_cast<float4*>(slab + (int64_t)row * N + col) = q;
      } else if constexpr (kPfAux) {
        float m[4];
        if constexpr (sizeof(TC) == 2) {
          const uint2 u = aq[i][pass];
          m[0] = __uint_as_float(u.x << 16); m[1] = __uint_as_float(u.x & 0xFFFF0000u);
          m[2] = __uint_as_float(u.y << 16); m[3] = __uint_as_float(u.y & 0xFFFF0000u);
        } else {
          const uint4 u = aq[i][pass];
          m[0] = __uint_as_float(u.x); m[1] = __uint_as_float(u.y);
          m[2] = __uint_as_float(u.z); m[3] = __uint_as_float(u.w);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = m[u] > 0.f ? v[u] : 0.f;
        epi4<kEpiNone, TC, ACCUM>(v, C, ldc, bias, aux, ldaux, row, col);
      } else {
        epi4<EPI, TC, ACCUM>(v, C, ldc, bias, aux, ldaux, row, col);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
}

// 8 waves (2 per SIMD) or 4 waves (1 per SIMD, up to 512 VGPR+AGPR per lane: large per-wave tiles).
// RAGGED: the shape is not a multiple of the tile (or K of BK * split_k); only then is the edge code compiled in,
// so aligned shapes run exactly the unpredicated kernel.
template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI, typename TC, bool ACCUM, bool SPLIT,
          bool DMA1 = false, bool RAGGED = false>
__global__ void __launch_bounds__(WM * WN * 64, WM * WN / 4)
    gemm_bf16_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb,
                     TC* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ bias, const TC* __restrict__ aux,
                     int64_t ldaux, int M, int N, int K, int split_k, float* __restrict__ ws,
                     float* __restrict__ colsum, WireOut wo) {
  constexpr int NT = WM * WN * 64;
  constexpr int A_BYTES = OpTile<BM, NT>::BYTES, B_BYTES = OpTile<BN, NT>::BYTES;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int S = (3 * STAGE <= 160 * 1024) ? 3 : 2;
  constexpr int G = OpTile<BM, NT>::GLDS + OpTile<BN, NT>::GLDS;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // per-wave sub-tile
  constexpr int MI = WTM / 16, NJ = WTN / 16;
  static_assert(WM * WN == 8 || WM * WN == 4, "4 or 8 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tiles_n = cdiv_i(N, BN);
  const int tiles_m = cdiv_i(M, BM);
  const int tiles = tiles_m * tiles_n;
  const int nwg = tiles * split_k;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tile = wg % tiles;
  const int ksplit = wg / tiles;
  // 2-D grouped order: consecutive tiles (one XCD's contiguous run after xcd_remap) walk GM tile-rows
  // before moving right, so an XCD works on a compact GM x (run/GM) block of C and its L2 holds
  // fewer distinct A/B panel slices per k-step.
  const int GM = tiles_m >= 4 ? 4 : tiles_m;
  const int grp = tile / (GM * tiles_n);
  const int gm = (tiles_m - grp * GM) < GM ? (tiles_m - grp * GM) : GM;
  const int in_grp = tile % (GM * tiles_n);
  const int m0 = (grp * GM + in_grp % gm) * BM;
  const int n0 = (in_grp / gm) * BN;
  // K-tiles of this split (a ragged K: the last split is shorter, the last K-tile is zero-filled past K)
  const int nkt = cdiv_i(K, BK);
  const int kt_per = cdiv_i(nkt, split_k);
  const int kt0 = ksplit * kt_per;
  const int nk = max(0, min(nkt, kt0 + kt_per) - kt0);
  const int kbeg = kt0 * BK;
  const bool mn_edge = RAGGED && (m0 + BM > M || n0 + BN > N);
  const bool edge = RAGGED && (mn_edge || (kt0 + nk) * BK > K);  // uniform: predicated staging for this workgroup

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // fused bias gradient: the waves of the first row-block sum the (MN-contiguous) B fragments they read
  const bool do_colsum = !BKC && colsum != nullptr && m0 == 0 && wm == 0;  // (SPLIT: partial sums)
  float cs[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) cs[j] = 0.f;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue_stage = [&](int kt_stage, int buf) {
    char* st = smem + buf * STAGE;
    if (edge) {
      stage_tile<AK, BM, NT, true>(A, lda, m0, kbeg + kt_stage * BK, st, wave, lane, M, K);
      stage_tile<BKC, BN, NT, true>(B, ldb, n0, kbeg + kt_stage * BK, st + A_BYTES, wave, lane, N, K);
    } else {
      stage_tile<AK, BM, NT>(A, lda, m0, kbeg + kt_stage * BK, st, wave, lane);
      stage_tile<BKC, BN, NT>(B, ldb, n0, kbeg + kt_stage * BK, st + A_BYTES, wave, lane);
    }
  };

  // Register budget per lane: 4 waves = 1 wave/SIMD (512 VGPR+AGPR), 8 waves = 2 waves/SIMD (256).
  constexpr int REG_BUDGET = NT == 256 ? 480 : 232;
  constexpr int ACC_R = MI * NJ * 4, FRAG_R = (MI + NJ) * 4;
  constexpr bool DBL = ACC_R + 2 * FRAG_R <= REG_BUDGET;
  // prologue: stages 0..S-2 in flight
#pragma unroll
  for (int s = 0; s < S - 1; ++s) {
    if (s < nk) issue_stage(s, s);
  }

  for (int kt = 0; kt < nk; ++kt) {
    FAN_STAMP(0);
    // retire stage kt (this wave's DMA), leaving the younger stages in flight
    if (S == 3 && kt + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    FAN_STAMP(1);
    __builtin_amdgcn_s_barrier();  // every wave retired stage kt and finished computing kt-1
    FAN_STAMP(2);
    const bool pf = kt + S - 1 < nk;
    char* pst = smem + ((kt + S - 1) % S) * STAGE;
    const int pk = kbeg + (kt + S - 1) * BK;
    if constexpr (DMA1 && S == 2 && NT == 512) {
      // DMA by waves 0..3 only (one per SIMD; waves w and w+4 share a SIMD): their partners go straight to the
      // fragment reads and MFMAs while the CU's load path drains the 64 KB stage burst. Measured in one process
      // (profiles/r1_gemm_dma_one_wave_ab.jsonl): bwd-weight layout (both operands MN-contiguous, 48 transposing
      // fragment reads per wave and K-tile) 3-10 % faster; with a K-contiguous A 12-25 % slower, so only the
      // bwd-weight layout uses it (launch_main).
      if (pf && wave < 4) {
        if (edge) {
          stage_tile<AK, BM, 256, true>(A, lda, m0, pk, pst, wave, lane, M, K);
          stage_tile<BKC, BN, 256, true>(B, ldb, n0, pk, pst + A_BYTES, wave, lane, N, K);
        } else {
          stage_tile<AK, BM, 256>(A, lda, m0, pk, pst, wave, lane);
          stage_tile<BKC, BN, 256>(B, ldb, n0, pk, pst + A_BYTES, wave, lane);
        }
      }
    } else if (pf) {
      if (edge) {
        stage_tile<AK, BM, NT, true>(A, lda, m0, pk, pst, wave, lane, M, K);
        stage_tile<BKC, BN, NT, true>(B, ldb, n0, pk, pst + A_BYTES, wave, lane, N, K);
      } else {
        stage_tile<AK, BM, NT>(A, lda, m0, pk, pst, wave, lane);
        stage_tile<BKC, BN, NT>(B, ldb, n0, pk, pst + A_BYTES, wave, lane);
      }
    }
    FAN_STAMP(3);
    const char* sa = smem + (kt % S) * STAGE;
    const char* sb = sa + A_BYTES;
    if constexpr (DBL) {
      // issue the fragment reads of BOTH k-steps up front: the k-step-1 reads overlap the k-step-0 MFMAs
      // (hipcc emits counted lgkmcnt waits per consumer)
      s16x8 af[2][MI], bfr[2][NJ];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < MI; ++i) af[ks][i] = read_frag<AK>(sa, wm * WTM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[ks][j] = read_frag<BKC>(sb, wn * WTN + j * 16, ks, lane);
        if (do_colsum) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) cs[j] += frag_sum(bfr[ks][j]);
        }
      }
      FAN_STAMP(4);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[ks][i]),
                                                                __builtin_bit_cast(bf16x8, bfr[ks][j]), acc[i][j],
                                                                0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    } else {
      // 128-accumulator tiles: one k-step of fragments live at a time (keeps VGPRs < 256 and leaves
      // register-file room for a co-resident communication wave on each SIMD)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s16x8 af[MI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i] = read_frag<AK>(sa, wm * WTM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = read_frag<BKC>(sb, wn * WTN + j * 16, ks, lane);
        if (do_colsum) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) cs[j] += frag_sum(bfr[j]);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                                __builtin_bit_cast(bf16x8, bfr[j]), acc[i][j], 0,
                                                                0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }

  if (do_colsum)
    colsum_finish<NJ, WTN, EPI, SPLIT>(cs, lane, n0 + wn * WTN, SPLIT ? ws + (int64_t)split_k * M * N + (int64_t)ksplit * N
                                                                      : colsum, wo, N);
  __syncthreads();  // all waves done reading the operand ring
  store_tile<MI, NJ, WTN, EPI, TC, ACCUM, SPLIT>(acc, smem, wave, lane, m0 + wm * WTM, n0 + wn * WTN, C, ldc, bias,
                                                 aux, ldaux, M, N, ksplit, ws, wo, mn_edge);
}

// ---------------------------------------------------------------------------------------------------------------
// Software-pipelined 256x256 kernel (8 waves, 2x4, 128x64 per wave) for the K-contiguous-A layouts.
//
// The one-role loop runs each K-tile as barrier -> DMA burst -> fragment reads -> MFMAs, with every wave in the same
// phase (one workgroup-wide barrier), so the MFMA pipes idle through the first three (r1 stamps: DMA issue ~1000,
// reads 500-800, MFMAs ~1300 of ~4000 cycles). Here every load hides under MFMAs:
//   * k-step 0 of K-tile t: 32 MFMAs on registers read earlier; under them the fragments of k-step (t, 1) are read
//     (A fragments rolling: A_i of the next k-step is read right after row i's MFMAs; B fragments double-buffered);
//   * then this wave's DMA of K-tile t+1 and its reads of (t, 1) retire (vmcnt(0), lgkmcnt(0)) and ONE barrier;
//   * k-step 1: 32 MFMAs; under them the fragments of (t+1, 0) are read from the other stage (complete for every
//     wave after the barrier) and the DMA of K-tile t+2 goes into stage t & 1 (nobody reads it any more: every wave
//     retired its reads of it before the barrier), one piece per 4 MFMAs.
// The DMA of a K-tile thus has two k-steps of MFMAs to land. LDS: 2 stages x 64 KiB. Glds with SGPR bases + 32-bit
// lane offsets computed once. Aligned shapes only (M, N % 256, K % (64 * split_k)); every layout and epilogue.
// M0 is written in the statement that reads it and not restored (cdna_hip_programming.md §5.7's clobbering form): the
// compiler emits no M0 access of its own in any kernel of this library (every M0 read or write in the built code
// objects is one of these statements' s_mov_b32 m0 / global_load_lds), and saving / restoring it cost 2 of the 3 SALU
// instructions per 1 KiB piece — the flagship step measured 1.0 % faster without them, 3 of 3 interleaved pairs
// (profiles/r5_glds_m0_ab.txt).
__device__ __forceinline__ void glds16_s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_addr)
               : "memory");
}

// The same with the LDS destination as a wave-uniform base + a compile-time byte offset, added into M0 by the
// statement itself (1 SALU per piece instead of the compiler's add + the move).
template <uint32_t OFF, bool SC1 = false>
__device__ __forceinline__ void glds16_si(const void* sbase, uint32_t voff, uint32_t lds_base) {
  if constexpr (SC1)  // bypassing this CU's L1 (the layer chain's handed-off operand: no stale L1 copy can be hit)
    asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 sc1" ::"v"(voff), "s"(sbase),
                 "s"(lds_base), "i"(OFF)
                 : "memory", "scc");
  else
    asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase),
                 "s"(lds_base), "i"(OFF)
                 : "memory", "scc");
}

// s_waitcnt vmcnt(VM) lgkmcnt(LGKM) through the compiler's builtin, so that its own wait insertion knows what the wait
// leaves outstanding: after an asm wait (opaque to it) it re-waits, lgkmcnt(N) by lgkmcnt(N), in front of the first use
// of every fragment read already complete — ~16 extra s_waitcnt per K-tile of the 4-wave loop. The empty asm keeps
// the LDS reads after it from being hoisted above it (the asm form's "memory" clobber). FAN_GEMM_ASM_WAITS (diagnostic
// builds): the asm form.
template <int VM, int LGKM>
__device__ __forceinline__ void waitcnt_known() {
  static_assert(VM >= 0 && VM <= 63 && LGKM >= 0 && LGKM <= 15, "s_waitcnt field ranges");
#ifdef FAN_GEMM_ASM_WAITS
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(%1)" ::"n"(VM), "n"(LGKM) : "memory");
#else
  __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (LGKM << 8) | ((VM >> 4) << 14));
  asm volatile("" ::: "memory");
#endif
}

// Byte offset (from the operand's K-tile origin) of this lane's chunk of glds instruction i: stage_one's address
// math without the base pointer.
template <bool KCONTIG, int OUTER, int NT>
__device__ __forceinline__ uint32_t piece_off(int64_t ld, int o0, int wave, int lane, int i) {
  using T = OpTile<OUTER, NT>;
  const int t = wave * 64 + lane;
  if (KCONTIG) {
    const int row = i * (T::IB / 128) + (t >> 3);
    const int c = (t & 7) ^ ((row >> 1) & 7);
    return (uint32_t)(((int64_t)(o0 + row) * ld + c * 8) * 2);
  } else {
    const int half = i / T::PER_HALF;
    const int krow = (i % T::PER_HALF) * (T::IB / 256) + (t >> 4);
    const int cs = t & 15;
    const int blk = (cs >> 1) ^ mn_swz(krow);
    return (uint32_t)(((int64_t)krow * ld + o0 + half * 128 + blk * 16 + (cs & 1) * 8) * 2);
  }
}

template <bool AK, bool BKC, int EPI, typename TC, bool ACCUM, bool SPLIT, bool COLSUM = false>
__global__ void __launch_bounds__(512, 2)
    gemm_pl_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb,
                   TC* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ bias, const TC* __restrict__ aux,
                   int64_t ldaux, int M, int N, int K, int split_k, float* __restrict__ ws,
                   float* __restrict__ colsum, WireOut wo) {
  constexpr int BM = 256, BN = 256, NT = 512;
  constexpr int A_BYTES = OpTile<BM, NT>::BYTES;
  constexpr int STAGE = A_BYTES + OpTile<BN, NT>::BYTES;
  constexpr int GA = OpTile<BM, NT>::GLDS, G = GA + OpTile<BN, NT>::GLDS;  // 4 + 4 pieces per wave and K-tile
  constexpr int WTM = 128, WTN = 64, MI = 8, NJ = 4;
  static_assert(G == 8, "8 glds pieces per wave and K-tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tiles_n = N / BN, tiles_m = M / BM, tiles = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, tiles * split_k);
  const int tile = wg % tiles, ksplit = wg / tiles;
  const int GM = tiles_m >= 4 ? 4 : tiles_m;
  const int grp = tile / (GM * tiles_n);
  const int gm = (tiles_m - grp * GM) < GM ? (tiles_m - grp * GM) : GM;
  const int in_grp = tile % (GM * tiles_n);
  const int m0 = (grp * GM + in_grp % gm) * BM;
  const int n0 = (in_grp / gm) * BN;
  const int k_per = K / split_k;
  const int kbeg = ksplit * k_per;
  const int nk = k_per / BK;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / 4, wn = wave % 4;
  // fused bias gradient (COLSUM: MN-contiguous B), waves wm == 0 sum the B fragments they use. Without split-K the
  // work is spread over the tile rows so no tile runs long (one round of tiles: the slowest sets the time): tile row
  // im sums K-tiles [cs0, cs1) into partial slab im of ws[]; with split-K (one partial per split, tile row 0) the
  // partials ride along with the slab reduce. An ordered reduce over the partials follows (launch_typed).
  const int im = SPLIT ? 0 : m0 / BM;
  const int cs0 = SPLIT ? (m0 == 0 ? 0 : nk) : im * nk / tiles_m;
  const int cs1 = SPLIT ? nk : (im + 1) * nk / tiles_m;
  const bool do_colsum = COLSUM && wm == 0;
  float cs[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) cs[j] = 0.f;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 fa[MI], fb[2][NJ];

  uint32_t off[G];
#pragma unroll
  for (int p = 0; p < GA; ++p) off[p] = piece_off<AK, BM, NT>(lda, m0, wave, lane, p);
#pragma unroll
  for (int p = GA; p < G; ++p) off[p] = piece_off<BKC, BN, NT>(ldb, n0, wave, lane, p - GA);
  const int64_t a_step = AK ? (int64_t)BK * 2 : (int64_t)BK * lda * 2;
  const int64_t b_step = BKC ? (int64_t)BK * 2 : (int64_t)BK * ldb * 2;
  const char* a_k0 = reinterpret_cast<const char*>(A) + (AK ? (int64_t)kbeg * 2 : (int64_t)kbeg * lda * 2);
  const char* b_k0 = reinterpret_cast<const char*>(B) + (BKC ? (int64_t)kbeg * 2 : (int64_t)kbeg * ldb * 2);
  const uint32_t lds0 = lds_addr_of(smem);

  auto piece = [&](int kt, int p) {  // glds piece p (0..7) of K-tile kt into stage kt & 1
    const uint32_t st = lds0 + (kt & 1) * STAGE + wave * 1024;
    if (p < GA) glds16_s(a_k0 + kt * a_step, off[p], st + p * OpTile<BM, NT>::IB);
    else glds16_s(b_k0 + kt * b_step, off[p], st + A_BYTES + (p - GA) * OpTile<BN, NT>::IB);
  };
  auto read_a = [&](const char* st, int ks, int i) { fa[i] = read_frag<AK>(st, wm * WTM + i * 16, ks, lane); };
  auto read_b = [&](const char* st, int ks, int set, int j) {
    fb[set][j] = read_frag<BKC>(st + A_BYTES, wn * WTN + j * 16, ks, lane);
  };
  // One k-step: 32 MFMAs (rows i of 4) on B set `cur`. READ: the next k-step's fragments (stage rd_st, k-step rd_ks)
  // are read under them — B_j into the other set during rows 0-1, A_i right after row i. DMA: one glds piece of
  // K-tile dma_kt per 4 MFMAs. Compile-time flags: no branches inside the MFMA stream.
  auto block = [&](auto cur_c, auto read_c, auto dma_c, const char* rd_st, int rd_ks, int dma_kt, bool csk) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool READ = decltype(read_c)::value, DMA = decltype(dma_c)::value;
    if (COLSUM && csk) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) cs[j] += frag_sum(fb[cur][j]);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (READ && i < 2 && (j & 1) == 0) read_b(rd_st, rd_ks, cur ^ 1, i * 2 + (j >> 1));
        if (DMA && j == 2) piece(dma_kt, i);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                            __builtin_bit_cast(bf16x8, fb[cur][j]), acc[i][j], 0, 0, 0);
      }
      if (READ) read_a(rd_st, rd_ks, i);
    }
    // keep the source order: the scheduler otherwise clusters the LDS reads at the end of the MFMA stream, where
    // the barrier's lgkmcnt(0) then waits on all of them
    if constexpr (READ) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (i < 2) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using T_ = std::true_type;
  using F_ = std::false_type;

  // prologue: K-tiles 0 and 1 in flight; retire 0 (this wave), barrier (every wave), read k-step (0, 0)
#pragma unroll
  for (int p = 0; p < G; ++p) piece(0, p);
  if (nk > 1) {
#pragma unroll
    for (int p = 0; p < G; ++p) piece(1, p);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < NJ; ++j) read_b(smem, 0, 0, j);
#pragma unroll
  for (int i = 0; i < MI; ++i) read_a(smem, 0, i);

  auto ktile = [&](int kt, auto more_c, auto more2_c) {
    const char* st = smem + (kt & 1) * STAGE;
    const bool csk = do_colsum && kt >= cs0 && kt < cs1;
    FAN_STAMP(0);
    __builtin_amdgcn_s_setprio(1);
    block(I0{}, T_{}, F_{}, st, 1, 0, csk);
    __builtin_amdgcn_s_setprio(0);
    FAN_STAMP(1);
    // this wave's DMA of K-tile kt+1 and its reads of (kt, 1) retired; after the barrier, every wave's
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    FAN_STAMP(2);
    __builtin_amdgcn_s_barrier();
    FAN_STAMP(3);
    __builtin_amdgcn_s_setprio(1);
    block(I1{}, more_c, more2_c, smem + ((kt + 1) & 1) * STAGE, 0, kt + 2, csk);
    __builtin_amdgcn_s_setprio(0);
    FAN_STAMP(4);
  };
  int kt = 0;
  for (; kt + 2 < nk; ++kt) ktile(kt, T_{}, T_{});
  if (kt + 1 < nk) ktile(kt++, T_{}, F_{});
  if (kt < nk) ktile(kt, F_{}, F_{});

  if (COLSUM && do_colsum && (!SPLIT || m0 == 0))
    colsum_finish<NJ, WTN, kEpiNone, true>(
        cs, lane, n0 + wn * WTN, ws + (SPLIT ? (int64_t)split_k * M * N + (int64_t)ksplit * N : (int64_t)im * N), wo,
        N);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every operand read retired before the epilogue reuses the LDS
  store_tile<MI, NJ, WTN, EPI, TC, ACCUM, SPLIT>(acc, smem, wave, lane, m0 + wm * WTM, n0 + wn * WTN, C, ldc, bias,
                                                 aux, ldaux, M, N, ksplit, ws, wo);
}

// ---------------------------------------------------------------------------------------------------------------
// Software-pipelined 256x256 kernel with 4 waves (2x2, one per SIMD, 128x128 per wave) and the accumulators in
// AGPRs: a 128x128 wave tile reads (128 + 128) x K fragments per 128x128 outputs where the 8-wave kernel's 128x64
// tiles read (128 + 64) per 128x64, so the CU's LDS read traffic per K-tile drops by a third (the hipBLASLt
// choice for these shapes, profiles/r1_gemm_experiments.md round 2). The MFMAs are inline asm with "+a"
// accumulator operands: 256 accumulators then stay in the AGPR file (hipcc's allocator otherwise rotates them
// through VGPRs); volatile asm also pins the issue order of the reads, DMA and MFMAs to the source order. Both
// fragment sets are double-buffered (VGPRs are free here), so a read never overwrites a register an MFMA of the
// same k-step still reads. Same K-tile schedule as gemm_pl_kernel: k-step 0 reads (t, 1); wait + barrier; k-step 1
// reads (t + 1, 0) and issues the DMA of K-tile t + 2 (16 pieces per wave, one per 4 MFMAs; one per 2 measured no
// faster).

// compile-time loop: f(integral_constant<int, 0..N-1>) in order (indices stay constants: no dynamic array access)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ void mfma_acc(f32x4& acc, const s16x8& a, const s16x8& b) {
#ifdef FAN_GEMM_NOMFMA  // diagnostic builds only: the main loop without its MFMAs (operands still read; timing)
  asm volatile("" : "+a"(acc) : "v"(a), "v"(b));
#else
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
#endif
}

// ---------------------------------------------------------------------------------------------------------------
// Layer-chain GEMM (gemm_chain_kernel, gemm_chain.hip): the GEMMs of a pass — the forward's X -> H1 -> H2 -> logits, the
// backward's dY -> dH2 -> dH1 — as ONE persistent launch, the GPU form of the reference's single `omp parallel` region
// whose layers hand over through barriers (sw/mlp_mpi_example_f32.cpp:690-788). Stage s + 1's A operand is stage s's
// output; an output tile of row panel r (256 rows) of stage s + 1 may start once every tile of row panel r of stage s
// has stored its output, so layer s + 1's first tiles run under layer s's last tiles and epilogue stores instead of
// after a grid-wide drain, a kernel boundary and a new fill.
//   * tickets: workgroup b belongs to group g = b % 8 (one XCD under the round-robin dispatch: speed only) and owns
//     the row panels [g * ppg, (g + 1) * ppg) of every stage; the group's tickets run stage by stage, row panel by row
//     panel (a group's 32 workgroups complete whole panels first). Ticket j of group g: the first gridDim / 8 are
//     static (j = b / 8), the rest come from a per-group atomic head. A workgroup takes its next ticket early in its
//     current tile (K-tile 1) and polls that ticket's dependency two K-tiles before the end, so the decision at the
//     last K-tile costs no latency; a dequeued ticket is always held by a running workgroup and depends only on
//     earlier stages, so the queue cannot deadlock whatever the residency (other streams' kernels, other processes).
//   * hand-off (MI355X_MICROARCH.md § visibility, valid form "agent-scope atomic adds ... sc1 load poll"): a producer
//     stage stores its tiles write-through (sc1, store_wt16); the tile's completion is added to its panel's ready
//     counter by wave 0 lane 0 after every wave's vmcnt(0) and a workgroup barrier (deferred to the next tile's
//     K-tile 1, whose wait and barrier provide exactly that, or to an explicit drain). The consumer polls the
//     counter relaxed (sc1), and EVERY wave then issues its own agent acquire (buffer_inv sc1) ahead of its own
//     LDS-DMA of the panel, so no extra barrier or wait is needed for the acquire.
//   * state: the counter block (per call site and stream) starts zeroed; the last workgroup to leave (an exit counter)
//     zeroes it again for the next launch (it is reached only after every workgroup's final add returned). A spin that
//     exceeds ~4 s stores an error code and gives up (garbage, not a hang); the host reads it (gemm_chain_error).
constexpr int kChainMaxStages = 8;
constexpr int kChainLdsCtl = 2 * (256 + 256) * BK * 2 + 4 * 16 * (64 + 4) * 4;  // past the OVL staging rows
constexpr int kChainLds = kChainLdsCtl + 64;
constexpr uint32_t kChainSpinLimit = 1u << 22;

struct ChainStageArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const bf16_t* bias;
  const void* aux;
  int64_t lda, ldb, ldc, ldaux;
  int M, N, K;
  int tn;      // column tiles
  int first;   // group-local ticket of this stage's first tile
  int dep;     // > 0: a tile waits until ready[stage - 1][its row panel] == dep (the previous stage's tn)
  int signal;  // a finished tile adds 1 to ready[stage][its row panel]
  int cfg;     // 0: the kernel's first tile configuration, 1: its second
};

struct ChainArgs {
  ChainStageArgs st[kChainMaxStages];
  int nstages;
  int total;   // tickets per group
  int ppg;     // row panels per group
  int panels;  // row panels of the pass (M / 256)
  unsigned* ctr;
  int prio;
  int flags;  // diagnostic builds of the schedule (kChainNoAcquire: unsafe; kChainRowsFastest)
};
constexpr int kChainNoAcquire = 1;    // skip the consumer's acquire (diagnostic A/B only: visibility not guaranteed)
constexpr int kChainRowsFastest = 2;  // a group's tiles rows-fastest (all its panels' column c, then c + 1) instead of
                                      // panel by panel

// counter block (uint32 words, one 64-B line each): head[8], exit, error, ready[stage][panel]
__host__ __device__ constexpr int chain_ctr_words(int nstages, int panels) { return (10 + nstages * panels) * 16; }
__device__ __forceinline__ int chain_ready_word(const ChainArgs& ca, int s, int panel) {
  return (10 + s * ca.panels + panel) * 16;
}
__device__ __forceinline__ int chain_stage_of(const ChainArgs& ca, int t) {
  int s = 0;
  while (s + 1 < ca.nstages && t >= ca.st[s + 1].first) ++s;
  return s;
}

// per-workgroup chain state (wave-uniform): the ticket to run next, whether its dependency is known to be met, and
// the ready-counter word of a finished tile whose completion is not yet published (-1: none)
struct ChainState {
  int ticket;
  int ready;
  int pending;
};

// one stage's schedule for the tile loop, derived once per stage run from the kernel arguments and passed by value so
// it lives in SGPRs: the loop never reads the kernel-argument block through a pointer (such reads are vector loads
// whose compiler-inserted vmcnt(0) would drain the loop's in-flight LDS-DMA and epilogue stores)
struct ChainRun {
  unsigned* ctr;
  int group, ppg, wpg;  // XCD group, its row panels, its static tickets
  int first, end, tn;   // this stage's ticket range and column tiles
  int dep;              // > 0: a tile waits until the previous stage's panel counter reaches dep
  int dep_word0;        // that counter's word for the group's first panel (+ 16 per panel)
  int sig_word0;        // this stage's counter word for the group's first panel; -1: no consumer stage
  int nx_end, nx_tn;    // the next stage's ticket end and column tiles (its tickets start at end)
  int flags;
};
__device__ __forceinline__ void chain_rc(const ChainRun& cr, int tn, int k, int& r, int& c) {
  if (cr.flags & kChainRowsFastest) {
    r = k % cr.ppg;
    c = k / cr.ppg;
  } else {
    r = k / tn;
    c = k % tn;
  }
}

__device__ __forceinline__ void chain_add(unsigned* ctr, int word) {
  __hip_atomic_fetch_add(ctr + word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned chain_poll(const unsigned* ctr, int word) {
  return __hip_atomic_load(ctr + word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// this wave's agent-scope acquire: its L1 invalidated before its own later loads (no wait needed for them)
__device__ __forceinline__ void chain_acquire(int flags = 0) {
  if (!(flags & kChainNoAcquire)) asm volatile("buffer_inv sc1" ::: "memory");
}
// row panel (group-local) and column tile of a stage's k-th tile in its group's ticket order
__device__ __forceinline__ void chain_tile_rc(const ChainArgs& ca, int tn, int k, int& r, int& c) {
  if (ca.flags & kChainRowsFastest) {
    r = k % ca.ppg;
    c = k / ca.ppg;
  } else {
    r = k / tn;
    c = k % tn;
  }
}

// dependency word / target of ticket t (group-local); word < 0: none
__device__ __forceinline__ void chain_dep_of(const ChainArgs& ca, int t, int& word, unsigned& target) {
  word = -1;
  target = 0;
  if (t >= ca.total) return;
  const int s = chain_stage_of(ca, t);
  const ChainStageArgs& S = ca.st[s];
  if (S.dep <= 0) return;
  int r, c;
  chain_tile_rc(ca, S.tn, t - S.first, r, c);
  word = chain_ready_word(ca, s - 1, (int)(blockIdx.x & 7) * ca.ppg + r);
  target = (unsigned)S.dep;
}

// The body of gemm_pl4_kernel as a device function: this workgroup runs virtual blocks v0, v0 + vstep, ... of the
// problem's tiles * split_k (COLSUM: the one tile v0). gemm_pl4_kernel passes (blockIdx.x, gridDim.x); the grouped
// kernel (gemm_groupn_kernel) gives each of its problems its own range of workgroups. vstep must be a multiple
// of the XCD count so a virtual block stays on its workgroup's XCD (xcd_remap).
// OVL (256x256 bf16 outputs, persistent, no split-K / bias gradient; FAN_GEMM_OVL): the tile transitions overlap.
// The epilogue stages through a region of its own beside the operand stages (64-column halves, 17 KiB), so the next
// tile's K-tiles 0 and 1 are fetched under the last k-step of this tile (its MFMAs read no fragments, the stages are
// free after its barrier), and the next tile waits only for its K-tile 0 (vmcnt(G + kS): the epilogue's kS stores
// are the youngest) and then for K-tile 1 with those stores still allowed in flight — vmcnt counts loads, stores and
// LDS-DMA together, in issue order (MI355X_MICROARCH.md). Same arithmetic: bit-identical to OVL off.
// CHAIN (gemm_chain_kernel): tiles come from the chain's ticket queue instead of the static stride (v0 / vstep
// unused), each tile of a dependent stage after its row panel's hand-off (see the layer-chain comment above); the
// run returns to the chain loop when the next ticket belongs to another stage or is not known ready (chs). WT: the
// bf16 epilogue stores write through the L2 (a producer stage of the chain).
template <bool AK, bool BKC, int EPI, typename TC, bool ACCUM, bool SPLIT, bool COLSUM = false, int BN_ = 256,
          int BM_ = 256, bool OVL = false, bool CHAIN = false, bool WT = false, bool ASC1 = false>
__device__ __forceinline__ void pl4_run(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
                                        int64_t ldb, TC* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ bias,
                                        const TC* __restrict__ aux, int64_t ldaux, int M, int N, int K, int split_k,
                                        float* __restrict__ ws, float* __restrict__ colsum, const WireOut& wo, int v0,
                                        int vstep, ChainRun cr = ChainRun{}, ChainState* chs = nullptr) {
  constexpr int BM = BM_, BN = BN_, NT = 256;
  constexpr int A_BYTES = OpTile<BM, NT>::BYTES;
  constexpr int STAGE = A_BYTES + OpTile<BN, NT>::BYTES;
  constexpr int GA = OpTile<BM, NT>::GLDS, G = GA + OpTile<BN, NT>::GLDS;  // 8 + 8 (BN 128: 8 + 4; BM 224: 7 + 4)
  constexpr int WTM = BM / 2, WTN = BN / 2, MI = WTM / 16, NJ = WTN / 16;
  constexpr int Q = MI * NJ, R = MI + NJ;  // MFMAs and fragment reads per k-step and wave
#ifndef FAN_GEMM_RSP_Q4
#define FAN_GEMM_RSP_Q4 3  // diagnostic builds: the fragment reads span this many quarters of a k-step
#endif
  constexpr int RSP = (Q * FAN_GEMM_RSP_Q4 / 4) / R, DSP = Q / G;  // read / DMA spacing in MFMAs (64 MFMAs: 3 / 4)
  static_assert(BN == 256 || BN == 128, "256x256 or 256x128 tiles");
  // 224x128 tiles: 1792 rows (the reference's per-rank batch, sw/run.sh:16) are 8 row tiles, so a 1792 x 4096 output
  // is 8 x 32 = 256 workgroups, one per CU (256-row tiles give 7 x 32 = 224 and leave 32 CUs idle). The A image is
  // K-contiguous ([rows][64 k], 32 rows per glds piece: 7 pieces); an MN-contiguous A stages 128-column halves.
  static_assert(BM == 256 || (BM == 224 && BN == 128 && AK && !COLSUM) || (BM == 128 && BN == 128),
                "256-row tiles; 224-row tiles (K-contiguous A, BN 128); 128x128 tiles");
  static_assert(OpTile<BM, NT>::BYTES % OpTile<BM, NT>::IB == 0, "whole glds pieces");
  // 256x128 tiles fit 3 operand stages in the LDS (144 KB): K-tile kt + 2 is then fetched during k-step 0 of kt
  // (its stage was consumed in kt - 1) instead of k-step 1, so 1.5 K-tiles of fetch latency are covered (the
  // classifier forward reads a 64 MB activation straight from HBM inside the step: 76 vs 63 us from the MALL).
  constexpr int STAGES = BN == 128 ? 3 : 2;
  static_assert(RSP >= 1 && DSP >= 1 && G * DSP <= Q, "schedule");
  static_assert(!OVL || (BM == 256 && BN == 256 && !COLSUM && !SPLIT && !ACCUM && sizeof(TC) == 2 &&
                         !is_wire_epi(EPI)),
                "overlapped transitions: 256x256 bf16 tiles without split-K or bias gradient");
  constexpr int kSW = OVL ? 64 : WTN;                             // epilogue staging width
  constexpr int kS = MI * (WTN / kSW) * (16 / (64 / (kSW / 8)));  // the epilogue's stores per wave and tile
  constexpr int DSP2 = Q / (2 * G);                               // OVL: the next tile's two K-tiles in one k-step
  static_assert(!OVL || (G + kS <= 63 && DSP2 >= 1), "vmcnt range / schedule");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tiles_n = N / BN, tiles_m = M / BM, tiles = tiles_m * tiles_n;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / 2, wn = wave % 2;
  const uint32_t lds0 = lds_addr_of(smem);
  if (wo.prio > 0) __builtin_amdgcn_s_setprio(2);
  // Persistent over its tiles when the grid is smaller than the tile count (one workgroup per CU, grid a multiple
  // of the XCD count, so virtual block v = blockIdx.x + i * gridDim.x stays on blockIdx.x's XCD): a workgroup's
  // next tile starts its operand DMA while the previous tile's epilogue stores drain, instead of a new workgroup
  // waiting for the old one to retire (the 2-round grids: 8192x4096 forward and bwd-data). Not with the fused
  // bias gradient: its extra live registers would spill in the loop (the launcher gives it one tile per workgroup).
  static_assert(!CHAIN || (!SPLIT && !COLSUM && !ACCUM && BM == 256), "layer chain: unsplit 256-row tiles");
  // output tile origin of virtual block v (CHAIN: of group-local ticket v, row panel by row panel)
  const int GM = tiles_m >= 4 ? 4 : tiles_m;
  auto tile_origin = [&](int v, int& m, int& n) __attribute__((always_inline)) {
    if constexpr (CHAIN) {
      int r, c;
      chain_rc(cr, cr.tn, v - cr.first, r, c);
      m = (cr.group * cr.ppg + r) * BM;
      n = c * BN;
    } else {
      const int t1 = xcd_remap(v, tiles * split_k) % tiles;
      const int g1 = t1 / (GM * tiles_n);
      const int gm1 = (tiles_m - g1 * GM) < GM ? (tiles_m - g1 * GM) : GM;
      const int i1 = t1 % (GM * tiles_n);
      m = (g1 * GM + i1 % gm1) * BM;
      n = (i1 / gm1) * BN;
    }
  };
  // CHAIN: the next ticket, whether its dependency is met, whether this run continues with it (same stage, OVL)
  int ch_next = 0, ch_rdy = 0;
  bool ch_cont = false;
  auto tile_body = [&](int v, bool first, int vn) __attribute__((always_inline)) {
  const int ksplit = CHAIN ? 0 : xcd_remap(v, tiles * split_k) / tiles;
  int m0, n0;
  tile_origin(v, m0, n0);
  const int k_per = K / split_k;
  const int kbeg = ksplit * k_per;
  const int nk = k_per / BK;

  // fused bias gradient: as gemm_pl_kernel (waves wm == 0; spread over the tile rows without split-K)
  const int im = SPLIT ? 0 : m0 / BM;
  const int cs0 = SPLIT ? (m0 == 0 ? 0 : nk) : im * nk / tiles_m;
  const int cs1 = SPLIT ? nk : (im + 1) * nk / tiles_m;
  const bool do_colsum = COLSUM && wm == 0;
  float cs[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) cs[j] = 0.f;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 fa[2][MI], fb[2][NJ];

  uint32_t off[G];
#pragma unroll
  for (int p = 0; p < GA; ++p) off[p] = piece_off<AK, BM, NT>(lda, m0, wave, lane, p);
#pragma unroll
  for (int p = GA; p < G; ++p) off[p] = piece_off<BKC, BN, NT>(ldb, n0, wave, lane, p - GA);
  const int64_t a_step = AK ? (int64_t)BK * 2 : (int64_t)BK * lda * 2;
  const int64_t b_step = BKC ? (int64_t)BK * 2 : (int64_t)BK * ldb * 2;
  const char* a_k0 = reinterpret_cast<const char*>(A) + (AK ? (int64_t)kbeg * 2 : (int64_t)kbeg * lda * 2);
  const char* b_k0 = reinterpret_cast<const char*>(B) + (BKC ? (int64_t)kbeg * 2 : (int64_t)kbeg * ldb * 2);

  // glds piece p (0..G-1) of K-tile kt into stage kt & 1 (the lambdas are forced inline: an out-of-line call puts
  // the accumulator array in scratch memory)
  auto piece = [&](int kt, auto pc) __attribute__((always_inline)) {
    constexpr int p = decltype(pc)::value;
    const uint32_t st = lds0 + (STAGES == 2 ? kt & 1 : kt % 3) * STAGE + wave * 1024;
    if constexpr (p < GA) glds16_si<p * OpTile<BM, NT>::IB, ASC1>(a_k0 + kt * a_step, off[p], st);
    else glds16_si<A_BYTES + (p - GA) * OpTile<BN, NT>::IB>(b_k0 + kt * b_step, off[p], st);
  };
  // next k-step's fragment r (0..R-1: A rows 0..7, then B columns 0..NJ-1) into set `set`
  auto read_next = [&](const char* st, int ks, int set, int r) __attribute__((always_inline)) {
    if (r < MI) fa[set][r] = read_frag<AK>(st, wm * WTM + r * 16, ks, lane);
    else fb[set][r - MI] = read_frag<BKC>(st + A_BYTES, wn * WTN + (r - MI) * 16, ks, lane);
  };
  // One k-step: Q MFMAs on set `cur`; READ: the R fragments of the next k-step into set cur ^ 1, one per RSP
  // MFMAs from the start (all issued by 3/4 of the block: the barrier's lgkmcnt(0) after k-step 0 then waits on
  // nothing young); DMA: the G pieces of K-tile dma_kt, one per DSP MFMAs.
  auto block = [&](auto cur_c, auto read_c, auto dma_c, const char* rd_st, int rd_ks, int dma_kt,
                   bool csk, auto next_c, bool next_on = false) __attribute__((always_inline)) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool READ = decltype(read_c)::value, DMA = decltype(dma_c)::value, NEXT = decltype(next_c)::value;
    if (COLSUM && csk)
      static_for<NJ>([&](auto jc) __attribute__((always_inline)) { cs[jc.value] += frag_sum(fb[cur][jc.value]); });
    static_for<MI * NJ>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      if constexpr (READ && q % RSP == 0 && q / RSP < R) read_next(rd_st, rd_ks, cur ^ 1, q / RSP);
#ifndef FAN_GEMM_NODMA  // diagnostic builds only: the main loop without its operand DMA (wrong results, timing)
      if constexpr (DMA && q % DSP == DSP / 2 && q / DSP < G) piece(dma_kt, std::integral_constant<int, q / DSP>{});
      // OVL: the next tile's K-tiles 0 and 1 (off[] already holds that tile's offsets)
      if constexpr (NEXT && q % DSP2 == 0 && q / DSP2 < 2 * G) {
        if (next_on) piece(q / DSP2 / G, std::integral_constant<int, q / DSP2 % G>{});
      }
#endif
      mfma_acc(acc[q / NJ][q % NJ], fa[cur][q / NJ], fb[cur][q % NJ]);
    });
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using T_ = std::true_type;
  using F_ = std::false_type;

  // prologue: K-tiles 0 and 1 in flight; retire 0 (this wave), barrier (every wave), read k-step (0, 0)
  // (OVL after a transition: both were fetched by the previous tile's last k-step, before its epilogue's stores)
  if (!OVL || first) static_for<G>([&](auto pc) __attribute__((always_inline)) { piece(0, pc); });
  if (nk > 1) {
    if (!OVL || first) {
      static_for<G>([&](auto pc) __attribute__((always_inline)) { piece(1, pc); });
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G + kS) : "memory");
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int r = 0; r < R; ++r) read_next(smem, 0, 0, r);

  // CHAIN ticket control, run after a K-tile's barrier by every wave (wave 0 lane 0 acts; its values go through the
  // LDS control words so that only the poll result lives in a register across K-tiles): at K-tile 1 publish the
  // previous tile (every wave's stores retired: each waited vmcnt(0) before this barrier) and take the next ticket
  // (ctl[0]); at nk - 3 poll its dependency — in this stage on the previous stage's panel, in the next stage on this
  // stage's panel, further stages left to the chain loop (ctl[2] = -2) — and at nk - 2 post the verdict (ctl[1]); at
  // the last K-tile every wave reads them (chain_decide). The host guarantees nk >= 6.
  unsigned ch_poll = 0;
  int* const ch_ctl = reinterpret_cast<int*>(smem + kChainLdsCtl);
  auto chain_hook = [&](int kt) __attribute__((always_inline)) {
    if constexpr (CHAIN) {
      if (kt == 1) {
        if (wave == 0 && lane == 0) {
          if (chs->pending >= 0) chain_add(cr.ctr, chs->pending);
          ch_ctl[0] = cr.wpg + (int)__hip_atomic_fetch_add(cr.ctr + cr.group * 16, 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
        }
        chs->pending = -1;
      } else if (kt == nk - 3) {
        if (wave == 0 && lane == 0) {
          const int t = ch_ctl[0];
          int r, c, word = -1, tgt = 0;
          if (t < cr.end) {
            if (cr.dep > 0) {
              chain_rc(cr, cr.tn, t - cr.first, r, c);
              word = cr.dep_word0 + r * 16;
              tgt = cr.dep;
            }
          } else if (t < cr.nx_end && cr.sig_word0 >= 0) {
            chain_rc(cr, cr.nx_tn, t - cr.end, r, c);
            word = cr.sig_word0 + r * 16;
            tgt = cr.tn;
          } else {
            word = -2;
          }
          ch_ctl[2] = word;
          ch_ctl[3] = tgt;
          if (word >= 0) ch_poll = chain_poll(cr.ctr, word);
        }
      } else if (kt == nk - 2) {
        if (wave == 0 && lane == 0) {
          const int word = ch_ctl[2];
          ch_ctl[1] = word == -1 || (word >= 0 && ch_poll >= (unsigned)ch_ctl[3]);  // 0: not met or not known
        }
      }
    }
  };
  auto chain_decide = [&]() __attribute__((always_inline)) {
    if constexpr (CHAIN) {
      ch_next = __builtin_amdgcn_readfirstlane(ch_ctl[0]);
      ch_rdy = __builtin_amdgcn_readfirstlane(ch_ctl[1]);
      ch_cont = OVL && ch_rdy && ch_next < cr.end;
      if (ch_cont && cr.dep > 0) chain_acquire(cr.flags);
    }
  };
  auto ktile = [&](int kt, auto more_c, auto more2_c) __attribute__((always_inline)) {
    const char* st = smem + (STAGES == 2 ? kt & 1 : kt % 3) * STAGE;
    const bool csk = do_colsum && kt >= cs0 && kt < cs1;
    FAN_STAMP(0);
    if constexpr (STAGES == 2) {
      constexpr bool kLast = OVL && !decltype(more_c)::value && !decltype(more2_c)::value;
      // the last K-tile: this tile's offsets are dead (its last DMA went out two K-tiles ago); the next tile's
      // (if any) take their place, for the DMA of its K-tiles 0 and 1 in k-step 1 below (CHAIN: known only after
      // this K-tile's barrier)
      auto next_offsets = [&](int vnn) __attribute__((always_inline)) {
        int m1, n1;
        tile_origin(vnn, m1, n1);
#pragma unroll
        for (int p = 0; p < GA; ++p) off[p] = piece_off<AK, BM, NT>(lda, m1, wave, lane, p);
#pragma unroll
        for (int p = GA; p < G; ++p) off[p] = piece_off<BKC, BN, NT>(ldb, n1, wave, lane, p - GA);
      };
      if constexpr (kLast && !CHAIN) {
        if (vn >= 0) next_offsets(vn);
      }
      block(I0{}, T_{}, F_{}, st, 1, 0, csk, F_{});
      FAN_STAMP(1);
      // (OVL, first K-tile after a transition: K-tile 1 landed, the previous epilogue's stores may stay in flight)
      if (OVL && kt == 0 && !first) waitcnt_known<kS, 0>();
      else waitcnt_known<0, 0>();
      FAN_STAMP(2);
      __builtin_amdgcn_s_barrier();
      FAN_STAMP(3);
      if constexpr (kLast) {
        int vnn = vn;
        if constexpr (CHAIN) {
          chain_decide();
          vnn = ch_cont ? ch_next : -1;
          if (vnn >= 0) next_offsets(vnn);
        }
        // fetch the next tile's first two K-tiles under this k-step's MFMAs (no fragment reads here: both stages
        // are free once every wave passed the barrier above)
        block(I1{}, F_{}, F_{}, smem, 0, 0, csk, T_{}, vnn >= 0);
      } else {
        if constexpr (!decltype(more_c)::value && !decltype(more2_c)::value) chain_decide();
        else chain_hook(kt);
        block(I1{}, more_c, more2_c, smem + ((kt + 1) & 1) * STAGE, 0, kt + 2, csk, F_{});
        // the next K-tile's k-step-0 fragments (read above, long complete): one wait here instead of the compiler's
        // per-fragment ones in front of the next k-step's MFMAs
        if constexpr (decltype(more_c)::value) waitcnt_known<63, 0>();
      }
    } else {
      // DMA of K-tile kt + 2 under k-step 0; the barrier then needs only K-tile kt + 1 (the G younger pieces of
      // kt + 2 may stay in flight)
      block(I0{}, T_{}, more2_c, st, 1, kt + 2, csk, F_{});
      FAN_STAMP(1);
      if constexpr (decltype(more2_c)::value) waitcnt_known<G, 0>();
      else waitcnt_known<0, 0>();
      FAN_STAMP(2);
      __builtin_amdgcn_s_barrier();
      FAN_STAMP(3);
      if constexpr (!decltype(more_c)::value && !decltype(more2_c)::value) chain_decide();
      else chain_hook(kt);
      block(I1{}, more_c, F_{}, smem + ((kt + 1) % 3) * STAGE, 0, 0, csk, F_{});
      if constexpr (decltype(more_c)::value) waitcnt_known<63, 0>();
    }
    FAN_STAMP(4);
  };
  int kt = 0;
  for (; kt + 2 < nk; ++kt) ktile(kt, T_{}, T_{});
  if (kt + 1 < nk) ktile(kt++, T_{}, F_{});
  if (kt < nk) ktile(kt, F_{}, F_{});

  // the last MFMAs' results land in the AGPRs before anything reads them (inline asm: no hazard tracking)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" : "+a"(acc[i][j]));
  if (COLSUM && do_colsum && (!SPLIT || m0 == 0))
    colsum_finish<NJ, WTN, kEpiNone, true>(
        cs, lane, n0 + wn * WTN, ws + (SPLIT ? (int64_t)split_k * M * N + (int64_t)ksplit * N : (int64_t)im * N), wo,
        N);
  if constexpr (OVL) {
    // staging rows of its own (wave-private) beside the operand stages: nothing to wait for (the operand reads
    // retired before the last barrier; the next tile's DMA into the stages must stay in flight)
    store_tile<MI, NJ, WTN, EPI, TC, ACCUM, SPLIT, kSW, WT>(acc, smem + 2 * STAGE, wave, lane, m0 + wm * WTM,
                                                            n0 + wn * WTN, C, ldc, bias, aux, ldaux, M, N, ksplit, ws,
                                                            wo);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every operand read retired before the epilogue reuses the LDS
    store_tile<MI, NJ, WTN, EPI, TC, ACCUM, SPLIT, WTN, WT>(acc, smem, wave, lane, m0 + wm * WTM, n0 + wn * WTN, C,
                                                            ldc, bias, aux, ldaux, M, N, ksplit, ws, wo);
  }
  };
  if constexpr (CHAIN) {
    // this stage's tiles while the next ticket continues it (the OVL transition already fetched its first K-tiles);
    // each finished tile's completion goes to the next tile's K-tile 1 or to the chain loop (chs->pending)
    int v = chs->ticket;
    for (bool first = true;; first = false) {
      tile_body(v, first, -1);
      if (cr.sig_word0 >= 0) {
        int r, c;
        chain_rc(cr, cr.tn, v - cr.first, r, c);
        chs->pending = cr.sig_word0 + r * 16;
      }
      chs->ticket = ch_next;
      chs->ready = ch_rdy;
      if constexpr (!OVL) __syncthreads();  // every wave's staging reads done before the next DMA reuses the LDS
      if (!ch_cont) break;
      v = ch_next;
    }
  } else if constexpr (COLSUM) {
    if (v0 < tiles * split_k) tile_body(v0, true, -1);
  } else {
    for (int v = v0; v < tiles * split_k; v += vstep) {
      tile_body(v, v == v0, v + vstep < tiles * split_k ? v + vstep : -1);
      // every wave's staging reads done before the next tile's DMA overwrites the LDS (OVL: its own staging rows,
      // and a barrier here would drain the next tile's DMA and this tile's stores)
      if constexpr (!OVL) __syncthreads();
    }
  }
}

template <bool AK, bool BKC, int EPI, typename TC, bool ACCUM, bool SPLIT, bool COLSUM = false, int BN_ = 256,
          int BM_ = 256, bool OVL = false>
__global__ void __launch_bounds__(256, 1)
    gemm_pl4_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb,
                    TC* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ bias, const TC* __restrict__ aux,
                    int64_t ldaux, int M, int N, int K, int split_k, float* __restrict__ ws,
                    float* __restrict__ colsum, WireOut wo) {
  pl4_run<AK, BKC, EPI, TC, ACCUM, SPLIT, COLSUM, BN_, BM_, OVL>(A, lda, B, ldb, C, ldc, bias, aux, ldaux, M,
                                                                           N, K, split_k, ws, colsum, wo,
                                                                           (int)blockIdx.x, (int)gridDim.x);
}

// ---------------------------------------------------------------------------------------------------------------
// One GEMM problem of a grouped launch (gemm_groupn_kernel) and its compile-time configuration. (A grouped launch of a
// layer's bwd-data + bwd-weight, the libxsmm PASS_BWD shape, measured no faster than two launches in round 5 and was
// removed: profiles/r5_gemm_bwd_pair_ab.jsonl.)
template <typename TC>
struct PlProblem {
  const bf16_t* A;
  int64_t lda;
  const bf16_t* B;
  int64_t ldb;
  TC* C;
  int64_t ldc;
  const bf16_t* bias;
  const TC* aux;
  int64_t ldaux;
  int M, N, K, split_k;
  float* ws;
  float* colsum;
  WireOut wo;
};

template <bool AK, bool BKC, int EPI, typename TC_, bool ACCUM, bool SPLIT, bool COLSUM, int BN_, int BM_ = 256>
struct PlCfg {
  using TC = TC_;
  static constexpr int kLds = (BN_ == 128 ? 3 : 2) * (BM_ + BN_) * BK * 2;
  static constexpr int kBM = BM_, kBN = BN_;
  __device__ static __forceinline__ void run(const PlProblem<TC>& p, int v0, int vstep) {
    pl4_run<AK, BKC, EPI, TC, ACCUM, SPLIT, COLSUM, BN_, BM_>(p.A, p.lda, p.B, p.ldb, p.C, p.ldc, p.bias, p.aux,
                                                             p.ldaux, p.M, p.N, p.K, p.split_k, p.ws, p.colsum, p.wo,
                                                             v0, vstep);
  }
};

// Grouped launch of up to kMaxGroup GEMMs of ONE configuration P, one tile per workgroup (P with the fused bias
// gradient): problem i owns workgroups [first[i], first[i + 1]), a range padded to a multiple of the XCD count so
// its local tile index keeps blockIdx.x's XCD (xcd_remap); the padding workgroups find no tile and exit. For a
// transformer layer's four bwd-weight GEMMs (dW = X^T . dY over the same tokens): each alone fills a fraction of
// the CUs and needs split-K slabs + a reduce pass, together they fill the chip once (bench/bert_overlap.py).
constexpr int kMaxGroup = 8;
template <typename TC>
struct PlGroup {
  PlProblem<TC> p[kMaxGroup];
  int first[kMaxGroup + 1];
  int n;
};

template <class P>
__global__ void __launch_bounds__(256, 1) gemm_groupn_kernel(PlGroup<typename P::TC> g) {
  const int b = (int)blockIdx.x;
  int i = 0;
  while (i + 1 < g.n && b >= g.first[i + 1]) ++i;  // workgroup-uniform
  P::run(g.p[i], b - g.first[i], g.first[i + 1] - g.first[i]);
}

// Ordered split-K reduction + epilogue (deterministic: slabs summed in split order). SK > 0: the split count as a
// compile-time constant, so every slab's load is issued before the first add (SK = 0: runtime split_k, one slab
// per loop trip).
template <int EPI, typename TC, bool ACCUM, int SK = 0>
__global__ void __launch_bounds__(256)
    splitk_reduce_kernel(const float* __restrict__ ws, int split_k, TC* __restrict__ C, int64_t ldc,
                         const bf16_t* __restrict__ bias, const TC* __restrict__ aux, int64_t ldaux, int M, int N) {
  const int64_t total4 = (int64_t)M * N / 4;
  const int sk = SK > 0 ? SK : split_k;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    const int row = (int)(e / N), col = (int)(e % N);
    float4 s = reinterpret_cast<const float4*>(ws)[i];
#pragma unroll
    for (int k = 1; k < (SK > 0 ? SK : sk); ++k) {
      const float4 t = reinterpret_cast<const float4*>(ws + (int64_t)k * M * N)[i];
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    float v[4] = {s.x, s.y, s.z, s.w};
    epi4<EPI, TC, ACCUM>(v, C, ldc, bias, aux, ldaux, row, col);
  }
}

// Split-K reduction for the wire epilogue: one thread per 16-column group sums the slabs in split order and
// encodes the group into the all-reduce wire (owner shard also in f32). With colsum, the threads past the
// M*N/16 groups reduce the split_k bias partial sums (ws[split_k * M * N + k * N]), write colsum[] and encode the
// bias segment of the [W | b] bucket.
template <bool UPD, int SK = 0>
__global__ void __launch_bounds__(256)
    splitk_reduce_wire_kernel(const float* __restrict__ ws, int split_k, float* __restrict__ C, int64_t ldc, int M,
                              int N, float* __restrict__ colsum, WireOut wo) {
  if constexpr (SK > 0) split_k = SK;  // compile-time split count: the slab loads are issued together
  const int gpr = N / 16;
  const int64_t groups = (int64_t)M * gpr;
  const int64_t total = groups + (colsum ? gpr : 0);
  const int64_t slab = (int64_t)M * N;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const bool bias = g >= groups;
    const int row = bias ? -1 : (int)(g / gpr);
    const int col = (int)((bias ? g - groups : g % gpr) * 16);
    const float* p = bias ? ws + (int64_t)split_k * slab + col : ws + (int64_t)row * N + col;
    const int64_t stride = bias ? N : slab;
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; u += 4) {
      const float4 q = *reinterpret_cast<const float4*>(p + u);
      v[u] = q.x; v[u + 1] = q.y; v[u + 2] = q.z; v[u + 3] = q.w;
    }
#pragma unroll
    for (int k = 1; k < (SK > 0 ? SK : split_k); ++k) {
#pragma unroll
      for (int u = 0; u < 16; u += 4) {
        const float4 q = *reinterpret_cast<const float4*>(p + k * stride + u);
        v[u] += q.x; v[u + 1] += q.y; v[u + 2] += q.z; v[u + 3] += q.w;
      }
    }
    if (!bias) {
      wire_epi16<UPD>(v, C, ldc, wo, row, col);
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u) colsum[col + u] = v[u];
      if (wo.bias_off > 0) wire_store16<UPD>(v, (uint32_t)wo.bias_off + (uint32_t)col, wo);
    }
  }
}

// Bias-gradient reduces of several GEMMs (colsum_reduce_group_kernel, splitk_reduce_wire4_kernel QCS).
struct ColsumGroup {
  const float* part[kMaxGroup];
  float* colsum[kMaxGroup];
  WireOut wo[kMaxGroup];
  int parts[kMaxGroup];
  int N[kMaxGroup];
  int first[kMaxGroup + 1];
  int n;
};
template <bool WIRE, bool UPD>
__device__ __forceinline__ void colsum_reduce_block(const float* __restrict__ part, int parts,
                                                    float* __restrict__ colsum, int N, const WireOut& wo, int blk);

// The fused update of 4 values of a group (flat index f, f % 4 == 0; shared exponent E): local_update16's operations
// on a quarter of the group.
__device__ __forceinline__ void local_update4(float v[4], uint32_t E, uint32_t f, const WireOut& wo) {
  float4 a = *reinterpret_cast<const float4*>(wo.um + f);
  float w[4] = {a.x, a.y, a.z, a.w}, m[4] = {0.f, 0.f, 0.f, 0.f};
  const bool hm = wo.umom != nullptr;
  if (hm) {
    const float4 b = *reinterpret_cast<const float4*>(wo.umom + f);
    m[0] = b.x; m[1] = b.y; m[2] = b.z; m[3] = b.w;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) sgd_apply(wire_roundtrip_rne(v[u], E), w[u], m[u], hm, wo.up);
  *reinterpret_cast<float4*>(wo.um + f) = make_float4(w[0], w[1], w[2], w[3]);
  if (hm) *reinterpret_cast<float4*>(wo.umom + f) = make_float4(m[0], m[1], m[2], m[3]);
  if (wo.ulp) *reinterpret_cast<uint2*>(wo.ulp + f) = make_uint2(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]));
}

// splitk_reduce_wire_kernel, lane-contiguous: each lane sums and finishes 4 consecutive values (one float4 per slab),
// 4 lanes a 16-column group, so every load and store of a wave covers 1 KiB contiguous (one lane per group strides
// 64 B per lane). The group's shared exponent is the max over its 4 lanes (quad xor shuffles: exact), and every
// value is summed in split order, encoded, rounded and updated as there: bit-identical. The bias partials (colsum)
// are reduced per 16-column group after the loop, as there. (M * N / 4 is a multiple of 4 — N % 16 == 0 — and the
// grid's thread count too, so a quad's lanes are always all in or all out of range.)
// QCS: the launch also runs bias-gradient reduces that earlier fused-update GEMMs of the stream queued (qcs, in its
// first qcs.first[qcs.n] blocks: one launch less per queued reduce, GemmArgs::defer_colsum).
template <bool UPD, int SK = 0, bool QCS = false>
__global__ void __launch_bounds__(256)
    splitk_reduce_wire4_kernel(const float* __restrict__ ws, int split_k, float* __restrict__ C, int64_t ldc, int M,
                               int N, float* __restrict__ colsum, WireOut wo, ColsumGroup qcs) {
  int bid = (int)blockIdx.x, nb = (int)gridDim.x;
  if constexpr (QCS) {
    const int nq = qcs.first[qcs.n];
    if (bid < nq) {
      int i = 0;
      while (i + 1 < qcs.n && bid >= qcs.first[i + 1]) ++i;
      colsum_reduce_block<true, true>(qcs.part[i], qcs.parts[i], qcs.colsum[i], qcs.N[i], qcs.wo[i],
                                      bid - qcs.first[i]);
      return;
    }
    bid -= nq;
    nb -= nq;
  }
  if constexpr (SK > 0) split_k = SK;
  const int64_t slab = (int64_t)M * N, quads = slab / 4;
  const int64_t t0 = bid * (int64_t)blockDim.x + threadIdx.x, step = (int64_t)nb * blockDim.x;
  for (int64_t q = t0; q < quads; q += step) {
    const int64_t e = q * 4;
    const int row = (int)(e / N), col = (int)(e % N);
    float4 a = *reinterpret_cast<const float4*>(ws + e);
#pragma unroll
    for (int k = 1; k < (SK > 0 ? SK : split_k); ++k) {
      const float4 b = *reinterpret_cast<const float4*>(ws + k * slab + e);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
    uint32_t mx = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) mx = max(mx, __float_as_uint(v[u]) & 0x7FFFFFFFu);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, 1));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, 2));
    const uint32_t E = mx >> 23;
    const uint32_t loc = (uint32_t)row * (uint32_t)ldc + (uint32_t)col;
    if constexpr (UPD) {
      local_update4(v, E, wo.off + loc, wo);
    } else {
      const int sub = (col & 15) >> 2;
      const uint32_t fg = wo.off + loc - 4u * (uint32_t)sub;  // the group's flat index
      const int sh = wire_shard_of(fg, wo);
      const uint32_t pos = fg - (uint32_t)sh * (uint32_t)wo.shard;
      uint32_t w = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) w |= ((uint32_t)wire_encode(v[u], E, wo.codec) & 0xFFu) << (8 * u);
      uint8_t* base = wire_shard_base(sh, wo);
      *reinterpret_cast<uint32_t*>(base + pos + 4 * sub) = w;
      if (sub == 0) base[wo.shard + pos / 16] = (uint8_t)E;
      if (wo.own == kWireOwnAll || (wo.period > 0 ? sh % wo.period : sh) == wo.own)
        *reinterpret_cast<float4*>(C + loc) = a;
    }
  }
  if (colsum) {
    for (int64_t g = t0; g < N / 16; g += step) {
      const int col = (int)g * 16;
      const float* p = ws + (int64_t)split_k * slab + col;
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; u += 4) {
        const float4 b = *reinterpret_cast<const float4*>(p + u);
        v[u] = b.x; v[u + 1] = b.y; v[u + 2] = b.z; v[u + 3] = b.w;
      }
      for (int k = 1; k < split_k; ++k) {
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
          const float4 b = *reinterpret_cast<const float4*>(p + (int64_t)k * N + u);
          v[u] += b.x; v[u + 1] += b.y; v[u + 2] += b.z; v[u + 3] += b.w;
        }
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) colsum[col + u] = v[u];
      if (wo.bias_off > 0) wire_store16<UPD>(v, (uint32_t)wo.bias_off + (uint32_t)col, wo);
    }
  }
}

// Ordered reduce of bias-gradient partial slabs part[p * N + n], p < parts, into colsum[n]; WIRE: also encodes the
// bias segment of the [W | b] bucket (flat wo.bias_off + n). One block per 64 columns: 16 lanes x float4 columns by
// 16 part classes (p % 16), each summed in p order, then the classes summed in class order (deterministic).
template <bool WIRE, bool UPD>
__device__ __forceinline__ void colsum_reduce_block(const float* __restrict__ part, int parts,
                                                    float* __restrict__ colsum, int N, const WireOut& wo, int blk) {
  __shared__ float4 red[16][16];
  __shared__ float fin[64];
  const int t = threadIdx.x, cg = t & 15, pc = t >> 4;
  const int col = blk * 64 + cg * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < N) {
    for (int p = pc; p < parts; p += 16) {
      const float4 q = *reinterpret_cast<const float4*>(part + (int64_t)p * N + col);
      acc.x += q.x; acc.y += q.y; acc.z += q.z; acc.w += q.w;
    }
  }
  red[pc][cg] = acc;
  __syncthreads();
  if (t < 16) {
    float4 s = red[0][t];
    for (int c = 1; c < 16; ++c) {
      const float4 q = red[c][t];
      s.x += q.x; s.y += q.y; s.z += q.z; s.w += q.w;
    }
    fin[t * 4] = s.x; fin[t * 4 + 1] = s.y; fin[t * 4 + 2] = s.z; fin[t * 4 + 3] = s.w;
    if (col < N) *reinterpret_cast<float4*>(colsum + col) = s;
  }
  if constexpr (WIRE) {
    __syncthreads();
    const int c16 = blk * 64 + t * 16;
    if (t < 4 && c16 < N && wo.bias_off > 0) {  // N % 16 == 0
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = fin[t * 16 + u];
      wire_store16<UPD>(v, (uint32_t)wo.bias_off + (uint32_t)c16, wo);
    }
  }
}

template <bool WIRE, bool UPD = false>
__global__ void __launch_bounds__(256)
    colsum_reduce_kernel(const float* __restrict__ part, int parts, float* __restrict__ colsum, int N, WireOut wo) {
  colsum_reduce_block<WIRE, UPD>(part, parts, colsum, N, wo, (int)blockIdx.x);
}

// Bias gradients of several GEMMs in one launch — the grouped GEMM's problems, or the bias-gradient reduces that
// fused-update bwd-weight GEMMs queued (GemmArgs::defer_colsum): entry i's blocks [first[i], first[i + 1]) reduce its
// partial slabs, the same ordered reduce as colsum_reduce_kernel (bit-identical).
template <bool WIRE, bool UPD = false>
__global__ void __launch_bounds__(256) colsum_reduce_group_kernel(ColsumGroup g) {
  const int b = (int)blockIdx.x;
  int i = 0;
  while (i + 1 < g.n && b >= g.first[i + 1]) ++i;
  colsum_reduce_block<WIRE, UPD>(g.part[i], g.parts[i], g.colsum[i], g.N[i], g.wo[i], b - g.first[i]);
}

}  // namespace gemm_detail
}  // namespace fan

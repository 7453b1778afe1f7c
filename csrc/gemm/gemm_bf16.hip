// bf16 MFMA GEMM for gfx950 (v_mfma_f32_16x16x32_bf16), LDS-tiled, global_load_lds staged.
//
// Block tile 128x128x64, 256 threads = 4 waves in a 2x2 arrangement, each wave a 64x64 sub-tile
// (4x4 MFMA 16x16 tiles = 64 accumulator VGPRs). Operand tiles are staged global->LDS with
// global_load_lds_dwordx4 (no VGPR round trip) into a double-buffered LDS ring (64 KiB):
//   K-contiguous operand  : LDS image [128 rows][64 k] (128-B rows), 16-B chunk c of row r stored at
//                           c ^ ((r>>1)&7)  -> ds_read_b128 fragment reads are conflict-free.
//   MN-contiguous operand : LDS image [64 k][128 cols] (256-B rows), 32-B block b of row k stored at
//                           b ^ ((k&3) | ((k>>3)&1)<<2) -> ds_read_b64_tr_b16 (hardware transpose)
//                           fragment reads are conflict-free.
// glds writes LDS linearly (wave base + lane*16), so the swizzle is applied to the per-lane GLOBAL
// source address and the matching XOR on the read (both sides, one involution).
// Workgroup -> tile mapping is XCD-aware: the 8 round-robin XCD groups each get a contiguous
// run of tiles so neighbouring tiles (shared A rows) hit the same L2.
#include "gemm/gemm.h"

namespace fan {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // one operand tile (16 KiB)
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;  // 64 KiB

__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// Stage one operand tile (outer extent 128 starting at o0, k extent 64 starting at k0).
template <bool KCONTIG>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ g, int64_t ld, int o0, int k0, char* lds_tile,
                                           int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = wave * 64 + lane;  // 0..255 within this block-instruction
    const bf16_t* src;
    if (KCONTIG) {
      const int row = i * 32 + (t >> 3);
      const int cs = t & 7;
      const int c = cs ^ ((row >> 1) & 7);
      src = g + (int64_t)(o0 + row) * ld + k0 + c * 8;
    } else {
      const int krow = i * 16 + (t >> 4);
      const int cs = t & 15;
      const int blk = (cs >> 1) ^ mn_swz(krow);
      src = g + (int64_t)(k0 + krow) * ld + o0 + blk * 16 + (cs & 1) * 8;
    }
    char* dst = lds_tile + i * 4096 + wave * 1024;  // wave-uniform base; hw adds lane*16
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)dst, 16, 0, 0);
  }
}

// Fragment (8 bf16 along k) for a 16-row/col subtile at outer offset o (within the tile), k-step ks.
template <bool KCONTIG>
__device__ __forceinline__ s16x8 read_frag(const char* lds_tile, int o, int ks, int lane) {
  if (KCONTIG) {
    const int row = o + (lane & 15);
    const int chunk = ks * 4 + (lane >> 4);
    const int off = row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
    return *reinterpret_cast<const s16x8*>(lds_tile + off);
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int kb = ks * 32 + 8 * (lane >> 4) + q;
    const int blk = o >> 4;
    const int off0 = kb * 256 + ((blk ^ mn_swz(kb)) << 5) + 8 * p;
    const int off1 = (kb + 4) * 256 + ((blk ^ mn_swz(kb + 4)) << 5) + 8 * p;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(lds_tile + off0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(lds_tile + off1));
    s16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % kNumXCD;
  const int q = nwg / kNumXCD, r = nwg % kNumXCD;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / kNumXCD;
}

template <typename TC>
__device__ __forceinline__ void store_c(TC* p, float v);
template <>
__device__ __forceinline__ void store_c<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void store_c<bf16_t>(bf16_t* p, float v) { *p = f32_to_bf16(v); }

template <typename TC>
__device__ __forceinline__ float load_c(const TC* p);
template <>
__device__ __forceinline__ float load_c<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float load_c<bf16_t>(const bf16_t* p) { return bf16_to_f32(*p); }

template <bool AK, bool BKC, int EPI, typename TC, bool ACCUM, bool SPLIT>
__global__ void __launch_bounds__(NT, 2)
    gemm_bf16_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb,
                     TC* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ bias, const TC* __restrict__ aux,
                     int64_t ldaux, int M, int N, int K, int split_k, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = N / BN;
  const int tiles = (M / BM) * tiles_n;
  const int nwg = tiles * split_k;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tile = wg % tiles;
  const int ksplit = wg / tiles;
  const int m0 = (tile / tiles_n) * BM;
  const int n0 = (tile % tiles_n) * BN;
  const int k_per = K / split_k;
  const int kbeg = ksplit * k_per;
  const int nk = k_per / BK;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue
  stage_tile<AK>(A, lda, m0, kbeg, smem, wave, lane);
  stage_tile<BKC>(B, ldb, n0, kbeg, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    char* sa = smem + cur * STAGE_BYTES;
    char* sb = sa + TILE_BYTES;
    if (kt + 1 < nk) {
      char* na = smem + (cur ^ 1) * STAGE_BYTES;
      stage_tile<AK>(A, lda, m0, kbeg + (kt + 1) * BK, na, wave, lane);
      stage_tile<BKC>(B, ldb, n0, kbeg + (kt + 1) * BK, na + TILE_BYTES, wave, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<AK>(sa, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BKC>(sb, wn * 64 + j * 16, ks, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                              __builtin_bit_cast(bf16x8, bfr[j]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds rows (lane>>4)*4 + r, column lane&15 of each 16x16 tile
  const int col_l = lane & 15;
  const int row_l = (lane >> 4) * 4;
  if (SPLIT) {
    float* slab = ws + (int64_t)ksplit * M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + col_l;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 64 + i * 16 + row_l + r;
          slab[(int64_t)row * N + col] = acc[i][j][r];
        }
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + col_l;
    float bv = 0.f;
    if (EPI == kEpiBias || EPI == kEpiBiasRelu) bv = bf16_to_f32(bias[col]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + row_l + r;
        float v = acc[i][j][r];
        if (EPI == kEpiBias || EPI == kEpiBiasRelu) v += bv;
        if (EPI == kEpiBiasRelu) v = fmaxf(v, 0.f);
        if (EPI == kEpiReluMask) v = load_c<TC>(aux + (int64_t)row * ldaux + col) > 0.f ? v : 0.f;
        TC* p = C + (int64_t)row * ldc + col;
        if (ACCUM) v += load_c<TC>(p);
        store_c<TC>(p, v);
      }
    }
  }
}

// Ordered split-K reduction + epilogue (deterministic: slabs summed in split order).
template <int EPI, typename TC, bool ACCUM>
__global__ void __launch_bounds__(256)
    splitk_reduce_kernel(const float* __restrict__ ws, int split_k, TC* __restrict__ C, int64_t ldc,
                         const bf16_t* __restrict__ bias, const TC* __restrict__ aux, int64_t ldaux, int M, int N) {
  const int64_t total4 = (int64_t)M * N / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    const int row = (int)(e / N), col = (int)(e % N);
    float4 s = reinterpret_cast<const float4*>(ws)[i];
    for (int k = 1; k < split_k; ++k) {
      const float4 t = reinterpret_cast<const float4*>(ws + (int64_t)k * M * N)[i];
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    float v[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (EPI == kEpiBias || EPI == kEpiBiasRelu) v[u] += bf16_to_f32(bias[col + u]);
      if (EPI == kEpiBiasRelu) v[u] = fmaxf(v[u], 0.f);
      if (EPI == kEpiReluMask) v[u] = load_c<TC>(aux + (int64_t)row * ldaux + col + u) > 0.f ? v[u] : 0.f;
      TC* p = C + (int64_t)row * ldc + col + u;
      if (ACCUM) v[u] += load_c<TC>(p);
      store_c<TC>(p, v[u]);
    }
  }
}

template <bool AK, bool BKC, int EPI, typename TC, bool ACCUM>
void launch_typed(const GemmArgs& a, hipStream_t s) {
  const int tiles = (a.M / BM) * (a.N / BN);
  const int sk = a.split_k > 1 ? a.split_k : 1;
  const int grid = tiles * sk;
  if (sk > 1) {
    hipLaunchKernelGGL((gemm_bf16_kernel<AK, BKC, EPI, TC, ACCUM, true>), grid, NT, LDS_BYTES, s,
                       (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb, (TC*)a.C, a.ldc,
                       (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, sk, (float*)a.workspace);
    hipLaunchKernelGGL((splitk_reduce_kernel<EPI, TC, ACCUM>), stream_grid((size_t)a.M * a.N / 4), 256, 0, s,
                       (const float*)a.workspace, sk, (TC*)a.C, a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux,
                       a.ldaux, a.M, a.N);
  } else {
    hipLaunchKernelGGL((gemm_bf16_kernel<AK, BKC, EPI, TC, ACCUM, false>), grid, NT, LDS_BYTES, s,
                       (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb, (TC*)a.C, a.ldc,
                       (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, 1, (float*)nullptr);
  }
}

template <bool AK, bool BKC>
void launch_layout(const GemmArgs& a, hipStream_t s) {
#define FAN_EPI_CASE(E)                                                       \
  case E:                                                                     \
    if (a.c_bf16) {                                                           \
      launch_typed<AK, BKC, E, bf16_t, false>(a, s);                          \
    } else if (a.accumulate) {                                                \
      launch_typed<AK, BKC, E, float, true>(a, s);                            \
    } else {                                                                  \
      launch_typed<AK, BKC, E, float, false>(a, s);                           \
    }                                                                         \
    break;
  switch (a.epilogue) {
    FAN_EPI_CASE(kEpiNone)
    FAN_EPI_CASE(kEpiBias)
    FAN_EPI_CASE(kEpiBiasRelu)
    FAN_EPI_CASE(kEpiReluMask)
    default: FAN_CHECK(false, "bad epilogue");
  }
#undef FAN_EPI_CASE
}

}  // namespace

bool gemm_bf16_supported(const GemmArgs& a) {
  const int sk = a.split_k > 1 ? a.split_k : 1;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
  if (a.M % BM || a.N % BN || a.K % (BK * sk)) return false;
  // 16-byte alignment of every staged row (glds dwordx4) and of the bases.
  if (a.lda % 8 || a.ldb % 8) return false;
  if (((uintptr_t)a.A | (uintptr_t)a.B) & 15) return false;
  if (a.accumulate && a.c_bf16) return false;
  if (sk > 1 && (a.workspace == nullptr || (a.N % 4) || (a.ldc != a.N))) return false;
  return true;
}

void launch_gemm_bf16(const GemmArgs& a, hipStream_t s) {
  FAN_CHECK(gemm_bf16_supported(a), "gemm_bf16: unsupported shape/layout (need M,N % 128 == 0, K % 64 == 0)");
  static bool attr_set = false;
  (void)attr_set;
  if (a.a_kcontig && a.b_kcontig) launch_layout<true, true>(a, s);
  else if (a.a_kcontig && !a.b_kcontig) launch_layout<true, false>(a, s);
  else if (!a.a_kcontig && a.b_kcontig) launch_layout<false, true>(a, s);
  else launch_layout<false, false>(a, s);
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace fan

// fp32 MFMA GEMM for gfx950 (v_mfma_f32_16x16x4_f32: exact f32 fma chain, no xf32 on CDNA4).
//
// Serves the reference-equivalent f32 MLP (sw/mlp_mpi_example_f32.cpp: libxsmm fc fwd/bwd in f32).
// Block tile 128x128x32, 4 waves (2x2), each wave 64x64 = 4x4 tiles of 16x16. Both operands are staged with
// global_load_lds_dwordx4 (no VGPR round trip, no synchronous register staging), swizzle on the source address:
//   * K-contiguous operand: LDS image [outer][k] (128-B rows of 32 f32), 16-B chunk c of row r at c ^ ((r>>1)&7);
//     a fragment is one ds_read_b128;
//   * MN-contiguous operand: LDS image [k][outer] (512-B rows of 128 f32), 16-float block b of row k at
//     b ^ ((k>>2)&3); a fragment is 4 ds_read_b32 (lanes of the 4 k-row groups hit 4 disjoint bank quarters).
// Within each 16-wide k chunk lane l feeds k = 4*(l>>4) + i to MFMA i (a consistent permutation of the k order
// for A and B).
// Any M, N, K that are multiples of 8: tiles are ceil-divided; a workgroup whose tile crosses an operand edge stages
// its out-of-range 16-B chunks from a zero page and stores only in-range elements (the reference's libxsmm
// blocking falls back to whole dimensions, sw/mlp_mpi_example_f32.cpp:498-506, so any MB / C works there).
#include "gemm/gemm.h"
#include "gemm/glds.h"

namespace fan {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int TILE_BYTES = 128 * BK * 4;  // 16 KiB
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

static __device__ __attribute__((aligned(256))) uint4 g_f32_zero16[16];  // zero page for edge-tile chunks

// EDGE: 16-B chunks at outer >= o_lim or k >= k_lim (multiples of 4 floats) load the zero page instead.
template <bool KCONTIG, bool EDGE = false>
__device__ __forceinline__ void stage(const float* __restrict__ g, int64_t ld, int o0, int k0, char* tile, int wave,
                                      int lane, int o_lim = 0, int k_lim = 0) {
  const int t = wave * 64 + lane;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float* src;
    bool out = false;
    if (KCONTIG) {
      const int row = i * 32 + (t >> 3);
      const int c = (t & 7) ^ swz(row);
      src = g + (int64_t)(o0 + row) * ld + k0 + c * 4;
      if (EDGE) out = o0 + row >= o_lim || k0 + c * 4 >= k_lim;
    } else {
      const int krow = i * 8 + (t >> 5);
      const int col = ((t & 31) * 4) ^ (((krow >> 2) & 3) << 4);
      src = g + (int64_t)(k0 + krow) * ld + o0 + col;
      if (EDGE) out = k0 + krow >= k_lim || o0 + col >= o_lim;
    }
    if (EDGE && out) src = reinterpret_cast<const float*>(g_f32_zero16);
    glds16((const void*)src, __builtin_amdgcn_readfirstlane(lds_addr_of(tile + i * 4096 + wave * 1024)));
  }
}

template <bool KCONTIG>
__device__ __forceinline__ f32x4 frag(const char* tile, int o, int kc, int lane) {
  if (KCONTIG) {
    const int row = o + (lane & 15);
    const int c = kc * 4 + (lane >> 4);
    return *reinterpret_cast<const f32x4*>(tile + row * 128 + ((c ^ swz(row)) << 4));
  } else {
    const int k0 = kc * 16 + 4 * (lane >> 4);
    const int col = (o + (lane & 15)) ^ ((lane >> 4) << 4);  // (k >> 2) & 3 == lane >> 4 for k0..k0+3
    f32x4 r;
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = *reinterpret_cast<const float*>(tile + (k0 + u) * 512 + col * 4);
    return r;
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % kNumXCD;
  const int q = nwg / kNumXCD, r = nwg % kNumXCD;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / kNumXCD;
}

template <bool AK, bool BKC, int EPI, bool ACCUM>
__global__ void __launch_bounds__(NT, 2)
    gemm_f32_kernel(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
                    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, const float* __restrict__ aux,
                    int64_t ldaux, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = (N + BN - 1) / BN;
  const int nwg = ((M + BM - 1) / BM) * tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nk = (K + BK - 1) / BK;
  const bool mn_edge = m0 + BM > M || n0 + BN > N;
  const bool edge = mn_edge || K % BK;  // uniform: predicated staging for this workgroup
  auto stage_ab = [&](int k0, char* dst) {
    if (edge) {
      stage<AK, true>(A, lda, m0, k0, dst, wave, lane, M, K);
      stage<BKC, true>(B, ldb, n0, k0, dst + TILE_BYTES, wave, lane, N, K);
    } else {
      stage<AK>(A, lda, m0, k0, dst, wave, lane);
      stage<BKC>(B, ldb, n0, k0, dst + TILE_BYTES, wave, lane);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage_ab(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    char* sa = smem + cur * STAGE_BYTES;
    char* sb = sa + TILE_BYTES;
    if (kt + 1 < nk) {
      stage_ab((kt + 1) * BK, smem + (cur ^ 1) * STAGE_BYTES);
    }
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      f32x4 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<AK>(sa, wm * 64 + i * 16, kc, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BKC>(sb, wn * 64 + j * 16, kc, lane);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][u], bfr[j][u], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + col_l;
    if (mn_edge && col >= N) continue;
    const float bv = (EPI == kEpiBias || EPI == kEpiBiasRelu) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + row_l + r;
        if (mn_edge && row >= M) continue;
        float v = acc[i][j][r] + bv;
        if (EPI == kEpiBiasRelu) v = fmaxf(v, 0.f);
        if (EPI == kEpiReluMask) v = aux[(int64_t)row * ldaux + col] > 0.f ? v : 0.f;
        float* p = C + (int64_t)row * ldc + col;
        if (ACCUM) v += *p;
        *p = v;
      }
  }
}

template <bool AK, bool BKC>
void launch_layout(const GemmArgs& a, hipStream_t s) {
  const int grid = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
#define FAN_F32_CASE(E)                                                                                       \
  case E:                                                                                                     \
    if (a.accumulate)                                                                                         \
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKC, E, true>), grid, NT, LDS_BYTES, s, (const float*)a.A, a.lda, \
                         (const float*)a.B, a.ldb, (float*)a.C, a.ldc, (const float*)a.bias, (const float*)a.aux,    \
                         a.ldaux, a.M, a.N, a.K);                                                            \
    else                                                                                                      \
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKC, E, false>), grid, NT, LDS_BYTES, s, (const float*)a.A, a.lda, \
                         (const float*)a.B, a.ldb, (float*)a.C, a.ldc, (const float*)a.bias, (const float*)a.aux,     \
                         a.ldaux, a.M, a.N, a.K);                                                             \
    break;
  switch (a.epilogue) {
    FAN_F32_CASE(kEpiNone)
    FAN_F32_CASE(kEpiBias)
    FAN_F32_CASE(kEpiBiasRelu)
    FAN_F32_CASE(kEpiReluMask)
    default: FAN_CHECK(false, "bad epilogue");
  }
#undef FAN_F32_CASE
}

}  // namespace

bool gemm_f32_supported(const GemmArgs& a) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
  if (a.M % 8 || a.N % 8 || a.K % 8) return false;
  if (a.lda % 4 || a.ldb % 4) return false;
  if (((uintptr_t)a.A | (uintptr_t)a.B) & 15) return false;
  if (a.c_bf16 || a.split_k > 1) return false;
  return true;
}

void launch_gemm_f32(const GemmArgs& a, hipStream_t s) {
  FAN_CHECK(gemm_f32_supported(a), "gemm_f32: unsupported shape/layout (need M, N, K % 8 == 0)");
  if (a.a_kcontig && a.b_kcontig) launch_layout<true, true>(a, s);
  else if (a.a_kcontig) launch_layout<true, false>(a, s);
  else if (a.b_kcontig) launch_layout<false, true>(a, s);
  else launch_layout<false, false>(a, s);
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace fan

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

// SPLIT: K split over split_k workgroups per tile (ragged ranges of K-tiles); each writes its raw f32 partial
// tile to slab ws[ksplit][M][N] and f32_splitk_reduce_kernel sums the slabs in split order (deterministic) and
// applies the epilogue. Small output grids (the reference workload's 672 / 448-row batches) fill the CUs this way.
template <bool AK, bool BKC, int EPI, bool ACCUM, bool SPLIT>
__global__ void __launch_bounds__(NT, 2)
    gemm_f32_kernel(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
                    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, const float* __restrict__ aux,
                    int64_t ldaux, int M, int N, int K, int split_k, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = (N + BN - 1) / BN;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int wg = xcd_remap(blockIdx.x, tiles * split_k);
  const int tile = wg % tiles, ksplit = wg / tiles;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nkt = (K + BK - 1) / BK;
  const int kt_per = (nkt + split_k - 1) / split_k;
  const int kt0 = ksplit * kt_per;
  const int nk = max(0, min(nkt, kt0 + kt_per) - kt0);
  const int kbeg = kt0 * BK;
  const bool mn_edge = m0 + BM > M || n0 + BN > N;
  const bool edge = mn_edge || (kt0 + nk) * BK > K;  // uniform: predicated staging for this workgroup
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

  if (nk > 0) stage_ab(kbeg, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    char* sa = smem + cur * STAGE_BYTES;
    char* sb = sa + TILE_BYTES;
    if (kt + 1 < nk) {
      stage_ab(kbeg + (kt + 1) * BK, smem + (cur ^ 1) * STAGE_BYTES);
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
    const float bv = (!SPLIT && (EPI == kEpiBias || EPI == kEpiBiasRelu)) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + row_l + r;
        if (mn_edge && row >= M) continue;
        if (SPLIT) {
          ws[((int64_t)ksplit * M + row) * N + col] = acc[i][j][r];
          continue;
        }
        float v = acc[i][j][r] + bv;
        if (EPI == kEpiBiasRelu) v = fmaxf(v, 0.f);
        if (EPI == kEpiReluMask) v = aux[(int64_t)row * ldaux + col] > 0.f ? v : 0.f;
        float* p = C + (int64_t)row * ldc + col;
        if (ACCUM) v += *p;
        *p = v;
      }
  }
}

// Ordered split-K reduction (slabs summed in split order) + the f32 epilogue.
template <int EPI, bool ACCUM>
__global__ void __launch_bounds__(256)
    f32_splitk_reduce_kernel(const float* __restrict__ ws, int split_k, float* __restrict__ C, int64_t ldc,
                             const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux, int M, int N) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(e / N), col = (int)(e % N);
    float v = ws[e];
    for (int k = 1; k < split_k; ++k) v += ws[(int64_t)k * total + e];
    if (EPI == kEpiBias || EPI == kEpiBiasRelu) v += bias[col];
    if (EPI == kEpiBiasRelu) v = fmaxf(v, 0.f);
    if (EPI == kEpiReluMask) v = aux[(int64_t)row * ldaux + col] > 0.f ? v : 0.f;
    float* p = C + (int64_t)row * ldc + col;
    if (ACCUM) v += *p;
    *p = v;
  }
}

template <bool AK, bool BKC, int EPI, bool ACCUM>
void launch_typed(const GemmArgs& a, int sk, hipStream_t s) {
  const int grid = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * sk;
  if (sk > 1) {
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKC, EPI, ACCUM, true>), grid, NT, LDS_BYTES, s, (const float*)a.A, a.lda,
                       (const float*)a.B, a.ldb, (float*)a.C, a.ldc, (const float*)a.bias, (const float*)a.aux, a.ldaux,
                       a.M, a.N, a.K, sk, (float*)a.workspace);
    hipLaunchKernelGGL((f32_splitk_reduce_kernel<EPI, ACCUM>), stream_grid((size_t)a.M * a.N), 256, 0, s,
                       (const float*)a.workspace, sk, (float*)a.C, a.ldc, (const float*)a.bias, (const float*)a.aux,
                       a.ldaux, a.M, a.N);
  } else {
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BKC, EPI, ACCUM, false>), grid, NT, LDS_BYTES, s, (const float*)a.A,
                       a.lda, (const float*)a.B, a.ldb, (float*)a.C, a.ldc, (const float*)a.bias, (const float*)a.aux,
                       a.ldaux, a.M, a.N, a.K, 1, nullptr);
  }
}

template <bool AK, bool BKC>
void launch_layout(const GemmArgs& a, hipStream_t s) {
  const int sk = gemm_f32_split(a.M, a.N, a.K, a.split_k);
#define FAN_F32_CASE(E)                                         \
  case E:                                                       \
    if (a.accumulate) launch_typed<AK, BKC, E, true>(a, sk, s); \
    else launch_typed<AK, BKC, E, false>(a, sk, s);             \
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

int gemm_f32_split(int M, int N, int K, int split_k) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int nkt = (K + BK - 1) / BK;
  if (split_k > 0) return std::min(split_k, std::max(1, nkt));
  int sk = 1;  // split K only when the output grid leaves more than half of the CUs idle
  if (tiles * 2 <= kNumCU)
    while (tiles * sk < kNumCU && sk < 8 && nkt / (sk * 2) >= 8) sk *= 2;
  return sk;
}

bool gemm_f32_supported(const GemmArgs& a) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
  if (a.M % 8 || a.N % 8 || a.K % 8) return false;
  if (a.lda % 4 || a.ldb % 4) return false;
  if (((uintptr_t)a.A | (uintptr_t)a.B) & 15) return false;
  if (a.c_bf16 || a.epilogue == kEpiWire || a.colsum) return false;
  if (gemm_f32_split(a.M, a.N, a.K, a.split_k) > 1 && a.workspace == nullptr) return false;
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

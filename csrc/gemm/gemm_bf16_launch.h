// Host-side launch logic of the bf16 MFMA GEMMs (gemm_bf16_kernel.h holds the kernels): main-loop selection per
// tile shape and layout, the persistent grid cap, split-K slab reduces and the bias-gradient reduce, and the
// compile-time dispatch over tiles and epilogues. Included by the explicit-instantiation TUs (gemm_bf16_l*.hip) and
// the planner (gemm_bf16_plan.hip).
#pragma once

#include "gemm/gemm_bf16_kernel.h"

namespace fan {
namespace gemm_detail {

template <int BM, int BN>
constexpr int lds_bytes() {
  constexpr int st = (BM + BN) * BK * 2;
  return ((3 * st <= 160 * 1024) ? 3 : 2) * st;
}

// 256x256 main loop selection (gemm_main_loop_flag(): 0 one-role, 2 pipelined (4 or 8 waves by layout / K),
// 3 pipelined 4-wave, 5 pipelined 8-wave), read per launch so A/B comparisons run in one process. (A staggered
// two-group loop, mode 1 in round 1, measured within ±5 % of the one-role loop and was removed:
// profiles/r1_gemm_experiments.md.)
inline int main_loop_mode() { return gemm_main_loop_flag().load(std::memory_order_relaxed); }
// grid of the persistent 4-wave kernel: at most gemm_persist_flag() workgroups (<= 0: one per tile)
inline int persist_grid(int grid) {
  const int cap = gemm_persist_flag().load(std::memory_order_relaxed);
  return cap > 0 && grid > cap ? cap : grid;
}

// Launches the main loop; returns the number of bias-gradient partial slabs it left in the workspace for an ordered
// reduce (split_k with split-K; without: the pipelined loop's tile rows, 0 = colsum written by the kernel).
template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI, typename TC, bool ACCUM, bool SPLIT>
int launch_main(const GemmArgs& a, int sk, const WireOut& wo, hipStream_t s) {
  const int grid = cdiv_i(a.M, BM) * cdiv_i(a.N, BN) * sk;
  if constexpr (BM == 256 && BN == 256 && WM * WN == 8) {
    // the pipelined loops have no edge path: aligned shapes only
    const int mode = main_loop_mode();
    const bool aligned = a.M % BM == 0 && a.N % BN == 0 && a.K % (BK * sk) == 0;
    // pipelined loops: 4 waves (128x128 per wave, AGPR accumulators) where they measured faster — an MN-contiguous
    // B, or a long K — else 8 waves: the 4-wave epilogue runs on half the waves (bwd-data at K 1024: 77 vs 70 us;
    // the in-kernel wire encode: bwd-weight 4096^2 +13 vs +7 us, profiles/r1_gemm_experiments.md); modes 3 / 5
    // force one of them
    // (the MLP's bwd-data with the ReLU-mask epilogue, activation loads prefetched: 4 waves 197 vs 200 us at
    // 8192x4096x4096, 67.9 vs 68.5 at K 1024, profiles/r2_gemm_loops_bwdd.jsonl)
    // (and the in-kernel wire encode: since the 4-wave kernel became persistent, the 4096^2 bwd-weight with the wire
    // + bias-gradient epilogue runs faster in the step there, 1.036-1.038 vs 1.042-1.052 ms/step,
    // profiles/r2_pl3_wire_ab.txt; in isolation it measured +13 vs +7 us for the encode)
    const bool pl4 = mode == 3 || (mode == 2 && (!BKC || a.K / sk >= 8192 || EPI == kEpiReluMask));
    if (pl4 && aligned && (!a.colsum || a.workspace)) {
      constexpr int lds = 2 * (BM + BN) * BK * 2;
      auto launch = [&](auto k, bool persist) {  // persist: the kernel loops over tiles (not with colsum)
        FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        hipLaunchKernelGGL(k, persist ? persist_grid(grid) : grid, 256, lds, s, (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb,
                           (TC*)a.C, a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, sk,
                           (float*)a.workspace, a.colsum, wo);
      };
      if constexpr (!SPLIT && !ACCUM && sizeof(TC) == 2 && !is_wire_epi(EPI)) {
        // overlapped tile transitions (pl4_run OVL, default on)
        if (gemm_ovl_flag().load(std::memory_order_relaxed) != 0 && !a.colsum && sk == 1 &&
            a.K >= 2 * BK) {  // (the last k-step fetches the next tile's K-tiles 0 AND 1)
          constexpr int lds_o = 2 * (BM + BN) * BK * 2 + 4 * 16 * (64 + 4) * 4;
          auto k = gemm_pl4_kernel<AK, BKC, EPI, TC, false, false, false, 256, 256, true>;
          FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds_o));
          hipLaunchKernelGGL(k, persist_grid(grid), 256, lds_o, s, (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B,
                             a.ldb, (TC*)a.C, a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K,
                             1, (float*)a.workspace, a.colsum, wo);
          return 0;
        }
      }
      if constexpr (!BKC) {
        if (a.colsum) {
          launch(gemm_pl4_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, true>, false);
          return SPLIT ? sk : a.M / BM;
        }
      }
      launch(gemm_pl4_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, false>, true);
      return 0;
    }
    if ((mode == 2 || mode == 5) && aligned && (!a.colsum || a.workspace)) {
      constexpr int lds = 2 * (BM + BN) * BK * 2;
      auto launch = [&](auto k) {
        FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        hipLaunchKernelGGL(k, grid, 512, lds, s, (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb, (TC*)a.C,
                           a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, sk,
                           (float*)a.workspace, a.colsum, wo);
      };
      if constexpr (!BKC) {
        if (a.colsum) {
          launch(gemm_pl_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, true>);
          return SPLIT ? sk : a.M / BM;
        }
      }
      launch(gemm_pl_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, false>);
      return 0;
    }
  }
  if constexpr (BM == 128 && BN == 128) {
    // 128x128 tiles on the 4-wave pipelined loop (64x64 per wave, 3 LDS stages): outputs too small for 256-wide tiles
    // to fill the CUs without split-K — the bwd-weight GEMMs of the 1024-wide layers (4096 x 1024, K = the batch:
    // 256 tiles, one per CU, no f32 slabs and no reduce pass) — instead of the one-role 8-wave loop
    const int mode = main_loop_mode();
    const bool aligned = a.M % BM == 0 && a.N % BN == 0 && a.K % (BK * sk) == 0;
    if ((mode == 2 || mode == 3) && aligned && (!a.colsum || a.workspace)) {
      constexpr int lds = 3 * (BM + BN) * BK * 2;
      auto launch = [&](auto k, bool persist) {
        FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        hipLaunchKernelGGL(k, persist ? persist_grid(grid) : grid, 256, lds, s, (const bf16_t*)a.A, a.lda,
                           (const bf16_t*)a.B, a.ldb, (TC*)a.C, a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux,
                           a.ldaux, a.M, a.N, a.K, sk, (float*)a.workspace, a.colsum, wo);
      };
      if constexpr (!BKC) {
        if (a.colsum) {
          launch(gemm_pl4_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, true, 128, 128>, false);
          return SPLIT ? sk : a.M / BM;
        }
      }
      launch(gemm_pl4_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, false, 128, 128>, true);
      return 0;
    }
  }
  if constexpr (BM == 256 && BN == 128) {
    // 256x128 tiles (grids that 256x256 tiles leave half empty, e.g. an 8192x1024 output): the 4-wave pipelined
    // loop with 128x64 per wave
    const int mode = main_loop_mode();
    const bool aligned = a.M % BM == 0 && a.N % BN == 0 && a.K % (BK * sk) == 0;
    // (also with the in-kernel BFP wire encode: only reached through a forced 256x128 plan for the bwd-weight)
    if ((mode == 2 || mode == 3) && aligned && (!a.colsum || a.workspace)) {
      constexpr int lds = 3 * (BM + BN) * BK * 2;  // 3 operand stages (gemm_pl4_kernel, BN 128)
      auto launch = [&](auto k, bool persist) {  // persist: the kernel loops over tiles (not with colsum)
        FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        hipLaunchKernelGGL(k, persist ? persist_grid(grid) : grid, 256, lds, s, (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb,
                           (TC*)a.C, a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, sk,
                           (float*)a.workspace, a.colsum, wo);
      };
      if constexpr (!BKC) {
        if (a.colsum) {
          launch(gemm_pl4_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, true, 128>, false);
          return SPLIT ? sk : a.M / BM;
        }
      }
      launch(gemm_pl4_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, false, 128>, true);
      return 0;
    }
  }
  if constexpr (BM == 224) {
    // 224x128 tiles (1792 rows = 8 row tiles: one workgroup per CU on 4096-wide outputs), 4-wave pipelined loop with
    // 112x64 per wave and 3 LDS stages; aligned shapes with a K-contiguous A only (the planner's condition)
    FAN_CHECK(AK && a.M % BM == 0 && a.N % BN == 0 && a.K % (BK * sk) == 0 && !a.colsum,
              "224x128 GEMM tiles: K-contiguous A, M % 224 == 0, N % 128 == 0, no fused bias gradient");
    if constexpr (AK && BN == 128) {
      constexpr int lds = 3 * (BM + BN) * BK * 2;
      auto k = gemm_pl4_kernel<AK, BKC, EPI, TC, ACCUM, SPLIT, false, 128, 224>;
      FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
      hipLaunchKernelGGL(k, persist_grid(grid), 256, lds, s, (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb,
                         (TC*)a.C, a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, sk,
                         (float*)a.workspace, a.colsum, wo);
    }
    return 0;
  } else {
  constexpr int lds = lds_bytes<BM, BN>();
  // bwd-weight layout (both operands MN-contiguous): next stage's DMA by one wave per SIMD; the other layouts issue
  // it from every wave right after the barrier. (Issuing it between the two k-steps' MFMA clusters made fwd1 5 %
  // faster in isolation but the flagship step 3 % slower, same box: profiles/r1_gemm_dma_position_layout_ab.jsonl,
  // r1_gemm_dma_position_flagship_ab.log.)
  const bool ragged = a.M % BM || a.N % BN || a.K % (BK * sk);
  auto k = ragged ? gemm_bf16_kernel<BM, BN, WM, WN, AK, BKC, EPI, TC, ACCUM, SPLIT, !AK && !BKC, true>
                  : gemm_bf16_kernel<BM, BN, WM, WN, AK, BKC, EPI, TC, ACCUM, SPLIT, !AK && !BKC, false>;
  FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL(k, grid, WM * WN * 64, lds, s, (const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb, (TC*)a.C,
                     a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, sk, (float*)a.workspace,
                     a.colsum, wo);
  return SPLIT && a.colsum ? sk : 0;
  }
}

template <bool WIRE, bool UPD = false>
void launch_colsum_reduce(const float* part, int parts, const GemmArgs& a, const WireOut& wo, hipStream_t s) {
  hipLaunchKernelGGL((colsum_reduce_kernel<WIRE, UPD>), cdiv_i(a.N, 64), 256, 0, s, part, parts, a.colsum, a.N, wo);
}

// Bias-gradient reduces queued by fused-update GEMMs (GemmArgs::defer_colsum), per stream, in issue order: the next
// split-K wire reduce of the stream runs them in its first blocks, gemm_flush_colsum launches what is left
// (gemm_bf16_plan.hip holds the queue).
struct PendingColsum {
  const float* part;
  int parts;
  float* colsum;
  int N;
  WireOut wo;
};
void push_pending_colsum(hipStream_t s, const PendingColsum& p);
// up to kMaxGroup of the stream's queued reduces (oldest first) as a group (n == 0: none); removes them from the queue
ColsumGroup take_pending_colsum(hipStream_t s);

// The split counts the planner and tuner use as compile-time constants of the slab reduce (others: runtime count).
template <typename F>
void with_split_count(int sk, F&& f) {
  switch (sk) {
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    default: f(std::integral_constant<int, 0>{}); break;
  }
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI, typename TC, bool ACCUM>
void launch_typed(const GemmArgs& a, int sk, hipStream_t s) {
  WireOut wo{a.wire, a.wire_shard, a.wire_own, a.wire_period, a.wire_codec,
                   a.wire_shard > 0 ? 1.0f / (float)a.wire_shard : 0.f,
                   a.colsum && a.wire ? (int)(a.wire_off + (int64_t)a.M * a.ldc) : 0,
                   a.upd_master, a.upd_lp, a.upd_mom, a.upd
#ifdef FAN_GEMM_STAMPS
                   , (unsigned long long*)gemm_stamp_buffer()
#endif
  };
  wo.off = (uint32_t)a.wire_off;
  wo.prio = gemm_prio_flag().load(std::memory_order_relaxed);

  if (sk > 1) {
    // f32 partial slabs ws[k][M][N] (+ bias-gradient partials ws[sk*M*N + p*N]), then an ordered reduce that
    // applies the epilogue (deterministic: slabs summed in split order)
    // (the split main loop only writes slabs: the wire / update variants share one kernel)
    constexpr int kMainEpi = EPI == kEpiWireUpd ? kEpiWire : EPI;
    const int parts = launch_main<BM, BN, WM, WN, AK, BKC, kMainEpi, TC, ACCUM, true>(a, sk, wo, s);
    if constexpr (is_wire_epi(EPI)) {
      const size_t items = (size_t)a.M * a.N / 16 + (a.colsum ? a.N / 16 : 0);
      const bool lane4 = gemm_reduce4_flag().load(std::memory_order_relaxed) != 0;
      // the stream's queued bias-gradient reduces ride along in the first blocks (one launch less each)
      const ColsumGroup q = lane4 ? take_pending_colsum(s) : ColsumGroup{};
      with_split_count(sk, [&](auto skc) {
        if (lane4 && q.n > 0)
          hipLaunchKernelGGL((splitk_reduce_wire4_kernel<EPI == kEpiWireUpd, decltype(skc)::value, true>),
                             stream_grid((size_t)a.M * a.N / 4) + q.first[q.n], 256, 0, s, (const float*)a.workspace,
                             sk, (float*)a.C, a.ldc, a.M, a.N, a.colsum, wo, q);
        else if (lane4)
          hipLaunchKernelGGL((splitk_reduce_wire4_kernel<EPI == kEpiWireUpd, decltype(skc)::value>),
                             stream_grid((size_t)a.M * a.N / 4), 256, 0, s, (const float*)a.workspace, sk, (float*)a.C,
                             a.ldc, a.M, a.N, a.colsum, wo, q);
        else
          hipLaunchKernelGGL((splitk_reduce_wire_kernel<EPI == kEpiWireUpd, decltype(skc)::value>),
                             stream_grid(items), 256, 0, s, (const float*)a.workspace, sk, (float*)a.C, a.ldc, a.M,
                             a.N, a.colsum, wo);
      });
    } else {
      if (a.defer_reduce) return;  // the caller folds the slabs (GemmArgs::defer_reduce)
      with_split_count(sk, [&](auto skc) {
        hipLaunchKernelGGL((splitk_reduce_kernel<EPI, TC, ACCUM, decltype(skc)::value>),
                           stream_grid((size_t)a.M * a.N / 4), 256, 0, s, (const float*)a.workspace, sk, (TC*)a.C,
                           a.ldc, (const bf16_t*)a.bias, (const TC*)a.aux, a.ldaux, a.M, a.N);
      });
      if (a.colsum)
        launch_colsum_reduce<false>((const float*)a.workspace + (size_t)sk * a.M * a.N, parts, a, wo, s);
    }
  } else {
    // bias-gradient partials at ws[p * N] (pipelined loop): ordered reduce (+ the bias segment's wire encode); a
    // fused-update GEMM may queue it instead (defer_colsum: its partials stay in a workspace of their own)
    const int parts = launch_main<BM, BN, WM, WN, AK, BKC, EPI, TC, ACCUM, false>(a, sk, wo, s);
    if (parts > 0) {
      if constexpr (EPI == kEpiWireUpd) {
        if (a.defer_colsum) {
          push_pending_colsum(s, PendingColsum{(const float*)a.workspace, parts, a.colsum, a.N, wo});
          return;
        }
      }
      launch_colsum_reduce<is_wire_epi(EPI), EPI == kEpiWireUpd>((const float*)a.workspace, parts, a, wo, s);
    }
  }
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC>
void launch_epi(const GemmArgs& a, int sk, hipStream_t s) {
#define FAN_EPI_CASE(E)                                                        \
  case E:                                                                      \
    if (a.c_bf16) launch_typed<BM, BN, WM, WN, AK, BKC, E, bf16_t, false>(a, sk, s); \
    else if (a.accumulate) launch_typed<BM, BN, WM, WN, AK, BKC, E, float, true>(a, sk, s); \
    else launch_typed<BM, BN, WM, WN, AK, BKC, E, float, false>(a, sk, s);  \
    break;
  switch (a.epilogue) {
    FAN_EPI_CASE(kEpiNone)
    FAN_EPI_CASE(kEpiBias)
    FAN_EPI_CASE(kEpiBiasRelu)
    FAN_EPI_CASE(kEpiReluMask)
    case kEpiWire:  // only the bwd-weight layout (A and B MN-contiguous) produces wire-ready gradients
      if constexpr (!AK && !BKC) {
        FAN_CHECK(!a.c_bf16 && !a.accumulate, "wire epilogue: f32, no accumulate");
        if (a.upd_master) launch_typed<BM, BN, WM, WN, AK, BKC, kEpiWireUpd, float, false>(a, sk, s);
        else launch_typed<BM, BN, WM, WN, AK, BKC, kEpiWire, float, false>(a, sk, s);
        break;
      }
      FAN_CHECK(false, "wire epilogue needs A and B MN-contiguous (bwd-weight layout)");
      break;
    default: FAN_CHECK(false, "bad epilogue");
  }
#undef FAN_EPI_CASE
}

template <bool AK, bool BKC>
void launch_tile(const GemmArgs& a, int bm, int bn, int waves, int sk, hipStream_t s) {
#ifdef FAN_GEMM_4WAVE
  // One wave per SIMD (2x2 waves, up to 512 VGPR+AGPR per lane). Measured 5-25% slower than the 8-wave
  // variants on every MLP / BERT / square shape (bench/gemm_bench.py --sweep), so not built by default.
  if (waves == 4) {
    if (bm == 256 && bn == 256) launch_epi<256, 256, 2, 2, AK, BKC>(a, sk, s);
    else if (bm == 256 && bn == 128) launch_epi<256, 128, 2, 2, AK, BKC>(a, sk, s);
    else if (bm == 128 && bn == 256) launch_epi<128, 256, 2, 2, AK, BKC>(a, sk, s);
    else launch_epi<128, 128, 2, 2, AK, BKC>(a, sk, s);
    return;
  }
#endif
  (void)waves;
  if (bm == 256 && bn == 256) launch_epi<256, 256, 2, 4, AK, BKC>(a, sk, s);
  else if (bm == 256 && bn == 128) launch_epi<256, 128, 4, 2, AK, BKC>(a, sk, s);
  else if (bm == 224 && bn == 128) {
    if constexpr (AK) launch_epi<224, 128, 2, 2, AK, BKC>(a, sk, s);
    else FAN_CHECK(false, "224x128 GEMM tiles need a K-contiguous A");
  }
  else if (bm == 128 && bn == 256) launch_epi<128, 256, 2, 4, AK, BKC>(a, sk, s);
  else launch_epi<128, 128, 2, 4, AK, BKC>(a, sk, s);
}

}  // namespace gemm_detail
}  // namespace fan

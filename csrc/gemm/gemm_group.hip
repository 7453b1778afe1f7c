// Grouped GEMM launches.
// * Up to kGroupMax bwd-weight GEMMs of one configuration in one dispatch (gemm_groupn_kernel): a transformer layer's
//   four projections (bench/bert_overlap.py), each too small to fill the CUs without split-K slabs and a reduce
//   pass, fill them once together.
#include "gemm/gemm_bf16_kernel.h"
#include "gemm/gemm_group.h"

namespace fan {

using namespace gemm_detail;

namespace {

template <typename TC>
PlProblem<TC> problem_of(const GemmArgs& a, const WireOut& wo) {
  return PlProblem<TC>{(const bf16_t*)a.A, a.lda, (const bf16_t*)a.B, a.ldb, (TC*)a.C, a.ldc, (const bf16_t*)a.bias,
                       (const TC*)a.aux, a.ldaux, a.M, a.N, a.K, 1, (float*)a.workspace, a.colsum, wo};
}

// WireOut of one problem, as launch_typed builds it (the bias segment right after C in the flat bucket)
WireOut wire_of(const GemmArgs& a) {
  WireOut wo{};
  wo.prio = gemm_prio_flag().load(std::memory_order_relaxed);
  if (a.wire) {
    wo.p = a.wire;
    wo.shard = a.wire_shard;
    wo.own = a.wire_own;
    wo.period = a.wire_period;
    wo.codec = a.wire_codec;
    wo.inv_shard = a.wire_shard > 0 ? 1.0f / (float)a.wire_shard : 0.f;
    wo.bias_off = a.colsum ? (int)(a.wire_off + (int64_t)a.M * a.ldc) : 0;
    wo.off = (uint32_t)a.wire_off;
  }
  return wo;
}

template <int EPI>
void launch_wgrad_group(const GemmArgs* a, int n, hipStream_t s) {
  using P = PlCfg<false, false, EPI, float, false, false, true, 128, 256>;
  PlGroup<float> g{};
  ColsumGroup cg{};
  g.n = cg.n = n;
  int wg = 0, cb = 0;
  for (int i = 0; i < n; ++i) {
    const WireOut wo = wire_of(a[i]);
    g.p[i] = problem_of<float>(a[i], wo);
    g.first[i] = wg;
    const int tiles = (a[i].M / 256) * (a[i].N / 128);
    wg += (tiles + kNumXCD - 1) / kNumXCD * kNumXCD;
    cg.part[i] = (const float*)a[i].workspace;
    cg.parts[i] = a[i].M / 256;
    cg.colsum[i] = a[i].colsum;
    cg.wo[i] = wo;
    cg.N[i] = a[i].N;
    cg.first[i] = cb;
    cb += (a[i].N + 63) / 64;
  }
  g.first[n] = wg;
  cg.first[n] = cb;
  auto k = gemm_groupn_kernel<P>;
  FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, P::kLds));
  hipLaunchKernelGGL(k, wg, 256, P::kLds, s, g);
  FAN_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL((colsum_reduce_group_kernel<is_wire_epi(EPI)>), cb, 256, 0, s, cg);
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace

int64_t gemm_wgrad_group_ws(const GemmArgs& a) { return (int64_t)(a.M / 256) * a.N; }

bool gemm_wgrad_group_supported(const GemmArgs* a, int n) {
  static_assert(kGroupMax == kMaxGroup, "group capacity");
  if (n < 1 || n > kGroupMax) return false;
  int64_t wg = 0;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& g = a[i];
    if (g.a_kcontig || g.b_kcontig || g.c_bf16 || g.accumulate || !g.colsum || !g.workspace) return false;
    if (g.epilogue != a[0].epilogue || (g.epilogue != kEpiNone && g.epilogue != kEpiWire)) return false;
    if (g.M <= 0 || g.N <= 0 || g.M % 256 || g.N % 128 || g.K <= 0 || g.K % 64 || g.ldc < g.N) return false;
    if (g.lda % 8 || g.ldb % 8 || g.ldc % 4 || ((uintptr_t)g.C & 15) || ((uintptr_t)g.colsum & 15)) return false;
    if (g.epilogue == kEpiWire) {
      if (!g.wire || g.wire_shard <= 0 || g.wire_shard % 256 || g.wire_off < 0 || g.wire_off % 16 || g.upd_master)
        return false;
      if (g.wire_off + (int64_t)g.M * g.ldc + g.N >= (1ll << 31)) return false;
    }
    wg += ((int64_t)(g.M / 256) * (g.N / 128) + kNumXCD - 1) / kNumXCD * kNumXCD;
  }
  return wg <= 64 * kNumCU;
}

void launch_gemm_wgrad_group(const GemmArgs* a, int n, hipStream_t s) {
  FAN_CHECK(gemm_wgrad_group_supported(a, n), "gemm_wgrad_group: unsupported shapes / layouts / epilogues");
  if (a[0].epilogue == kEpiWire) launch_wgrad_group<kEpiWire>(a, n, s);
  else launch_wgrad_group<kEpiNone>(a, n, s);
}

}  // namespace fan

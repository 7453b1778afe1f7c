// bf16 GEMM planner + dispatch. The kernel template lives in gemm_bf16_kernel.h; each operand layout is
// instantiated in its own translation unit (gemm_bf16_l*.hip) so the ~200 kernels build in parallel.
#include "gemm/gemm_bf16_launch.h"

#include <algorithm>
#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

namespace fan {

static std::atomic<void*> g_stamp_buffer{nullptr};
void* gemm_stamp_buffer() { return g_stamp_buffer.load(std::memory_order_relaxed); }
void gemm_set_stamp_buffer(void* p) {
#ifdef FAN_GEMM_STAMPS
  g_stamp_buffer.store(p);
#else
  (void)p;
  FAN_CHECK(false, "built without FAN_GEMM_STAMPS");
#endif
}

using gemm_detail::BK;
using gemm_detail::kDefaultWaves;
using gemm_detail::launch_tile;

namespace gemm_detail {  // instantiated in gemm_bf16_l{00,01,10,11}.hip
extern template void launch_tile<false, false>(const GemmArgs&, int, int, int, int, hipStream_t);
extern template void launch_tile<false, true>(const GemmArgs&, int, int, int, int, hipStream_t);
extern template void launch_tile<true, false>(const GemmArgs&, int, int, int, int, hipStream_t);
extern template void launch_tile<true, true>(const GemmArgs&, int, int, int, int, hipStream_t);
}  // namespace gemm_detail

namespace gemm_detail {
namespace {
std::mutex g_pend_mu;
std::map<hipStream_t, std::vector<PendingColsum>>& pend_map() {
  static std::map<hipStream_t, std::vector<PendingColsum>> m;
  return m;
}
}  // namespace

void push_pending_colsum(hipStream_t s, const PendingColsum& p) {
  std::lock_guard<std::mutex> g(g_pend_mu);
  pend_map()[s].push_back(p);
}

ColsumGroup take_pending_colsum(hipStream_t s) {
  ColsumGroup g{};
  std::lock_guard<std::mutex> lk(g_pend_mu);
  auto it = pend_map().find(s);
  if (it == pend_map().end() || it->second.empty()) return g;
  auto& v = it->second;
  const int n = (int)std::min<size_t>(v.size(), kMaxGroup);
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    g.part[i] = v[i].part;
    g.parts[i] = v[i].parts;
    g.colsum[i] = v[i].colsum;
    g.N[i] = v[i].N;
    g.wo[i] = v[i].wo;
    g.first[i] = blocks;
    blocks += cdiv_i(v[i].N, 64);
  }
  g.first[n] = blocks;
  g.n = n;
  v.erase(v.begin(), v.begin() + n);
  return g;
}
}  // namespace gemm_detail

int gemm_flush_colsum(hipStream_t s) {
  int ran = 0;
  for (;;) {
    const gemm_detail::ColsumGroup g = gemm_detail::take_pending_colsum(s);
    if (g.n == 0) return ran;
    hipLaunchKernelGGL((gemm_detail::colsum_reduce_group_kernel<true, true>), g.first[g.n], 256, 0, s, g);
    ran += g.n;
  }
}

int gemm_pending_colsum(hipStream_t s) {
  std::lock_guard<std::mutex> g(gemm_detail::g_pend_mu);
  auto it = gemm_detail::pend_map().find(s);
  return it == gemm_detail::pend_map().end() ? 0 : (int)it->second.size();
}

std::atomic<int>& gemm_prio_flag() {
  static std::atomic<int> flag{[] {
    // default on: the multi-rank step 1.087-1.089 vs 1.093-1.101 ms/step (1-rank group, sharded update), config 5
    // 2.562-2.571 vs 2.587-2.629 ms (profiles/r5_gemm_prio_ab.txt); no other waves share the CU at world 1
    const char* e = getenv("FAN_GEMM_PRIO");
    return e && e[0] == '0' ? 0 : 1;
  }()};
  return flag;
}

std::atomic<int>& gemm_ovl_flag() {
  static std::atomic<int> flag{[] {
    // default on: the flagship step 0.9868 / 0.9903 / 0.9921 vs 0.9946-1.0034 ms/step off, interleaved on one box
    // (profiles/r5_gemm_ovl_ab.txt); bit-identical (tests/test_gpu_gemm_ovl.py)
    const char* e = getenv("FAN_GEMM_OVL");
    return e && e[0] == '0' ? 0 : 1;
  }()};
  return flag;
}

std::atomic<int>& gemm_reduce4_flag() {
  static std::atomic<int> flag{[] {
    const char* e = getenv("FAN_GEMM_REDUCE4");
    return e && e[0] == '0' ? 0 : 1;
  }()};
  return flag;
}

std::atomic<int>& gemm_main_loop_flag() {
  // 256x256 main loop (aligned shapes): 2 software-pipelined, 4 or 8 waves by layout / K (default), 0 one-role
  // loop (FAN_GEMM_PL=0), 3 / 5 pipelined 4-wave / 8-wave only. Selectable for in-process A/B (gemm_set_main_loop).
  static std::atomic<int> flag{[] {
    const char* pl = getenv("FAN_GEMM_PL");
    const int m = pl && pl[0] >= '0' && pl[0] <= '5' ? pl[0] - '0' : 2;
    return m == 1 || m == 4 ? 2 : m;
  }()};
  return flag;
}

std::atomic<int>& gemm_persist_flag() {
  static std::atomic<int> flag{[] {
    const char* e = getenv("FAN_GEMM_PERSIST");
    return e ? atoi(e) : kNumCU;
  }()};
  return flag;
}

// Measured plans for shapes where the heuristic below is not the fastest (bench/gemm_bench.py --sweep on MI355X,
// profiles/r1_gemm_bert_sweep.jsonl): the BERT-base encoder-layer backward GEMMs at 4096 tokens (BASELINE config
// 5). Under-filled grids there favour the big tile (and a split-K that keeps one round of workgroups) over
// "at least one workgroup per CU".
struct TunedPlan {
  int M, N, K, bm, bn, sk;
};
static constexpr TunedPlan kTuned[] = {
    {4096, 3072, 768, 256, 256, 1},   // ffn_out dgrad: 29.4 us vs 34.4 (128x256)
    {3072, 768, 4096, 256, 256, 4},   // ffn_out wgrad: 42.2 us vs 50.5 (128x128)
    {768, 3072, 4096, 256, 256, 4},   // ffn_in wgrad: 42.2 us vs 51.0 (128x128)
    {768, 768, 4096, 128, 128, 4},    // attn_out wgrad: 23.2 us vs 28.2 (split 8)
    {768, 2304, 4096, 128, 256, 4},   // qkv wgrad: 32.6 us vs 38.6 (128x128 split 4)
};

// Plan overrides from the environment, for in-step A/B of tile choices without a rebuild:
// FAN_GEMM_PLAN="MxNxK=bm,bn,sk;MxNxK=bm,bn,sk". Parsed once; a malformed value raises on every plan.
struct EnvPlans {
  std::vector<TunedPlan> plans;
  bool bad = false;
};
static const EnvPlans& env_plans() {
  static const EnvPlans ep = [] {
    EnvPlans r;
    const char* e = getenv("FAN_GEMM_PLAN");
    for (const char* q = e; q && *q;) {
      TunedPlan t{};
      int used = 0;
      if (sscanf(q, "%dx%dx%d=%d,%d,%d%n", &t.M, &t.N, &t.K, &t.bm, &t.bn, &t.sk, &used) != 6 ||
          (t.bm != 128 && t.bm != 256 && t.bm != 224) || (t.bn != 128 && t.bn != 256) ||
          (t.bm == 224 && t.bn != 128) || t.sk < 1) {
        r.bad = true;
        break;
      }
      r.plans.push_back(t);
      q += used;
      if (*q == ';') ++q;
    }
    return r;
  }();
  FAN_CHECK(!ep.bad, "FAN_GEMM_PLAN: expected MxNxK=bm,bn,sk[;...] with bm, bn in {128, 256} (or 224x128)");
  return ep;
}

// Shapes that are not multiples of the tile (any M, N, K that are multiples of 8, e.g. the reference workload's
// 672 or 1344 rows per rank at 8 or 4 ranks): ceil-divided tiles with zero-filled edges. Take the largest tile
// that still gives one workgroup per CU and pads each dimension by at most ~15 %, else 128x128; split K over
// the CUs when even 128x128 tiles leave more than half of them idle (ragged splits are allowed).
static GemmPlan plan_ragged(int M, int N, int K, int split_k, int tile_bm, int tile_bn) {
  GemmPlan p{0, 0, 1, kDefaultWaves};
  const int cand[4][2] = {{256, 256}, {128, 256}, {256, 128}, {128, 128}};
  auto pad_ok = [](int x, int b) { return (int64_t)((x + b - 1) / b) * b * 100 <= (int64_t)x * 115; };
  int best = 3;
  for (int c = 0; c < 4; ++c) {
    const int bm = cand[c][0], bn = cand[c][1];
    if (tile_bm > 0) {
      if (bm == tile_bm && bn == tile_bn) best = c;
      continue;
    }
    const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    if (tiles >= kNumCU && pad_ok(M, bm) && pad_ok(N, bn)) {
      best = c;
      break;
    }
  }
  p.bm = cand[best][0];
  p.bn = cand[best][1];
  const int tiles = ((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
  const int nkt = (K + BK - 1) / BK;
  int sk = 1;
  if (split_k > 0) {
    sk = split_k;
    if (sk > nkt) return GemmPlan{0, 0, 1, kDefaultWaves};
  } else if (tiles * 2 <= kNumCU) {
    while (tiles * sk < kNumCU && sk < 8 && nkt / (sk * 2) >= 8) sk *= 2;
  }
  p.split_k = sk;
  return p;
}

GemmPlan gemm_bf16_plan(int M, int N, int K, int split_k, int tile_bm, int tile_bn, int tile_waves) {
  GemmPlan p{0, 0, 1, 8};
  if (M <= 0 || N <= 0 || K <= 0 || M % 8 || N % 8 || K % 8) return p;
  if (tile_bm == 224) {  // 224x128 tiles, explicit only (the plan tuner's candidate for M % 224 == 0): aligned shapes
    const int sk = split_k > 0 ? split_k : 1;
    if (tile_bn != 128 || M % 224 || N % 128 || K % (BK * sk)) return p;
    return GemmPlan{224, 128, sk, kDefaultWaves};
  }
  if (tile_bm != 0 && ((tile_bm != 128 && tile_bm != 256) || (tile_bn != 128 && tile_bn != 256))) return p;
  if (tile_bm == 0 && split_k <= 0) {
    for (const TunedPlan& t : env_plans().plans)
      if (t.bm == 224 && t.M == M && t.N == N && t.K == K) return gemm_bf16_plan(M, N, K, t.sk, 224, 128, 0);
  }
  if (M % 128 || N % 128 || K % BK ||
      (tile_bm > 0 && (M % tile_bm || N % tile_bn)) || (split_k > 1 && K % (BK * split_k)))
    return plan_ragged(M, N, K, split_k, tile_bm, tile_bn);
  if (tile_bm == 0 && split_k <= 0) {
    for (const TunedPlan& t : env_plans().plans) {
      if (t.M == M && t.N == N && t.K == K && M % t.bm == 0 && N % t.bn == 0 && K % (BK * t.sk) == 0) {
        p.bm = t.bm;
        p.bn = t.bn;
        p.split_k = t.sk;
        p.waves = kDefaultWaves;
        return p;
      }
    }
    for (const TunedPlan& t : kTuned) {
      if (t.M == M && t.N == N && t.K == K && K % (BK * t.sk) == 0) {
        p.bm = t.bm;
        p.bn = t.bn;
        p.split_k = t.sk;
        p.waves = kDefaultWaves;
        return p;
      }
    }
  }
  // Measured on MI355X (bench/gemm_bench.py --sweep, MLP shapes + 4k/8k squares): take the largest tile
  // that still gives >= one workgroup per CU (256), preferring 256x128 (4-wave pipelined loop) over 128x256
  // (one-role loop: the 8192x1024x4096 forward 61.9 vs 72.9 us, hipBLASLt 64.5); split K only when even 128x128
  // tiles leave more than half the CUs idle (split-K costs an f32 slab round trip).
  const int cand[4][2] = {{256, 256}, {256, 128}, {128, 256}, {128, 128}};
  int best = -1;
  for (int c = 0; c < 4 && best < 0; ++c) {
    const int bm = cand[c][0], bn = cand[c][1];
    if (M % bm || N % bn) continue;
    if (tile_bm > 0 && (bm != tile_bm || bn != tile_bn)) continue;
    if (tile_bm > 0 || (M / bm) * (N / bn) >= kNumCU) best = c;
  }
  if (best < 0) {  // small output: the tile with the most workgroups
    for (int c = 3; c >= 0 && best < 0; --c) {
      const int bm = cand[c][0], bn = cand[c][1];
      if (M % bm || N % bn) continue;
      if (tile_bm > 0 && (bm != tile_bm || bn != tile_bn)) continue;
      best = c;
    }
  }
  if (best < 0) return p;
  int sk = 1;
  // Narrow output with a long K (the MLP's 1024x4096 bwd-weight, K = minibatch): 128x128 tiles fill the CUs but
  // stream twice the operand bytes per FLOP; 256x256 tiles with K split over the CUs win despite the f32 slab
  // round trip (measured at K = 8192: 256x256 split 4 = 82 us vs 128x128 = 100 us).
  if (tile_bm == 0 && split_k <= 0 && best == 3 && M % 256 == 0 && N % 256 == 0) {
    const int t256 = (M / 256) * (N / 256);
    int s = 1;
    while (t256 * s < kNumCU && K % (BK * s * 2) == 0 && K / (s * 2) >= 1024) s *= 2;
    if (t256 * s >= kNumCU) {
      best = 0;
      sk = s;
    }
  }
  const int tiles = (M / cand[best][0]) * (N / cand[best][1]);
  if (sk > 1) {
  } else if (split_k > 0) {
    sk = split_k;
    if (K % (BK * sk)) return p;
  } else if (tiles * 2 <= kNumCU) {
    while (tiles * sk < kNumCU && sk < 8 && K % (BK * sk * 2) == 0 && K / (sk * 2) >= 512) sk *= 2;
  }
  p.bm = cand[best][0];
  p.bn = cand[best][1];
  p.split_k = sk;
#ifdef FAN_GEMM_4WAVE
  p.waves = tile_waves == 4 || tile_waves == 8 ? tile_waves : kDefaultWaves;
#else
  p.waves = kDefaultWaves;
  (void)tile_waves;
#endif
  return p;
}

bool gemm_bf16_supported(const GemmArgs& a) {
  const GemmPlan p = gemm_bf16_plan(a.M, a.N, a.K, a.split_k, a.tile_bm, a.tile_bn, a.tile_waves);
  if (p.bm == 0) return false;
  if (a.lda % 8 || a.ldb % 8 || a.ldc % 4 || (a.aux && a.ldaux % 4)) return false;
  if (((uintptr_t)a.A | (uintptr_t)a.B) & 15) return false;
  if (((uintptr_t)a.C) & (a.c_bf16 ? 7 : 15)) return false;
  if (a.accumulate && a.c_bf16) return false;
  if (p.split_k > 1 && a.workspace == nullptr) return false;
  if (a.colsum && a.b_kcontig) return false;
  if (p.bm == 224 && (!a.a_kcontig || a.colsum)) return false;  // 224-row tiles: K-contiguous A image only
  if (a.epilogue == kEpiWire) {
    if (a.a_kcontig || a.b_kcontig || a.c_bf16 || a.accumulate || !a.wire || a.N % 16) return false;
    if (a.wire_shard <= 0 || a.wire_shard % 256 || a.ldc % 16) return false;
    if (a.wire_codec != kBfpTrunc && a.wire_codec != kBfpRne) return false;
    if (a.wire_off < 0 || a.wire_off % 16 || a.wire_off + (int64_t)a.M * a.ldc + a.N >= (int64_t(1) << 31))
      return false;
  }
  return true;
}

void launch_gemm_bf16(const GemmArgs& a, hipStream_t s) {
  FAN_CHECK(gemm_bf16_supported(a), "gemm_bf16: unsupported shape/layout (need M, N, K % 8 == 0)");
  const GemmPlan p = gemm_bf16_plan(a.M, a.N, a.K, a.split_k, a.tile_bm, a.tile_bn, a.tile_waves);
  if (a.c_bf16 && !a.wire) {  // the bf16 epilogue stores 8 columns (16 B) per lane (store_tile, epi8_bf16)
    const bool mask = a.epilogue == kEpiReluMask;
    const bool bias = a.epilogue == kEpiBias || a.epilogue == kEpiBiasRelu;
    FAN_CHECK(((uintptr_t)a.C & 15) == 0 && a.ldc % 8 == 0 && (!bias || ((uintptr_t)a.bias & 15) == 0) &&
                  (!mask || (((uintptr_t)a.aux & 15) == 0 && a.ldaux % 8 == 0)),
              "gemm_bf16: bf16 output, bias and activation must be 16-B aligned with ldc, ldaux % 8 == 0");
  }
  if (a.a_kcontig && a.b_kcontig) launch_tile<true, true>(a, p.bm, p.bn, p.waves, p.split_k, s);
  else if (a.a_kcontig && !a.b_kcontig) launch_tile<true, false>(a, p.bm, p.bn, p.waves, p.split_k, s);
  else if (!a.a_kcontig && a.b_kcontig) launch_tile<false, true>(a, p.bm, p.bn, p.waves, p.split_k, s);
  else launch_tile<false, false>(a, p.bm, p.bn, p.waves, p.split_k, s);
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace fan

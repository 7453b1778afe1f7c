// Layer-chain GEMM launches (gemm_chain.h): the forward's and the backward-data's GEMMs of the MLP as ONE persistent
// launch each. Reference: the whole FWD + BWD loop runs inside one `#pragma omp parallel` region whose layers hand
// over through barriers, with no per-layer team start-up (sw/mlp_mpi_example_f32.cpp:690-788); here a layer's row
// panel hands over to the next layer's tiles of that panel through a ready counter instead of a kernel boundary, so
// the per-launch fill / drain (profiles/r5_gemm_k_scaling.jsonl: ~20 us per GEMM) is paid once per pass.
#include "gemm/gemm_bf16_kernel.h"
#include "gemm/gemm_chain.h"

#include <cstdlib>

namespace fan {

using namespace gemm_detail;

namespace gemm_detail {

// one stage's tile configuration: the persistent 4-wave loop in chain mode
template <bool AK, bool BKC, int EPI, typename TC, int BN_, bool OVL, bool WT, bool ASC1 = false>
struct ChainCfg {
  __device__ static __forceinline__ void run(const ChainArgs& ca, ChainState* cs, int s) {
    const ChainStageArgs& S = ca.st[s];
    WireOut wo{};
    wo.prio = ca.prio;
    ChainRun cr;
    cr.ctr = ca.ctr;
    cr.group = (int)(blockIdx.x & 7);
    cr.ppg = ca.ppg;
    cr.wpg = (int)(gridDim.x >> 3);
    cr.first = S.first;
    cr.end = s + 1 < ca.nstages ? ca.st[s + 1].first : ca.total;
    cr.tn = S.tn;
    cr.dep = S.dep;
    cr.dep_word0 = s > 0 ? chain_ready_word(ca, s - 1, cr.group * ca.ppg) : 0;
    cr.sig_word0 = S.signal ? chain_ready_word(ca, s, cr.group * ca.ppg) : -1;
    cr.nx_end = s + 2 < ca.nstages ? ca.st[s + 2].first : ca.total;
    cr.nx_tn = s + 1 < ca.nstages ? ca.st[s + 1].tn : 1;
    cr.flags = ca.flags;
    pl4_run<AK, BKC, EPI, TC, false, false, false, BN_, 256, OVL, true, WT, ASC1>(
        S.A, S.lda, S.B, S.ldb, reinterpret_cast<TC*>(S.C), S.ldc, S.bias, reinterpret_cast<const TC*>(S.aux),
        S.ldaux, S.M, S.N, S.K, 1, nullptr, nullptr, wo, 0, 0, cr, cs);
  }
};

// Wait (wave 0 lane 0 spins) for the ticket's row panel, after publishing this workgroup's finished tile (every
// wave drains its stores first); then every wave's own acquire.
__device__ __forceinline__ void chain_wait(const ChainArgs& ca, ChainState& cs, int wave, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wave == 0 && lane == 0) {
    if (cs.pending >= 0) chain_add(ca.ctr, cs.pending);
    int w;
    unsigned tgt;
    chain_dep_of(ca, cs.ticket, w, tgt);
    if (w >= 0) {
      for (uint32_t n = 0; chain_poll(ca.ctr, w) < tgt;) {
        __builtin_amdgcn_s_sleep(2);
        if (++n > kChainSpinLimit) {  // give up: garbage results, an error code for the host, no hang
          __hip_atomic_store(ca.ctr + 9 * 16, 1u + (unsigned)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  cs.pending = -1;
  __syncthreads();
  chain_acquire(ca.flags);
}

// Publish the last tile; the last workgroup out zeroes the counter block for the next launch (every other
// workgroup's final add has returned before its exit add).
__device__ __forceinline__ void chain_exit(const ChainArgs& ca, const ChainState& cs, int wave, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wave != 0) return;
  unsigned last = 0;
  if (lane == 0) {
    if (cs.pending >= 0) {
      const unsigned o = __hip_atomic_fetch_add(ca.ctr + cs.pending, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("" ::"v"(o));  // returned: performed before the exit add below
    }
    last = __hip_atomic_fetch_add(ca.ctr + 8 * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  if (__builtin_amdgcn_readfirstlane(last)) {
    const int words = 10 + ca.nstages * ca.panels;
    for (int i = lane; i < words; i += 64)
      if (i != 9) __hip_atomic_store(ca.ctr + i * 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <class C0, class C1>
__global__ void __launch_bounds__(256, 1) gemm_chain_kernel(ChainArgs ca) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  ChainState cs{(int)(blockIdx.x >> 3), 0, -1};
  {
    int w;
    unsigned tgt;
    chain_dep_of(ca, cs.ticket, w, tgt);
    cs.ready = w < 0;
  }
  while (cs.ticket < ca.total) {
    const int s = chain_stage_of(ca, cs.ticket);
    if (!cs.ready) chain_wait(ca, cs, wave, lane);
    else if (ca.st[s].dep > 0) chain_acquire(ca.flags);  // met at the poll: this wave's acquire before its own loads
    if (ca.st[s].cfg == 0) C0::run(ca, &cs, s);
    else C1::run(ca, &cs, s);
  }
  chain_exit(ca, cs, wave, lane);
}

}  // namespace gemm_detail

namespace {

constexpr int kPanel = 256;

using FwdHidden = ChainCfg<true, false, kEpiBiasRelu, bf16_t, 256, true, true>;
using FwdLogits = ChainCfg<true, false, kEpiBias, float, 128, false, false>;
using BwdData = ChainCfg<true, true, kEpiReluMask, bf16_t, 256, true, true>;
// diagnostic (FAN_CHAIN_WT=0, unsafe): plain producer stores
using FwdHiddenP = ChainCfg<true, false, kEpiBiasRelu, bf16_t, 256, true, false>;
using BwdDataP = ChainCfg<true, true, kEpiReluMask, bf16_t, 256, true, false>;
// diagnostic (FAN_CHAIN_ASC1=1): the A operand's LDS-DMA bypasses L1 (sc1) and no acquire
using FwdHiddenS = ChainCfg<true, false, kEpiBiasRelu, bf16_t, 256, true, true, true>;
using FwdLogitsS = ChainCfg<true, false, kEpiBias, float, 128, false, false, true>;
using BwdDataS = ChainCfg<true, true, kEpiReluMask, bf16_t, 256, true, true, true>;

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// the stage's tile configuration index for the kernel of `kind` (-1: not a configuration of that chain)
int stage_cfg(const GemmArgs& g, int kind, bool last) {
  const bool aligned = g.M % (kPanel * kNumXCD) == 0 && g.K % BK == 0 && g.K / BK >= 6 && !g.accumulate &&
                       g.split_k <= 1 && !g.colsum && !g.wire && g.a_kcontig;
  if (!aligned) return -1;
  if (kind == kChainFwd) {
    if (!g.b_kcontig && g.epilogue == kEpiBiasRelu && g.c_bf16 && g.N % 256 == 0 && g.bias) return 0;
    if (last && !g.b_kcontig && g.epilogue == kEpiBias && !g.c_bf16 && g.N % 128 == 0 && g.bias) return 1;  // logits
    return -1;
  }
  if (kind == kChainBwdData) {
    if (g.b_kcontig && g.epilogue == kEpiReluMask && g.c_bf16 && g.N % 256 == 0 && g.aux) return 0;
    return -1;
  }
  return -1;
}

}  // namespace

int gemm_chain_counter_words(int n, int M) { return chain_ctr_words(n, M / kPanel); }
int gemm_chain_max_stages() { return kChainMaxStages; }

bool gemm_chain_supported(const GemmArgs* a, int n, int kind) {
  if (n < 1 || n > kChainMaxStages) return false;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& g = a[i];
    if (stage_cfg(g, kind, i == n - 1) < 0 || g.M != a[0].M) return false;
    if (g.lda % 8 || g.ldb % 8 || g.ldc % 8 || (g.aux && g.ldaux % 8)) return false;
    if (((uintptr_t)g.A | (uintptr_t)g.B | (uintptr_t)g.C) & 15) return false;
    if ((g.bias && ((uintptr_t)g.bias & 15)) || (g.aux && ((uintptr_t)g.aux & 15))) return false;
    if (i > 0 && (g.A != a[i - 1].C || g.lda != a[i - 1].ldc || g.K != a[i - 1].N || !a[i - 1].c_bf16)) return false;
  }
  return true;
}

void launch_gemm_chain(const GemmArgs* a, int n, int kind, unsigned* counters, hipStream_t s) {
  FAN_CHECK(gemm_chain_supported(a, n, kind), "gemm_chain: unsupported stages / shapes / layouts");
  FAN_CHECK(counters != nullptr, "gemm_chain: counter block");
  ChainArgs ca{};
  const int M = a[0].M;
  ca.nstages = n;
  ca.panels = M / kPanel;
  ca.ppg = ca.panels / kNumXCD;
  ca.ctr = counters;
  ca.prio = gemm_prio_flag().load(std::memory_order_relaxed);
  // diagnostic schedule variants (A/B probes only): FAN_CHAIN_ACQ=0 skips the acquire, FAN_CHAIN_ORDER=1 rows-fastest
  static const int diag_flags = (env_int("FAN_CHAIN_ACQ", 1) == 0 ? kChainNoAcquire : 0) |
                                (env_int("FAN_CHAIN_ORDER", 0) == 1 ? kChainRowsFastest : 0);
  static const bool plain = env_int("FAN_CHAIN_WT", 1) == 0;
  static const bool asc1 = env_int("FAN_CHAIN_ASC1", 0) == 1;
  ca.flags = diag_flags | (asc1 ? kChainNoAcquire : 0);
  int first = 0;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& g = a[i];
    ChainStageArgs& S = ca.st[i];
    S.A = reinterpret_cast<const bf16_t*>(g.A);
    S.B = reinterpret_cast<const bf16_t*>(g.B);
    S.C = g.C;
    S.bias = reinterpret_cast<const bf16_t*>(g.bias);
    S.aux = g.aux;
    S.lda = g.lda;
    S.ldb = g.ldb;
    S.ldc = g.ldc;
    S.ldaux = g.ldaux;
    S.M = g.M;
    S.N = g.N;
    S.K = g.K;
    S.cfg = stage_cfg(g, kind, i == n - 1);
    S.tn = g.N / (S.cfg == 1 ? 128 : 256);
    S.first = first;
    S.dep = i > 0 ? ca.st[i - 1].tn : 0;
    S.signal = i + 1 < n;
    first += ca.ppg * S.tn;
  }
  ca.total = first;
  auto k = kind == kChainFwd
               ? (asc1 ? gemm_chain_kernel<FwdHiddenS, FwdLogitsS>
                       : plain ? gemm_chain_kernel<FwdHiddenP, FwdLogits> : gemm_chain_kernel<FwdHidden, FwdLogits>)
               : (asc1 ? gemm_chain_kernel<BwdDataS, BwdDataS>
                       : plain ? gemm_chain_kernel<BwdDataP, BwdDataP> : gemm_chain_kernel<BwdData, BwdData>);
  FAN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, kChainLds));
  hipLaunchKernelGGL(k, kNumCU, 256, kChainLds, s, ca);
  FAN_HIP_CHECK(hipGetLastError());
}

}  // namespace fan

// MFMA GEMM entry points (gfx950).
//
// C[M][N] (row-major, ldc) = sum_k A(m,k) * B(k,n), with fused epilogues. Operand layouts:
//   A K-contiguous : A stored [M][K] (lda)      A MN-contiguous : A stored [K][M] (lda)
//   B K-contiguous : B stored [N][K] (ldb)      B MN-contiguous : B stored [K][N] (ldb)
// so forward (X·W, W=[in][out]), backward-data (dZ·Wᵀ) and backward-weight (Xᵀ·dZ) of the
// MLP all run without a transpose pass (reference: libxsmm fc fwd/bwd, sw/mlp_mpi_example_f32.cpp:708, 741, 770).
#pragma once
#include <atomic>

#include "bfp/bfp_format.h"  // SgdParams (fused local update)
#include "common/hip_common.h"

namespace fan {

enum GemmEpilogue : int {
  kEpiNone = 0,
  kEpiBias = 1,       // + bias[n]
  kEpiBiasRelu = 2,   // relu(x + bias[n])
  kEpiReluMask = 3,   // x * (aux[m][n] > 0)   (ReLU backward fused into the bwd-data GEMM)
  kEpiWire = 4,       // BFP-encode the f32 result straight into all-reduce wire shards (see GemmArgs::wire)
  kEpiWireUpd = 5,    // kernel-internal: kEpiWire with the fused local update (GemmArgs::upd_master set)
};
constexpr bool is_wire_epi(int e) { return e == kEpiWire || e == kEpiWireUpd; }

// GemmArgs::wire_own value: every shard is also written to C in f32 (the ring needs every local slice in f32:
// each reduce hop adds the local f32 contribution, hw/all_reduce.sv:1168-1183)
constexpr int kWireOwnAll = -2;

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  const void* bias;  // dtype = operand dtype
  const void* aux;   // bf16/f32 (same as C dtype), [M][N] with ldaux
  int64_t lda, ldb, ldc, ldaux;
  int M, N, K;
  bool a_kcontig, b_kcontig;
  int epilogue;
  bool c_bf16;       // output dtype (bf16 or f32)
  bool accumulate;   // C += result (f32 output only)
  int split_k;       // 0: auto; >=1: K split over workgroups (fp32 partial slabs + ordered reduce)
  void* workspace;   // split-K slabs: split_k * M * N floats (+ split_k * N with colsum: bias-gradient partials)
  int tile_bm = 0;   // 0: automatic tile choice; else force BM x BN (128/256)
  int tile_bn = 0;
  int tile_waves = 0;  // 0: default; 4 or 8 waves per workgroup
  float* colsum = nullptr;  // optional: colsum[n] = sum_k B(k, n) (bias gradient fused into bwd-weight;
                            // B MN-contiguous, no split-K); written, not accumulated
  // kEpiWire: element (m, n) of C sits at flat index f = m*ldc + n of a bucket split into shards of
  // wire_shard elements; it is encoded (groups of 16 along n) into the wire layout of shard f / wire_shard
  // (bfp_format.h). Elements of shard wire_own (>= 0) are also written to C in f32 (the owner's
  // un-quantised local contribution for the mesh reduce). f32 output, no split-K, no accumulate.
  // With colsum, the column sums are also encoded as the bucket segment that follows C (flat M*ldc + n: the
  // bias gradient of the [W | b] bucket). The bucket must have fewer than 2^31 elements.
  uint8_t* wire = nullptr;
  int64_t wire_shard = 0;
  int wire_own = -1;
  int wire_period = 0;  // > 0: every shard s with s % wire_period == wire_own is owned (chunked mesh buckets)
  int wire_codec = 1;  // kBfpTrunc or kBfpRne
  int64_t wire_off = 0;  // flat bucket index of C(0, 0): f = wire_off + m*ldc + n (a tensor inside a larger bucket)
  // kEpiWire fused local update (single-rank engine): instead of storing the wire, every encoded group is decoded
  // in registers and applied by SGD to the bucket planes at the same flat indices (upd_master f32, upd_lp bf16
  // copy, upd_mom optional; wire_own must be -1). See WireOut::um (gemm_bf16_kernel.h).
  float* upd_master = nullptr;
  bf16_t* upd_lp = nullptr;
  float* upd_mom = nullptr;
  SgdParams upd{};
  // fused update with colsum on an unsplit plan: the bias-gradient reduce is queued on the stream instead of launched
  // (the next split-K wire reduce of the stream runs it in its first blocks, gemm_flush_colsum what is left); the
  // partials in `workspace` must stay untouched until then (the caller gives such a GEMM a workspace of its own)
  bool defer_colsum = false;
  // split-K plans of the f32 bias epilogue: the slab reduce is NOT launched — the caller consumes the slabs itself
  // (the classifier's softmax folds them: launch_softmax_xent_slabs)
  bool defer_reduce = false;
};

struct GemmPlan {
  int bm, bn, split_k, waves;  // bm == 0: unsupported; waves: 8 (2/SIMD) or 4 (1/SIMD)
};

// Tile / split-K choice for a shape (split_k <= 0: automatic).
GemmPlan gemm_bf16_plan(int M, int N, int K, int split_k, int tile_bm = 0, int tile_bn = 0, int tile_waves = 0);

// Returns false if the shape is not supported by the MFMA path (caller must then error out).
bool gemm_bf16_supported(const GemmArgs& a);
void launch_gemm_bf16(const GemmArgs& a, hipStream_t stream);
// launches the bias-gradient reduces queued on the stream (GemmArgs::defer_colsum) as grouped launches; returns how
// many ran. gemm_pending_colsum: how many are queued.
int gemm_flush_colsum(hipStream_t stream);
int gemm_pending_colsum(hipStream_t stream);

// 256x256 tiles: main-loop selection (0 one-role, 2 pipelined by layout / K, 3 pipelined 4-wave, 5 8-wave).
std::atomic<int>& gemm_main_loop_flag();
// grid cap of the persistent 4-wave pipelined kernel (FAN_GEMM_PERSIST, default 256 = one workgroup per CU; 0: one
// workgroup per tile); settable for in-process A/B and for tests that force several tiles per workgroup
std::atomic<int>& gemm_persist_flag();
// the 4-wave pipelined GEMM waves at s_setprio 2, so another stream's kernels sharing their CUs (the all-reduce's)
// issue in the GEMM waves' stalls only (default on; FAN_GEMM_PRIO=0, gemm_set_prio)
std::atomic<int>& gemm_prio_flag();
// 256x256 bf16 plans on the persistent loop whose tile transitions overlap the epilogue with the next tile's first
// K-tiles (pl4_run OVL; default on, FAN_GEMM_OVL=0, gemm_set_ovl)
std::atomic<int>& gemm_ovl_flag();
// split-K wire / fused-update reduce: lane-contiguous form, 4 values per lane (1, default) or one 16-value group per
// lane (0) (FAN_GEMM_REDUCE4, gemm_set_reduce4); bit-identical either way
std::atomic<int>& gemm_reduce4_flag();
// diagnostic builds (-DFAN_GEMM_STAMPS): device buffer for the one-role loop's s_memtime stamps (nullptr: off)
void gemm_set_stamp_buffer(void* p);
void* gemm_stamp_buffer();

// f32 GEMM split-K factor for a shape (split_k <= 0: automatic); workspace: split * M * N floats when > 1.
int gemm_f32_split(int M, int N, int K, int split_k);
bool gemm_f32_supported(const GemmArgs& a);
void launch_gemm_f32(const GemmArgs& a, hipStream_t stream);

}  // namespace fan

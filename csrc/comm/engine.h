// Native compressed all-reduce engine (C++): the MI355X counterpart of the reference NIC's request path.
//
// Reference behaviour being re-expressed:
//   * all_reduce_setup(done, count, node_id)   -> AllReduceEngine(comm, rank, world, cfg)
//   * all_reduce(buf, weight_out, flags, ...)  -> submit(): enqueue pack -> xGMI exchange -> reduce ->
//                                                 exchange -> fused SGD epilogue on a high-priority comm stream
//   * 8 done slots, round-robin 3-bit done_id  -> kSlots request slots; completion is a 32-bit sequence number
//     (hw/all_reduce.sv:1228, 1368-1375)          written by the GPU (hipStreamWriteValue32) into host-mapped memory
//   * wait(done_buf) busy spin (sw:157-180)     -> synchronize(slot, timeout): polls the done word with a bounded
//                                                 timeout + RCCL async-error check (never spins forever)
//   * get_all_reduce_latency (sw:100-106)       -> latency_ms(slot) from device timestamps
// Algorithms: mesh (pack / all-to-all / owner reduce / re-encode / all-gather) and the reference ring schedule
// (native planner, any N, R arc-disjoint rings) with one fused decode+add+encode kernel per hop.
#pragma once
#include <array>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "bfp/bfp_format.h"
#include "comm/native_comm.h"
#include "comm/planner.h"
#include "comm/slot_table.h"
#include "comm/verify.h"

namespace fan {

struct EngineConfig {
  int codec = kBfpRne;
  int algo = 0;  // 0 mesh, 1 ring
  int rings = 1;
  int64_t max_slice_elems = 1 << 22;
  bool compat_owner_fp32 = false;
  double timeout_s = 600.0;
  int stream_priority = -1;
  bool force_comm = false;  // world 1 still runs the collectives (exercises the multi-rank path)
  int verify = -1;          // debug verify mode (message tags + sequence numbers); -1: from FAN_VERIFY
  // mesh: buckets above this many elements stream through the collectives in chunks (block pipeline, bounded
  // scratch); 0: from FAN_CHUNK_ELEMS, default 64 Mi elements (256 MB of f32 gradient: at world 1 the chunked
  // pipeline measured 29 % slower on a 256 MB request, profiles/r2_allreduce_bw_1gpu_chunked8M.jsonl)
  int64_t chunk_elems = 0;
  // ring: direct links (row-major world x world, links[a*world+b]: a can send to b); empty = fully connected
  std::vector<char> links;
  // world 1 (inline, no communication phase): run each committed epilogue (decode + SGD) on an engine stream
  // beside the producer's next kernels instead of in the producer's stream order; -1: from FAN_SIDE_EPI
  int side_epilogue = -1;
  // direct-P2P ring: each hop's message streams in this many sub-slices, each with its own ready flag, so the
  // downstream rank reduces sub-slice s of round t as soon as it lands (the NIC's beat-level send_fifo pipeline,
  // hw/all_reduce.sv:1155-1166) instead of after the whole slice; capped by the P2P arena depth - 1. 0: from
  // FAN_RING_SUB (default 1: lock-step hops).
  int ring_sub = 0;
  // mesh, multi-rank: sharded weight update (ZeRO-1 style). The owner of shard q fuses its reduce with the BFP round
  // trip + SGD of that shard (master / momentum of shard q are kept current on its owner only) and the ranks
  // all-gather the updated bf16 WEIGHTS instead of the reduced gradient; the request writes its submit's `lp`
  // (the trainer passes the layer's next weight buffer), so no epilogue waits for the bwd-data GEMM. Bit-identical
  // weights to the unsharded schedule. Update requests of bf16 models without out_sum only. -1: FAN_SHARD_UPDATE.
  int shard_update = -1;
};

struct EngineLayout {
  int64_t n = 0, n_pad = 0;
  int algo = 0;
  int64_t shard = 0;        // mesh (per chunk)
  int64_t chunks = 1;       // mesh: chunks of N shards each (shard-major: shard s of chunk c is wire shard c*N+s)
  int64_t slice = 0;        // ring
  int64_t blocks = 0;       // ring
  int rings = 1;
  int64_t part = 0;         // ring: padded elements per ring part
  int sub = 1;              // ring: sub-slices (wire sub-shards of slice / sub elements) per hop message
};

// Per-engine performance counters: the reference NIC's perf/debug registers re-expressed (hw/all_reduce.sv:92-98,
// 892-1085: lpbk_latency active cycles, stall_host_in/out; sw/mlp_mpi_example_f32.cpp:100-112: the getters).
struct EngineCounters {
  uint64_t requests = 0;
  int64_t logical_bytes = 0;   // fp32 gradient bytes requested (n_valid * 4)
  int64_t wire_bytes = 0;      // bytes this rank sends over the fabric
  double host_wait_s = 0.0;    // host time blocked in synchronize() (stall_host analogue)
  uint64_t host_waits = 0;     // synchronize() calls that had to wait
  uint64_t host_spins = 0;     // done-word polls while waiting
  double device_ms = 0.0;      // summed device time of timed requests (lpbk_latency analogue)
  uint64_t timed_requests = 0;
  uint64_t forced_commits = 0;  // deferred epilogues committed because their slot was needed (> kSlots deferred)
  uint64_t verified_rows = 0;   // verify mode: message rows whose tags were checked on arrival
  uint64_t direct_rounds = 0;   // direct P2P rounds (kernels stored into / read from peer receive slots in place)
  uint64_t sharded_updates = 0; // requests that ran the sharded update (owner reduce + SGD, weight all-gather)
  std::vector<int64_t> peer_bytes;  // message bytes sent to each peer (all-to-all, all-gather, ring hops, direct)
};

// Device-side request trace: GPU timestamps (timing events) at the phase boundaries of each request, the MI355X
// counterpart of the NIC's per-state cycle counters (lpbk_latency and the stall_* attributions,
// hw/all_reduce.sv:892-1085) and of get_all_reduce_latency (sw/mlp_mpi_example_f32.cpp:100-106). Points are
// recorded on the stream the phase runs on; the ring schedule has no separate pack / exchange / reduce phases
// (every hop fuses them), so its middle points coincide with the end of communication.
enum TracePoint : int {
  kTpStart = 0,   // request starts on the comm stream (producer done, previous request drained)
  kTpPacked,      // pack / encode pass done (mesh)
  kTpExchanged,   // all-to-all of the packed shards done (mesh)
  kTpReduced,     // owner-shard reduce done (mesh)
  kTpCommEnd,     // all-gather done: end of the communication phase
  kTpEpiEnd,      // decode + SGD epilogue done
  kTpCount
};

struct TraceSummary {
  uint64_t requests = 0, dropped = 0;
  int64_t logical_bytes = 0, wire_bytes = 0;
  double ms[kTpCount] = {0, 0, 0, 0, 0, 0};  // ms[p] = summed time between point p-1 and p (ms[0] unused)
  double comm_ms = 0.0;                       // summed kTpStart -> kTpCommEnd
  double total_ms = 0.0;                      // summed kTpStart -> kTpEpiEnd
  // ring hops (per round: start -> credits granted -> kernels done -> upstream data ready), summed over the traced
  // requests' rounds; hop_max_ms: the longest single round
  uint64_t hop_rounds = 0;
  double hop_credit_ms = 0.0, hop_kernel_ms = 0.0, hop_ready_ms = 0.0, hop_max_ms = 0.0;
};

// verify-error sites (VerifyError::site): copying paths 1-3, direct P2P paths 4-6
enum VerifySite : uint32_t {
  kSiteMeshAllToAll = 1,
  kSiteMeshAllGather = 2,
  kSiteRingRound = 3,
  kSiteMeshDirectSend = 4,
  kSiteMeshDirectGather = 5,
  kSiteRingDirect = 6,
  kSiteMeshWeightGather = 7,  // the sharded update's bf16 weight all-gather (run_mesh)
};

// Deferred epilogue of a request (decode + SGD), launched on the given stream at commit().
using EpiThunk = std::function<void(hipStream_t)>;

// The HIP device policy of the request-slot state machine (slot_table.h): events, stream waits, and the done
// words the GPU writes into host-mapped memory (one 64-B line per slot).
struct HipSlotDevice {
  using Stream = hipStream_t;
  using Event = hipEvent_t;
  volatile uint32_t* host_words = nullptr;
  uint32_t* dev_words = nullptr;
  void record(Event e, Stream s) { FAN_HIP_CHECK(hipEventRecord(e, s)); }
  void wait(Stream s, Event e) { FAN_HIP_CHECK(hipStreamWaitEvent(s, e, 0)); }
  bool query(Event e) {
    const hipError_t r = hipEventQuery(e);
    if (r != hipSuccess) (void)hipGetLastError();  // not-ready is not an error
    return r == hipSuccess;
  }
  void write_done(Stream s, int slot, uint32_t seq) {
    FAN_HIP_CHECK(hipStreamWriteValue32(s, dev_words + slot * 16, seq, 0));
  }
  uint32_t read_done(int slot) { return host_words[slot * 16]; }
};

class AllReduceEngine {
 public:
  static constexpr int kSlots = SlotTable<HipSlotDevice>::kSlots;

  AllReduceEngine(Comm* comm, int rank, int world, EngineConfig cfg, int device);
  ~AllReduceEngine();

  // Layout of a bucket of n elements. shard / chunks > 0 (mesh): an explicit chunked layout of `chunks` chunks of
  // world shards of `shard` elements each (a multiple of 256): the trainer's row-panel split of a bucket submits
  // each chunk as a request of its own (chunks = 1) with the same shard size as the whole-bucket layout, so both
  // schedules reduce every element on the same owner, bit for bit.
  EngineLayout layout(int64_t n, int64_t shard = 0, int64_t chunks = 0) const;
  const std::vector<std::vector<int>>& orders() const { return orders_; }
  hipStream_t stream() const { return stream_; }
  Comm* comm() const { return comm_; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  bool is_inline() const { return table_->config().inline_mode; }
  int codec() const { return cfg_.codec; }
  int ring_sub() const;  // sub-slices per ring hop this engine runs (1 unless direct P2P ring streaming)
  bool shard_update() const { return shard_upd_; }  // sharded weight update (EngineConfig::shard_update) in force
  // All-gather an f32 bucket plane whose shard q is current on rank q only (a sharded-update engine's master /
  // momentum) in place, in pieces that fit the transport; checkpoints and replica checks call it. Host-blocking.
  void gather_owned(float* plane, int64_t n);

  // Enqueue the communication phase of a request. grad: padded flat buffer (f32 or bf16) ready on `producer`.
  // on_producer (multi-rank): the phase runs on the producer stream itself (SlotTable::begin), not the comm stream.
  // If `defer`, the weight update is enqueued later by commit(); otherwise immediately. Returns the slot.
  // prepacked (BFP codecs): the producer already encoded flat elements [0, prepacked_elems) of the bucket into
  // `prepacked` (shard layout of prepack_shape(): mesh shards, or ring slices ring-major); the engine packs the
  // rest (bias + padding) and skips its own encode of them (mesh: the pack pass, and at world 1 the reduce pass;
  // ring: every SEND_LOCAL). The shards prepack_shape() names as owned must also be present in f32 in `grad`
  // (mesh: the owner shard; ring: all of them).
  int submit(const void* grad, int grad_dtype, float* master, bf16_t* lp, float* mom, int64_t n_valid,
             SgdParams sgd, hipStream_t producer, bool defer, bool update = true, float* out_sum = nullptr,
             const uint8_t* prepacked = nullptr, int64_t prepacked_elems = 0, int64_t layout_shard = 0,
             int64_t layout_chunks = 0, bool on_producer = false);
  // (shard elements, shards, owner shard whose f32 values the reduce needs or -1) for a prepacked bucket,
  // or shard elements 0 when this configuration cannot take prepacked input.
  std::array<int64_t, 3> prepack_shape(int64_t n) const;
  // Enqueue the deferred SGD epilogue; with `after_producer`, after everything currently enqueued on
  // `producer`. The flag is separate from the handle because the default (legacy null) stream IS nullptr:
  // torch's default stream hands us 0, and treating that as "no producer" skipped the ordering wait.
  // `seq` (0: whoever holds the slot) names the request: a handle whose slot was since reused by a newer
  // request never commits or waits on that newer request's behalf (its own epilogue was committed when the
  // slot was reused, see submit()).
  void commit(int slot, bool after_producer, hipStream_t producer, uint32_t seq = 0);
  void wait_stream(int slot, hipStream_t s, uint32_t seq = 0);  // GPU-side wait
  bool query(int slot, uint32_t seq = 0);                       // host: request done?
  // the slot's host-mapped done word: the last completed sequence number, written only when done words are on
  // (FAN_DONE_WORDS=1; off by default, then it stays 0 and debug_status reports the done event instead)
  uint32_t done_word(int slot) const { return flags_host_[slot * 16]; }
  uint32_t slot_seq(int slot) const { return table_->slot(slot).seq; }
  void synchronize(int slot, double timeout_s = -1.0, uint32_t seq = 0);  // host: bounded wait (throws)
  float latency_ms(int slot);
  void set_timing(bool on) { timing_ = on; }
  // Request tracing (device timestamps per phase, see TracePoint): enabling resets the trace pool; requests
  // beyond its capacity are counted as dropped. trace_summary() waits for the traced requests.
  void set_tracing(bool on, int capacity = 1024);
  bool tracing() const { return tracing_; }
  TraceSummary trace_summary();
  // Side-stream engine: run each request's epilogue on the stream passed to commit() (after its communication
  // phase) instead of on the comm stream.
  void set_epilogue_on_producer(bool on) { table_->set_epi_on_producer(on); }
  bool epilogue_on_producer() const { return table_->config().epi_on_producer; }
  bool side_epilogue() const { return table_->config().side_epi; }
  std::string diagnostics(int slot) const;
  // Debug snapshot (the NIC's debug_status register, hw/all_reduce.sv:1415-1421), JSON: engine configuration,
  // every slot (sequence, pending epilogue, done word, stream kind), counters, the communicator's async error and,
  // on the P2P transport, its flag block and device stall counters. Host-only reads except the P2P flag copy.
  std::string debug_status();
  bool verify() const { return verify_; }
  // verify mode: raise (with site, row, checksums, sequence numbers) if any message so far failed its check
  void check_verify();
  // test-only fault injection (FAN_FAULT grammar, see verify.h); replaces the rules taken from the environment
  void set_fault(const std::string& spec) { fault_ = FaultInjector(spec); }
  uint64_t requests() const { return submitted_; }
  const EngineCounters& counters() const { return counters_; }
  uint64_t skipped_waits() const { return table_->skipped_waits(); }  // redundant cross-stream waits elided
  void reset_counters() { counters_ = EngineCounters{}; }
  int64_t wire_bytes(const EngineLayout& L) const;
  // device scratch the engine holds (wire staging buffers; per-slot gathered wire of deferred requests)
  size_t scratch_bytes() const {
    size_t t = 0;
    for (const auto& kv : scratch_) t += kv.second.second;
    return t;
  }

 private:
  // Per-slot engine data beside the state machine (slot_table.h holds sequence / pending / streams / events).
  struct SlotExtra {
    hipEvent_t t0 = nullptr, t1 = nullptr;
    bool timed = false;
    bool counted = false;   // device time already added to counters_
    double t_issue = 0.0;
    int trace = -1;  // index into trace_pool_ (-1: not traced)
  };
  std::array<SlotExtra, kSlots> extra_;
  // Inline requests record their done event lazily (only when a host query / other stream needs it): an event
  // marker after every inline epilogue left the GPU idle ~5.5 us before the next GEMM (3x per step,
  // profiles/r2_lazy_done_event.txt). FAN_LAZY_DONE=0 records every request's done event at commit.
  HipSlotDevice dev_;
  std::unique_ptr<SlotTable<HipSlotDevice>> table_;
  std::vector<hipEvent_t> slot_events_;
  struct RequestTrace {
    hipEvent_t ev[kTpCount] = {};
    int64_t logical_bytes = 0, wire_bytes = 0;
    size_t hop_first = 0, hop_count = 0;  // ring rounds: 4 events each in hop_pool_
    bool hop_kernel_first = false;         // point order: credit, kernels, ready (copying) or credit, ready, kernels
  };
  std::vector<hipEvent_t> hop_pool_;
  size_t hop_used_ = 0;
  void hop_mark(int point);  // ring round timestamp of the traced request being built (point 0..3)
  // verify mode on the direct P2P paths: tag a message where it landed (trailer of its slot) / check one on arrival
  void tag_direct(const uint8_t* msg, size_t bytes, uint8_t* trailer, uint32_t seq, hipStream_t st);
  void verify_direct(const uint8_t* msg, size_t bytes, const uint8_t* trailer, uint32_t seq, uint32_t site,
                     uint32_t row, hipStream_t st);
  // record trace point tp of the request being built on the stream its phases run on
  void mark(int tp) {
    trace_marked_ |= 1u << tp;
    if (cur_trace_ >= 0) FAN_HIP_CHECK(hipEventRecord(trace_pool_[cur_trace_].ev[tp], run_stream_));
  }
  void count_peers(size_t bytes, P2PComm* direct = nullptr);  // `bytes` sent to every other rank
  uint8_t* scratch(const std::string& key, size_t bytes);
  std::vector<EpiThunk> run_mesh(const EngineLayout& L, const void* grad, int gdt, float* master,
                                              bf16_t* lp, float* mom, int64_t n_valid, SgdParams p, bool update,
                                              float* out_sum, const uint8_t* prepacked, int64_t prepacked_elems);
  std::vector<EpiThunk> run_mesh_direct(P2PComm* d, const EngineLayout& L, const void* grad, int gdt, float* master,
                                        bf16_t* lp, float* mom, int64_t n_valid, SgdParams p, bool update,
                                        float* out_sum, const uint8_t* prepacked, bool defer);
  std::vector<EpiThunk> run_mesh_chunked(const EngineLayout& L, const void* grad, int gdt, float* master,
                                         bf16_t* lp, float* mom, int64_t n_valid, SgdParams p, bool update,
                                         float* out_sum, const uint8_t* prepacked, bool defer);
  std::vector<EpiThunk> run_ring(const EngineLayout& L, const void* grad, int gdt, float* master,
                                              bf16_t* lp, float* mom, int64_t n_valid, SgdParams p, bool update,
                                              float* out_sum, const uint8_t* prepacked, int64_t prepacked_elems);
  std::vector<EpiThunk> run_ring_direct(P2PComm* d, const EngineLayout& L, const void* grad, int gdt, float* master,
                                        bf16_t* lp, float* mom, int64_t n_valid, SgdParams p, bool update,
                                        float* out_sum, const uint8_t* prepacked);

  Comm* comm_;
  int rank_, world_, device_;
  EngineConfig cfg_;
  std::vector<std::vector<int>> orders_;
  hipStream_t stream_ = nullptr;
  hipStream_t aux_stream_ = nullptr;  // chunked mesh: owner reduces + per-chunk epilogues beside the collectives
  hipStream_t epi_stream_ = nullptr;  // world-1 side epilogues (normal priority: the producer's GEMMs keep theirs)
  hipEvent_t cev_[4][2] = {};         // chunked mesh pipeline events: [all-to-all, reduce, all-gather, epilogue][parity]
  // world 1 without forced collectives: nothing to overlap, so requests run inline on the producer's
  // stream (no cross-stream event packets); run_stream_ is the stream of the request being issued.
  bool inline_ = false;
  bool shard_upd_ = false;
  hipStream_t run_stream_ = nullptr;
  volatile uint32_t* flags_host_ = nullptr;  // host-mapped done words (one 64-B line per slot)
  uint32_t* flags_dev_ = nullptr;
  bool timing_ = false;
  uint64_t submitted_ = 0;
  EngineCounters counters_;
  std::map<std::string, std::pair<uint8_t*, size_t>> scratch_;
  int epi_slot_ = 0;  // slot of the request being built
  hipStream_t cur_producer_ = nullptr;  // producer stream of the request being built
  // deferred chunked requests: the whole-bucket gathered wire, one per bucket size, and who used it last
  struct GallBuf {
    int slot = 0;
    uint32_t seq = 0;
    hipEvent_t free = nullptr;  // recorded on the epilogue stream after the last user's epilogue
  };
  std::map<std::string, GallBuf> gall_;
  bool cur_defer_ = false;  // the request being built defers its epilogue
  bool tracing_ = false;
  std::vector<RequestTrace> trace_pool_;
  size_t trace_used_ = 0;
  uint64_t trace_dropped_ = 0;
  int cur_trace_ = -1;  // trace of the request being built
  // verify mode / fault injection (verify.h): tag buffers (device), first-error block (device) + its host mirror
  bool verify_ = false;
  FaultInjector fault_;
  uint32_t* tags_ = nullptr;  // [kTagRows][4] x 5 regions: send, recv, scratch, gather-send, gather-recv
  VerifyError* verr_dev_ = nullptr;
  VerifyError* verr_host_ = nullptr;
  uint32_t req_seq_ = 0;  // sequence number of the request being built (what its tags carry)
  static constexpr int kTagRows = 64;
  uint32_t* tag_region(int r) { return tags_ + (size_t)r * kTagRows * 4; }
  void verify_rows(const uint8_t* rows, size_t row_bytes, int nrows, const uint32_t* recv_tags, uint32_t site,
                   uint32_t row_base, hipStream_t st);
  unsigned trace_marked_ = 0;  // trace points the schedule of the request being built has recorded
  // Scratch that a deferred epilogue reads: per request slot, so a later request of the same size cannot
  // overwrite it before this request commits (the trainer commits every request at the end of backward).
  uint8_t* epi_scratch(const std::string& base, size_t bytes);
};

}  // namespace fan

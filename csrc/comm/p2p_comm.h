// Direct peer-to-peer transport over xGMI (SURVEY.md §5.8 transport (b), §7.1 transport_p2p).
//
// No RCCL in the data path: every rank exposes a receive ARENA and a FLAG block in its HBM through HIP IPC;
// peers write message payloads straight into the arena over xGMI (stream-ordered device copies into the
// IPC-mapped peer pointer) and then publish a 64-bit sequence number into the receiver's flag block with
// hipStreamWriteValue64. The receiver's stream waits on that flag with hipStreamWaitValue64 — a
// command-processor wait, so no CU spins and nothing can deadlock on occupancy — copies the payload out
// and acknowledges into the sender's flag block, which frees that arena slot for reuse.
//
// Arena: world x depth slots of slot_bytes, at most kMaxArenaBytes in all (a ring of `depth` slots per sender,
// indexed by sequence mod depth; depth 2 = double-buffered by parity), so a sender only stalls when it is `depth`
// messages ahead of a receiver — a ring hop streamed in P sub-slices consumes each message P sub-rounds after it
// lands and needs depth >= P + 1.
// Flags: ready[world] + ack[world] (uint64 each, monotone sequence numbers).
// Reference analogue: the NIC's Ethernet link + credit flow control (hw/all_reduce.sv:468-483) and the
// done-flag writes (hw/all_reduce.sv:1368-1375); here sequence numbers play the role of both.
//
// Memory ordering (why a reader never sees a stale payload, across GPUs whose per-XCD L2s are not coherent):
//   1. writer: the producing kernels store the payload into the peer's arena (stores over xGMI land in the peer's
//      HBM; the writer's own L2 does not keep remote lines); before the flag writes the stream records a system-scope
//      release event (hipEventReleaseToSystem: the command processor waits for the round's kernels and writes back
//      / makes their stores visible at system scope) — FAN_P2P_RELEASE=block|thread put the release inside the
//      kernels instead (bfp_format.h p2p_release);
//   2. the flag write (hipStreamWriteValue64) is stream-ordered after that release, so it becomes visible to the
//      peer only after the payload;
//   3. reader: its stream's hipStreamWaitValue64 (the command processor polls the flag in memory, not a cache)
//      releases the copy-out kernel only once the flag carries the message's sequence number;
//   4. arena and flags are allocated UNCACHED (hipDeviceMallocUncached): the reader's loads bypass L2, so no stale
//      line from the previous message in that slot can be hit — the acquire side needs no invalidate. (If the
//      allocator refuses the flag, coarse-grained memory is used and the reader's kernel-start L2 invalidate does
//      that job; uncached() reports which.)
//   5. WAR: a sender reuses a parity slot only after the receiver's ack (written after its copy-out kernel
//      completed) shows the previous message in it was consumed.
//   Cross-device peers: the command-processor release (mode "cp", the default) was measured only with every rank on
//   ONE GPU, where system and device scope coincide. Whether posted xGMI stores to another GPU's arena are visible
//   before a flag written after a hipEventReleaseToSystem marker is UNVERIFIED on this pool (no multi-GPU node), so
//   connect() switches a process whose peers live on other devices to the in-kernel per-workgroup system-scope
//   release ("block") unless FAN_P2P_RELEASE names a mode explicitly; verify mode (trailer tags, below) checks the
//   ordering in band on whichever mode runs.
// Verify trailer: the last kTrailerBytes of every slot hold up to 16 message tags ({s1, s2, seq, bytes}, verify.h);
// messages use at most payload_bytes() of a slot.
// Pure data movement (prepacked sends, FORWARD hops, arena -> scratch) goes through move(): the CU copy kernel, or
// with FAN_P2P_COPY=sdma the copy engines (hipMemcpyDeviceToDeviceNoCU: no CU, so beside a persistent GEMM that
// holds every CU the copy still runs).
// abort() releases every stream parked on this rank's flags (poison value) so a dead peer cannot hang the GPU;
// the communicator then refuses further calls.
// Kernel flags (set_kernel_flags, FAN_P2P_FLAGS=kernel; the A/B's *_kflag arms): the flag writes and waits run as
// tiny kernels instead of command-processor packets — a one-workgroup kernel stores each ready / ack word with a
// system-scope release (sc0 sc1), and a one-workgroup kernel spins (relaxed system-scope loads + s_sleep, bounded:
// past ~8 s it records an error and gives up) until every awaited word reaches its sequence number, then acquires at
// system scope; the consuming kernel follows it in stream order (the consumer spins in-kernel).
// The CP-independent path in case command-processor polling of another GPU's uncached word is slow or misbehaves on
// xGMI; it costs a kernel launch per flag batch. abort()'s poison values release these spins too.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "comm/native_comm.h"

namespace fan {

struct P2PCopy {
  const void* src;
  void* dst;
  size_t bytes;
};
// All segments in one (or few) kernel launches; segments 16-B aligned, sizes multiples of 16 B.
void launch_multi_copy(const std::vector<P2PCopy>& segs, hipStream_t stream);
// Kernel flags (P2PComm::set_kernel_flags): store each word's value with a system-scope release / spin until every
// word reaches its value (bounded; *err = 1 when a spin gave up), then a system-scope acquire. One launch per batch
// of up to 16 words.
void launch_flag_write(const std::vector<std::pair<uint64_t*, uint64_t>>& w, hipStream_t stream);
void launch_flag_wait(const std::vector<std::pair<uint64_t*, uint64_t>>& w, unsigned* err, hipStream_t stream);
// Segments merged into contiguous runs (source and destination both continue the previous segment); empty ones
// dropped. The copy-engine path issues one command per run.
std::vector<P2PCopy> coalesce_copies(const std::vector<P2PCopy>& segs);
// Whether a round must record the system-scope release event before its flag writes: always in release mode 3
// (cp); in the in-kernel modes only when bytes of the round were moved outside a peer-storing kernel (copy engines,
// hipMemcpyAsync fallback), since no kernel released those.
bool p2p_release_event_needed(int mode, bool copy_engine_bytes);

// The flag words one round touches (pure host logic, unit-tested on CPU: tests/test_p2p_host_logic.py). Flag block of
// every rank: words [0, world) "ready from src", [world, 2 world) "ack from dst". A round with sequence number seq
// sending to `to` and receiving from `from`:
//   credit_waits: own word world + p >= the sequence last sent to p in this round's slot (seq % depth), if any
//   ready_writes: peer p's word rank := seq (after the payload)
//   ready_waits:  own word q >= seq (before reading q's message)
//   ack_writes:   peer q's word world + rank := seq (after the consumer: frees the slot for q)
struct FlagRef {
  int peer;    // whose flag block (== rank for an own word)
  int word;
  uint64_t value;
};
struct RoundFlags {
  std::vector<FlagRef> credit_waits, ready_writes, ready_waits, ack_writes;
};
RoundFlags p2p_round_flags(int rank, int world, uint64_t seq, const std::vector<int>& to, const std::vector<int>& from,
                           const std::vector<uint64_t>& last_sent_in_slot);

class P2PComm : public Comm {
 public:
  P2PComm(int rank, int world, int device, size_t slot_bytes, int depth = 2);
  ~P2PComm() override;
  static constexpr size_t kTrailerBytes = 256;  // per slot: 16 verify tags of 16 B
  // the arena (world x depth slots) is one IPC-exported allocation of at most this size: slot_bytes() is clamped to
  // fit (FAN_P2P_ARENA_MAX_MB overrides; see the constructor for the 2 GiB import hang that sets it)
  static constexpr size_t kMaxArenaBytes = (size_t)1 << 30;
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  size_t slot_bytes() const { return slot_; }
  int depth() const { return depth_; }
  size_t payload_bytes() const { return slot_ - kTrailerBytes; }  // what the messages of one slot may use

  // IPC bootstrap: this rank's (arena, flags) handles as bytes; connect() with every rank's bytes (in rank
  // order) opens the peers' mappings. connect_local() wires ranks living in one process (no IPC).
  std::string handles() const;
  void connect(const std::vector<std::string>& all_handles);
  static void connect_local(const std::vector<P2PComm*>& ranks);

  void sendrecv(const std::vector<P2POp>& sends, const std::vector<P2POp>& recvs, hipStream_t s) override;
  P2PComm* direct() override { return this; }

  // Direct rounds (every rank sends to every peer): the engine's producing kernel stores straight into the peers'
  // receive slots and its consuming kernel reads this rank's slots in place — no staging copy on either side
  // (the encoder is the sender, as on the NIC, hw/all_reduce.sv:1155-1166).
  //   begin():    new round; the stream waits until every peer acknowledged the previous message in the slots
  //               this round reuses (credit flow control, hw/all_reduce.sv:468-483)
  //   dst(p):     where to store the message for peer p (peer p's arena slot of this rank; p == rank: this
  //               rank's own slot, for a producer that also keeps its own copy)
  //   publish():  ready flags to every peer, stream-ordered after the producer (which released its stores)
  //   wait():     the stream waits for every peer's ready flag; then src_base() + q * src_stride() is the
  //               message from rank q (q == rank: whatever the producer stored into dst(rank))
  //   release():  acknowledge every peer's slot (after the consumer), freeing it for the sender
  struct Round {
    uint64_t seq;
  };
  Round begin(hipStream_t s);
  uint8_t* dst(const Round& r, int peer) const { return slot_ptr(peer_arena_[peer], rank_, r.seq); }
  void publish(const Round& r, hipStream_t s);
  void wait(const Round& r, hipStream_t s);
  const uint8_t* src_base(const Round& r) const { return arena_ + (r.seq % depth_) * slot_; }
  size_t src_stride() const { return (size_t)depth_ * slot_; }
  void release(const Round& r, hipStream_t s);
  // The same round protocol restricted to a peer subset (ring rounds: send to the downstream neighbours, receive
  // from the upstream ones). Every rank must start the same number of rounds (begin / begin_to) in the same order.
  Round begin_to(const std::vector<int>& to, hipStream_t s);
  void publish_to(const Round& r, const std::vector<int>& to, hipStream_t s);
  void wait_from(const Round& r, const std::vector<int>& from, hipStream_t s);
  void release_from(const Round& r, const std::vector<int>& from, hipStream_t s);
  // message from rank `src` in round r, in this rank's arena
  const uint8_t* src(const Round& r, int from) const { return slot_ptr(arena_, from, r.seq); }
  // verify tag k (16 B) of this rank's slot at `peer` / of `from`'s slot here, for round r
  uint8_t* dst_tag(const Round& r, int peer, int k) const { return dst(r, peer) + payload_bytes() + 16 * (size_t)k; }
  uint8_t* src_tag(const Round& r, int from, int k) const {
    return slot_ptr(arena_, from, r.seq) + payload_bytes() + 16 * (size_t)k;
  }
  // flag writes / waits as kernels instead of command-processor packets (see the header comment); switch only
  // between rounds (the A/B flips it per arm after the previous arm's requests finished)
  bool kernel_flags() const { return kflags_; }
  void set_kernel_flags(bool on) { kflags_ = on; }
  // a kernel-flag wait gave up after its spin bound (0: never); host read, for diagnostics
  unsigned kernel_flag_error() const;
  // pure copies (see the header comment): CU kernel or copy engines
  void move(const std::vector<P2PCopy>& segs, hipStream_t s);
  bool sdma() const { return sdma_; }
  void set_sdma(bool on) { sdma_ = on; }
  // some peer's arena lives on another GPU (or host): set by connect()
  bool cross_device() const { return cross_device_; }
  void all_to_all(const void* send, void* recv, size_t bytes_per_peer, hipStream_t s) override;
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override;
  std::string async_error() override { return aborted_ ? "p2p transport aborted" : ""; }
  void abort() override;
  int ranks_seen() override {
    int n = 1;
    for (int p = 0; p < world_; ++p) n += (p != rank_ && peer_arena_[p] != nullptr && peer_flags_[p] != nullptr);
    return n;
  }
  const char* kind() const override { return "p2p"; }
  uint64_t sequence() const { return seq_; }
  bool uncached() const { return uncached_; }
  const std::string& arena_memory() const { return arena_mem_; }
  uint8_t* arena() const { return arena_; }
  size_t arena_bytes() const { return (size_t)world_ * depth_ * slot_; }

  // Device-side stall counters (the NIC's stall_* / credit registers, hw/all_reduce.sv:892-1085, 468-483): every
  // flag wait the command processor parks a stream on, split into ready waits (data from a peer) and credit waits
  // (a peer acknowledging a slot); with timing on, each wait is bracketed by timing events on its stream, so the
  // stall time is device time. bytes_to_peer: message bytes this rank stored into / copied to each peer.
  struct Stats {
    uint64_t ready_waits = 0, credit_waits = 0, timed_waits = 0;
    double ready_stall_ms = 0.0, credit_stall_ms = 0.0;
    std::vector<int64_t> bytes_to_peer;
  };
  void set_timing(bool on) { timing_ = on; }
  // wait=true: waits for the timed waits' events. wait=false (diagnostics of a possibly hung run): folds in only
  // the timed waits whose end event has already completed and keeps the others for later.
  Stats stats(bool wait = true);
  void reset_stats();
  void count_sent(int peer, size_t bytes) { bytes_to_peer_[peer] += (int64_t)bytes; }
  // flag block snapshot (ready-from-src[world], ack-from-dst[world]) for diagnostics. The copy runs on a stream of
  // its own and is polled for at most timeout_s, so a snapshot taken while a stream is parked on one of these flags
  // (the hang it is meant to diagnose) returns instead of blocking; empty when the copy did not complete in time.
  std::vector<uint64_t> flags_snapshot(double timeout_s = 2.0) const;

 private:
  void copy(const std::vector<P2PCopy>& segs, hipStream_t s);
  uint8_t* slot_ptr(uint8_t* arena, int src, uint64_t seq) const {
    return arena + ((size_t)src * depth_ + seq % depth_) * slot_;
  }
  int rank_, world_, device_;
  size_t slot_;
  int depth_;
  uint8_t* arena_ = nullptr;   // local receive arena
  uint64_t* flags_ = nullptr;  // local flags: [0, world) ready-from-src, [world, 2 world) ack-from-dst
  std::vector<uint8_t*> peer_arena_;
  std::vector<uint64_t*> peer_flags_;
  std::vector<bool> opened_;   // peer mapping opened through IPC (to be closed)
  std::vector<std::vector<uint64_t>> last_sent_;  // per slot index (seq % depth): last sequence sent to each peer
  uint64_t seq_ = 0;
  bool aborted_ = false;
  // flag operations of one round step, batched: one command-processor packet per word, or one kernel for all
  using FlagOp = std::pair<uint64_t*, uint64_t>;
  std::vector<FlagOp> flag_ptrs(const std::vector<FlagRef>& refs) const;
  std::vector<int> others() const;
  void write_flags(hipStream_t s, const std::vector<FlagOp>& w);
  void wait_flags(hipStream_t s, const std::vector<FlagOp>& w, bool credit);
  bool kflags_ = false;
  unsigned* kflag_err_ = nullptr;  // device word: a kernel-flag wait gave up
  // stall accounting
  bool timing_ = false;
  uint64_t ready_waits_ = 0, credit_waits_ = 0;
  struct TimedWait {
    hipEvent_t ev[2];
    bool credit;
  };
  std::vector<TimedWait> tw_;
  size_t tw_used_ = 0;
  double stall_ms_[2] = {0.0, 0.0};
  uint64_t timed_ = 0;
  std::vector<int64_t> bytes_to_peer_;
  bool uncached_ = false;
  std::string arena_mem_;
  hipEvent_t rel_ev_ = nullptr;  // system-scope release before the flag writes (release mode "cp", copy-engine bytes)
  bool sdma_ = false;
  bool nonkernel_pending_ = false;  // bytes of the current round moved by the copy engines / hipMemcpyAsync
  bool cross_device_ = false;
  void release_before_flags(hipStream_t s);
};

}  // namespace fan

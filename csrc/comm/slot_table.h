// Request-slot state machine of the all-reduce engine, free of HIP: the host-side logic that decides which stream
// waits for which event, when a deferred epilogue is committed and on which stream, when a request counts as done.
//
// Reference behaviour: the NIC accepts at most 8 requests, processes them in
// order and signals each by writing 1 to done_addr + done_id, done_id cycling 0..7 (hw/all_reduce.sv:1228,
// 1368-1375; sw/mlp_mpi_example_f32.cpp:114-180). Here a request is (a) a communication phase enqueued at submit and
// (b) a decode + SGD epilogue that may be DEFERRED until the producer's remaining work (the bwd-data GEMM that still
// reads the weights) is enqueued; completion is a 32-bit sequence number the GPU writes into host-mapped memory.
//
// The class is a template over a device policy D so the same code runs on HIP (engine.cpp) and on a simulated
// device with random stream interleavings under AddressSanitizer / UBSan (tests/native/slot_table_selftest.cpp).
// D provides:
//   using Stream; using Event;                           (Stream values compare by identity; any value is a real
//                                                         stream, including the null/legacy stream 0)
//   void record(Event, Stream); void wait(Stream, Event); bool query(Event);
//   void write_done(Stream, int slot, uint32_t seq);     GPU writes the done word of a slot, stream-ordered
//   uint32_t read_done(int slot);                        host read of that word
//
// Invariants (checked by the self-test):
//   I1 a request's epilogue runs after its own communication phase and, when committed "after the producer",
//      after everything the producer stream had enqueued at commit time;
//   I2 a slot's buffers are not rewritten by a new request while the previous request's epilogue on that slot
//      (wherever it runs) may still read them;
//   I3 query()/synchronize() report a request done only once its epilogue has executed; wait_stream(s) orders
//      stream s after it; both stay correct for a handle whose slot has since been reused (superseded), and across
//      the 32-bit sequence wrap-around;
//   I4 more than kSlots deferred requests never drop one: the oldest is committed when its slot is needed.
#pragma once
#include <array>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <vector>

namespace fan {

template <class D>
class SlotTable {
 public:
  using Stream = typename D::Stream;
  using Event = typename D::Event;
  using Thunk = std::function<void(Stream)>;
  static constexpr int kSlots = 8;

  struct Config {
    bool inline_mode = false;     // world 1, no collectives: requests run in the producer's stream order
    bool epi_on_producer = false; // multi-rank: epilogue on the committing (compute) stream after comm_done
    bool side_epi = false;        // world 1: epilogue on the side stream after the producer's enqueued work
    bool lazy_done = true;        // inline: record the done event only when something needs it
    bool elide_waits = true;      // skip cross-stream waits implied by an earlier wait on the comm stream
    // multi-rank requests finishing on the comm stream: the GPU writes the slot's done word into host memory (the
    // NIC's done write). Off: their completion is the done event like every other request's — the write is a blit
    // dispatch on the comm stream (hipStreamWriteValue32, ~20 us of stream time with its two dispatch gaps per
    // request, profiles/r5_config5_comm_trace.txt)
    bool done_words = true;
    Stream comm{};                // the engine's communication stream (multi-rank)
    Stream side{};                // the world-1 side-epilogue stream (side_epi)
  };

  struct Slot {
    Event ready{}, update{}, comm_done{}, done{};
    uint32_t seq = 0;
    bool pending = false;        // epilogue not yet committed
    bool used = false;           // has held a request
    Stream stream{};             // stream the communication phase ran on
    Stream epi_stream{};         // stream the epilogue was enqueued on
    bool done_lazy = false;      // inline request whose done event is not recorded yet
    bool keep_done = false;      // the engine times / traces this request: record its done event at commit
    bool on_producer = false;    // multi-rank request that ran on its producer stream (begin(.., true))
    uint64_t comm_done_mark = 0; // comm-stream order of the last comm_done / done record (0: not on the comm stream)
    uint64_t done_mark = 0;
    std::vector<Thunk> thunks;
  };

  // hooks the engine uses for its timing / tracing events (called on the epilogue stream, after the thunks)
  std::function<void(int slot, Stream epi)> on_epilogue;
  // called when a deferred request is force-committed because its slot is needed (> kSlots deferred)
  std::function<void(int slot)> on_forced_commit;

  SlotTable(D& dev, Config cfg, const std::vector<Event>& events) : dev_(dev), cfg_(cfg) {
    if (events.size() != (size_t)kSlots * 4) throw std::invalid_argument("SlotTable: need 4 events per slot");
    for (int i = 0; i < kSlots; ++i) {
      slots_[i].ready = events[i * 4 + 0];
      slots_[i].update = events[i * 4 + 1];
      slots_[i].comm_done = events[i * 4 + 2];
      slots_[i].done = events[i * 4 + 3];
    }
  }

  const Config& config() const { return cfg_; }
  void set_epi_on_producer(bool on) { cfg_.epi_on_producer = on && !cfg_.inline_mode; }
  void set_seq(uint32_t s) { seq_ = s; }  // test hook: start near the 32-bit wrap-around
  uint32_t last_seq() const { return seq_; }
  int next_slot() const { return next_; }
  const Slot& slot(int i) const { return slots_.at(i); }
  uint64_t skipped_waits() const { return skipped_waits_; }

  // A new request from `producer`: takes the next slot (force-committing a still-deferred occupant), orders the
  // request after anything that may still read that slot's buffers, and returns (slot, stream its communication
  // phase runs on). For a multi-rank request the comm stream waits for the producer's work so far.
  struct Begin {
    int slot;
    Stream run;
    uint32_t seq;  // the sequence number this request will carry
  };
  // on_producer (multi-rank): this request's communication phase runs on the producer stream itself instead of the
  // comm stream — for the last request of a backward, which nothing is left to overlap with: it saves the two
  // cross-stream hand-offs (producer -> comm, comm -> the next forward; ~25-30 us each on MI355X,
  // profiles/r5_forced_step_timeline.txt) on the critical path. Ordering then is the producer's own stream order.
  Begin begin(Stream producer, bool on_producer = false) {
    const int s = next_;
    next_ = (s + 1) % kSlots;
    Slot& sl = slots_[s];
    if (sl.pending) {  // I4: the 9th deferred request commits the oldest, ordered after the producer
      if (on_forced_commit) on_forced_commit(s);
      commit_slot(s, true, producer);
    }
    const Stream run = (cfg_.inline_mode || on_producer) ? producer : cfg_.comm;
    // I2: the slot's previous epilogue may run on another stream than this request and read this slot's
    // buffers (a side epilogue, or one committed on another producer stream). A multi-rank request waits for
    // `ready` on the producer below, which covers an epilogue enqueued there.
    if (sl.used && !(sl.epi_stream == run) && !(!cfg_.inline_mode && sl.epi_stream == producer)) {
      ensure_done(sl);
      wait_m(run, sl.done, sl.done_mark);
    }
    sl.stream = run;
    sl.keep_done = false;
    sl.on_producer = !cfg_.inline_mode && on_producer;
    if (!cfg_.inline_mode && !(run == producer)) {
      dev_.record(sl.ready, producer);
      dev_.wait(run, sl.ready);
    } else if (!cfg_.inline_mode) {
      // on-producer request: the communicator's earlier requests (on the comm stream) finish first, so its
      // collectives / P2P rounds never run beside theirs (RCCL serialises a communicator's operations by issue order;
      // a P2P flag wait parked on this stream would otherwise block a comm-stream round a peer needs, when the two
      // streams share a hardware queue). Usually already complete when the backward's last GEMM ends.
      const uint64_t m = record_m(sl.ready, cfg_.comm);
      dev_.wait(producer, sl.ready);
      cover(producer, m, true);
    }
    return Begin{s, run, following(seq_)};
  }

  // The request's communication phase is enqueued (on Begin::run); `thunks` enqueue its epilogue on a given
  // stream. Immediate requests commit now (in the comm stream's order).
  uint32_t end(int s, std::vector<Thunk> thunks, bool defer) {
    Slot& sl = slots_.at(s);
    if (!cfg_.inline_mode) sl.comm_done_mark = record_m(sl.comm_done, sl.stream);
    sl.thunks = std::move(thunks);
    sl.pending = true;
    sl.used = true;
    sl.seq = seq_ = following(seq_);
    if (!defer) commit_slot(s, false, Stream{});
    return sl.seq;
  }

  // Enqueue a deferred epilogue; `seq` (0: whoever holds the slot) names the request — a superseded handle's
  // epilogue was committed when its slot was reused, so it never commits the newer request.
  void commit(int s, bool after_producer, Stream producer, uint32_t seq = 0) {
    Slot& sl = slots_.at(s);
    if (seq != 0 && seq != sl.seq) return;
    commit_slot(s, after_producer, producer);
  }

  // GPU-side: stream `st` waits for the request.
  void wait_stream(int s, Stream st, uint32_t seq = 0) {
    Slot& sl = slots_.at(s);
    // A superseded request: if the newer one is still pending, the slot's done event still marks the old
    // request's completion; otherwise it marks the newer one, later in every stream order the old request
    // shares (a conservative wait). Never commit the newer request on the old handle's behalf.
    const bool own = seq == 0 || seq == sl.seq;
    if (own && sl.pending) commit_slot(s, true, st);
    if (!(st == sl.epi_stream) || !own) {
      ensure_done(sl);
      wait_m(st, sl.done, sl.done_mark);
    }
  }

  // Host: is the request done (its epilogue executed)?
  bool query(int s, uint32_t seq = 0) {
    Slot& sl = slots_.at(s);
    ensure_done(sl);  // a lazily recorded done event (this request's, or a superseded one's: conservative)
    if (seq != 0 && seq != sl.seq) {
      // superseded: done if the newer request's done word has passed it (wrap-safe), else the slot's done event
      if (!cfg_.inline_mode && cfg_.done_words && ((dev_.read_done(s) - seq) & 0xFFFFFFFFu) < (1u << 31)) return true;
      return dev_.query(sl.done);
    }
    if (sl.pending) return false;
    if (cfg_.inline_mode || sl.on_producer || !cfg_.done_words || !(sl.epi_stream == sl.stream))
      return dev_.query(sl.done);
    return dev_.read_done(s) == sl.seq;
  }

  // commit an own pending request before a host wait (synchronize)
  void commit_for_host_wait(int s, uint32_t seq) {
    Slot& sl = slots_.at(s);
    if ((seq == 0 || seq == sl.seq) && sl.pending) commit_slot(s, false, Stream{});
  }

  // Inline requests complete in their producer's stream order, so nothing needs their done event unless the host
  // polls it or another stream waits on it: record it then (later in that stream = a conservative completion point).
  void ensure_done(Slot& sl) {
    if (!sl.done_lazy) return;
    sl.done_mark = record_m(sl.done, sl.epi_stream);
    sl.done_lazy = false;
  }
  void ensure_done(int s) { ensure_done(slots_.at(s)); }
  void set_keep_done(int s, bool on) { slots_.at(s).keep_done = on; }
  bool done_words() const { return cfg_.done_words && !cfg_.inline_mode; }
  // completion of a slot's request for diagnostics, without recording anything: -1 unknown (pending, or its done
  // event still lazy), else the done event's query
  int peek_done(int s) {
    Slot& sl = slots_.at(s);
    if (!sl.used) return 1;
    if (sl.pending || sl.done_lazy) return -1;
    return dev_.query(sl.done) ? 1 : 0;
  }

  // destructor helper: every slot's epilogue that may still run
  template <class F>
  void for_each_used(F f) {
    for (int i = 0; i < kSlots; ++i)
      if (slots_[i].used) {
        ensure_done(slots_[i]);
        f(i, slots_[i]);
      }
  }

 private:
  // sequence numbers run 1, 2, ..., 2^32-1, 1, ...: 0 means "no request / whoever holds the slot"
  static uint32_t following(uint32_t q) { return q == 0xFFFFFFFFu ? 1u : q + 1u; }

  void commit_slot(int s, bool after_producer, Stream producer) {
    Slot& sl = slots_[s];
    if (!sl.pending) return;
    sl.epi_stream = sl.stream;
    bool on_producer = false;
    if (cfg_.epi_on_producer && !cfg_.inline_mode && after_producer && !(producer == sl.stream)) {
      // epilogue on the producer (compute) stream, after the request's communication phase: it runs after
      // everything already enqueued there and never concurrently with the producer's GEMMs
      wait_m(producer, sl.comm_done, sl.comm_done_mark);
      sl.epi_stream = producer;
      on_producer = true;
    } else if (cfg_.side_epi && after_producer) {
      // world 1: no communication phase; decode + SGD on the side stream after the producer's enqueued work and
      // after the request's own inline work (on the stream it was submitted from, when another stream commits)
      dev_.record(sl.update, producer);
      dev_.wait(cfg_.side, sl.update);
      if (!(producer == sl.stream)) {
        sl.comm_done_mark = record_m(sl.comm_done, sl.stream);
        dev_.wait(cfg_.side, sl.comm_done);
      }
      sl.epi_stream = cfg_.side;
    } else if (after_producer && !(producer == sl.stream)) {
      dev_.record(sl.update, producer);
      dev_.wait(sl.stream, sl.update);
    }
    for (auto& t : sl.thunks) t(sl.epi_stream);
    sl.thunks.clear();
    if (on_epilogue) on_epilogue(s, sl.epi_stream);
    // multi-rank requests finishing on the comm stream: the GPU writes the done word ("write 1 to done_addr +
    // done_id"); requests finishing on the critical compute stream skip that packet: their completion is the event
    // (on-producer requests too: the host-memory write cost ~50 us before the next forward's first kernel,
    // profiles/r5_forced_step_timeline.txt)
    if (cfg_.done_words && sl.epi_stream == sl.stream && !cfg_.inline_mode && !sl.on_producer)
      dev_.write_done(sl.stream, s, sl.seq);
    // Lazy done event: the epilogue ran in its own stream's order (inline requests; multi-rank epilogues on the
    // producer stream), so nothing needs the event unless the host polls the request or another stream waits on
    // it; ensure_done() records it then. Each eager record is a marker packet on the critical compute stream.
    sl.done_lazy = cfg_.lazy_done && !sl.keep_done &&
                   ((cfg_.inline_mode && sl.epi_stream == sl.stream) || on_producer || sl.on_producer);
    if (!sl.done_lazy) sl.done_mark = record_m(sl.done, sl.epi_stream);
    sl.pending = false;
  }

  // Redundant cross-stream waits. Each event record on the comm stream gets the next comm-stream mark; a wait of
  // stream st on such a record orders st after everything enqueued on the comm stream up to that mark. A later wait
  // of st on a comm-stream record with a mark at or below it is then implied (in-order streams) and skipped: each
  // such wait is a barrier packet costing ~25-30 us on the critical compute stream even when its event is long
  // complete (profiles/r5_forced_step_timeline.txt). The case it is for: the backward's last request runs on the
  // producer after a wait on the comm stream (begin on_producer), so the next forward's waits on the step's earlier
  // requests, and their epilogues committed on the producer after it, need no packets of their own. One stream is
  // tracked (the producer of the latest on-producer request).
  uint64_t record_m(Event e, Stream s) {
    dev_.record(e, s);
    return (!cfg_.inline_mode && s == cfg_.comm) ? ++comm_mark_ : 0;
  }
  void cover(Stream st, uint64_t m, bool take) {
    if (m == 0) return;
    if (cover_valid_ && st == cover_stream_) {
      if (m > cover_mark_) cover_mark_ = m;
    } else if (take || !cover_valid_) {
      cover_valid_ = true;
      cover_stream_ = st;
      cover_mark_ = m;
    }
  }
  void wait_m(Stream st, Event e, uint64_t m) {
    if (cfg_.elide_waits && m != 0 && cover_valid_ && st == cover_stream_ && m <= cover_mark_) {
      ++skipped_waits_;
      return;
    }
    dev_.wait(st, e);
    cover(st, m, false);
  }

  D& dev_;
  Config cfg_;
  std::array<Slot, kSlots> slots_;
  uint32_t seq_ = 0;
  int next_ = 0;
  uint64_t comm_mark_ = 0;
  bool cover_valid_ = false;
  Stream cover_stream_{};
  uint64_t cover_mark_ = 0;
  uint64_t skipped_waits_ = 0;
};

}  // namespace fan

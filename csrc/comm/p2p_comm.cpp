// Direct peer-to-peer transport. See p2p_comm.h.
#include "comm/p2p_comm.h"

#include "bfp/bfp_format.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <thread>

#include <unistd.h>

namespace fan {

namespace {

struct Handles {
  hipIpcMemHandle_t arena;
  hipIpcMemHandle_t flags;
  char host[64];  // where the arena lives: a peer on another (host, PCI bus) is a cross-device peer
  char bus[32];
};

void device_identity(int device, char* host, size_t host_len, char* bus, size_t bus_len) {
  std::memset(host, 0, host_len);
  std::memset(bus, 0, bus_len);
  gethostname(host, host_len - 1);
  if (hipDeviceGetPCIBusId(bus, (int)bus_len - 1, device) != hipSuccess) {
    (void)hipGetLastError();
    std::snprintf(bus, bus_len, "dev%d", device);
  }
}

}  // namespace

P2PComm::P2PComm(int rank, int world, int device, size_t slot_bytes, int depth)
    : rank_(rank), world_(world), device_(device), slot_((slot_bytes + 255) / 256 * 256), depth_(depth) {
  FAN_CHECK(depth >= 2 && depth <= 16, "p2p: 2 <= depth <= 16 arena slots per sender");
  FAN_CHECK(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
  // One IPC-exported allocation stays <= kMaxArenaBytes: on this image a peer's hipIpcOpenMemHandle of a 2 GiB
  // allocation never returned (4 processes, uncached and coarse alike; 1 GiB arenas open in 0.1-0.3 ms —
  // tools/probes/p2p_connect_probe.py), and 8 ranks x depth 4 x 128 MB slots would be 4 GiB. The slot shrinks
  // instead; the engine chunks its messages to payload_bytes() (engine.cpp layout), so only the chunk count grows.
  size_t cap = kMaxArenaBytes;
  if (const char* c = std::getenv("FAN_P2P_ARENA_MAX_MB")) cap = (size_t)std::atoll(c) << 20;
  const size_t max_slot = cap / ((size_t)world * depth) / 256 * 256;
  if (slot_ > max_slot) {
    if (std::getenv("FAN_P2P_DEBUG"))
      std::fprintf(stderr, "[p2p rank %d] slot %zu -> %zu B (arena cap %zu MB)\n", rank, slot_, max_slot, cap >> 20);
    slot_ = max_slot;
  }
  FAN_CHECK(slot_ > kTrailerBytes, "slot_bytes must exceed the 256-B verify trailer");
  if (const char* c = std::getenv("FAN_P2P_COPY")) sdma_ = !std::strcmp(c, "sdma");
  if (const char* c = std::getenv("FAN_P2P_FLAGS")) kflags_ = !std::strcmp(c, "kernel");
  FAN_HIP_CHECK(hipSetDevice(device));
  // Arena and flags UNCACHED (see the memory-ordering argument in p2p_comm.h): peers write them over xGMI, so no
  // line of them may sit in this GPU's (per-XCD, non-coherent) L2 when the reader consumes a new message.
  // Fallback to coarse-grained memory only if the allocator refuses the flag (the ordering then rests on the
  // kernel-boundary L2 invalidate of the reading kernel, which reads each arena byte once per message).
  // FAN_P2P_MEM=uncached (default) | fine | coarse: memory type of the arena (A/B; the flags stay uncached)
  const char* me = std::getenv("FAN_P2P_MEM");
  const std::string mem = me ? me : "uncached";
  unsigned aflag = mem == "fine" ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
  uncached_ = mem != "coarse" && mem != "fine" &&
              hipExtMallocWithFlags(reinterpret_cast<void**>(&arena_), (size_t)world * depth_ * slot_, aflag) == hipSuccess;
  if (!uncached_) {
    (void)hipGetLastError();
    if (mem == "fine") {
      FAN_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&arena_), (size_t)world * depth_ * slot_, aflag));
    } else {
      FAN_HIP_CHECK(hipMalloc(&arena_, (size_t)world * depth_ * slot_));
    }
  }
  arena_mem_ = uncached_ ? "uncached" : mem == "fine" ? "fine" : "coarse";
  if (std::getenv("FAN_P2P_DEBUG"))
    std::fprintf(stderr, "[p2p rank %d] arena %zu MB (%s) allocated\n", rank, ((size_t)world * depth_ * slot_) >> 20,
                 arena_mem_.c_str());
  // flags are polled by the command processor (hipStreamWaitValue64) and written by peers' command
  // processors (hipStreamWriteValue64); device memory supports both and HIP IPC export (probed on
  // MI355X: tools/probes/stream_wait_probe.cpp)
  void* f = nullptr;
  if (hipExtMallocWithFlags(&f, (size_t)2 * world * sizeof(uint64_t), hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    FAN_HIP_CHECK(hipMalloc(&f, (size_t)2 * world * sizeof(uint64_t)));
  }
  flags_ = reinterpret_cast<uint64_t*>(f);
  FAN_HIP_CHECK(hipMemset(flags_, 0, (size_t)2 * world * sizeof(uint64_t)));
  FAN_HIP_CHECK(hipDeviceSynchronize());
  peer_arena_.assign(world, nullptr);
  peer_flags_.assign(world, nullptr);
  opened_.assign(world, false);
  peer_arena_[rank] = arena_;
  peer_flags_[rank] = flags_;
  last_sent_.assign(depth_, std::vector<uint64_t>(world, 0));
  bytes_to_peer_.assign(world, 0);
  FAN_HIP_CHECK(hipEventCreateWithFlags(&rel_ev_, hipEventDisableTiming | hipEventReleaseToSystem));
}

bool p2p_release_event_needed(int mode, bool copy_engine_bytes) {
  // mode 3 (cp): the command processor's system-scope release orders every round's stores before its flags. In the
  // in-kernel modes (1 block, 2 thread) the peer-storing kernels release their own stores, but bytes moved by the copy
  // engines or by hipMemcpyAsync (SDMA arms, unaligned fallback) went through no such kernel: the event is still
  // needed for that round, else a cross-device peer could see the flag before those bytes.
  return mode == 3 || copy_engine_bytes;
}

RoundFlags p2p_round_flags(int rank, int world, uint64_t seq, const std::vector<int>& to, const std::vector<int>& from,
                           const std::vector<uint64_t>& last_sent_in_slot) {
  RoundFlags r;
  for (int p : to) {
    if (last_sent_in_slot[p]) r.credit_waits.push_back({rank, world + p, last_sent_in_slot[p]});
    r.ready_writes.push_back({p, rank, seq});
  }
  for (int q : from) {
    r.ready_waits.push_back({rank, q, seq});
    r.ack_writes.push_back({q, world + rank, seq});
  }
  return r;
}

void P2PComm::release_before_flags(hipStream_t s) {
  if (p2p_release_event_needed(p2p_release_mode(), nonkernel_pending_)) FAN_HIP_CHECK(hipEventRecord(rel_ev_, s));
  nonkernel_pending_ = false;
}

void P2PComm::write_flags(hipStream_t s, const std::vector<FlagOp>& w) {
  if (w.empty()) return;
  if (kflags_) {
    launch_flag_write(w, s);
    return;
  }
  for (const FlagOp& f : w) FAN_HIP_CHECK(hipStreamWriteValue64(s, f.first, f.second, 0));
}

void P2PComm::wait_flags(hipStream_t s, const std::vector<FlagOp>& w, bool credit) {
  if (w.empty()) return;
  (credit ? credit_waits_ : ready_waits_) += w.size();
  TimedWait* t = nullptr;
  if (timing_) {
    if (tw_used_ == tw_.size()) {
      TimedWait n{};
      FAN_HIP_CHECK(hipEventCreate(&n.ev[0]));
      FAN_HIP_CHECK(hipEventCreate(&n.ev[1]));
      tw_.push_back(n);
    }
    t = &tw_[tw_used_++];
    t->credit = credit;
    FAN_HIP_CHECK(hipEventRecord(t->ev[0], s));
  }
  if (kflags_) {
    if (kflag_err_ == nullptr) {
      FAN_HIP_CHECK(hipMalloc(&kflag_err_, sizeof(unsigned)));
      FAN_HIP_CHECK(hipMemset(kflag_err_, 0, sizeof(unsigned)));
    }
    launch_flag_wait(w, kflag_err_, s);
  } else {
    for (const FlagOp& f : w) FAN_HIP_CHECK(hipStreamWaitValue64(s, f.first, f.second, hipStreamWaitValueGte));
  }
  if (t) FAN_HIP_CHECK(hipEventRecord(t->ev[1], s));
}

unsigned P2PComm::kernel_flag_error() const {
  if (kflag_err_ == nullptr) return 0;
  unsigned v = 0;
  FAN_HIP_CHECK(hipMemcpy(&v, kflag_err_, sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

P2PComm::Stats P2PComm::stats(bool wait) {
  // fold the recorded waits into the totals, then recycle the events (in order: a wait still parked keeps itself
  // and every later one for the next call)
  size_t i = 0;
  for (; i < tw_used_; ++i) {
    if (!wait && hipEventQuery(tw_[i].ev[1]) != hipSuccess) break;
    float ms = 0.f;
    FAN_HIP_CHECK(hipEventSynchronize(tw_[i].ev[1]));
    FAN_HIP_CHECK(hipEventElapsedTime(&ms, tw_[i].ev[0], tw_[i].ev[1]));
    stall_ms_[tw_[i].credit ? 1 : 0] += ms;
    timed_++;
  }
  (void)hipGetLastError();  // a not-ready query is not an error
  if (i > 0 && i < tw_used_) std::rotate(tw_.begin(), tw_.begin() + i, tw_.begin() + tw_used_);
  tw_used_ -= i;
  Stats r;
  r.ready_waits = ready_waits_;
  r.credit_waits = credit_waits_;
  r.timed_waits = timed_;
  r.ready_stall_ms = stall_ms_[0];
  r.credit_stall_ms = stall_ms_[1];
  r.bytes_to_peer = bytes_to_peer_;
  return r;
}

void P2PComm::reset_stats() {
  stats();  // drain pending timed waits
  ready_waits_ = credit_waits_ = timed_ = 0;
  stall_ms_[0] = stall_ms_[1] = 0.0;
  bytes_to_peer_.assign(world_, 0);
}

std::vector<uint64_t> P2PComm::flags_snapshot(double timeout_s) const {
  const size_t n = (size_t)2 * world_;
  // pinned staging + a non-blocking stream of its own: nothing here waits on the (possibly parked) engine streams;
  // on timeout the staging buffer and stream are leaked on purpose (the copy may still land in them later)
  void* h = nullptr;
  hipStream_t s = nullptr;
  if (hipHostMalloc(&h, n * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    return {};
  }
  std::vector<uint64_t> v;
  if (hipMemcpyAsync(h, flags_, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s) == hipSuccess) {
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q;
    while ((q = hipStreamQuery(s)) == hipErrorNotReady &&
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < timeout_s)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (q == hipSuccess) {
      v.assign(static_cast<const uint64_t*>(h), static_cast<const uint64_t*>(h) + n);
      hipStreamDestroy(s);
      hipHostFree(h);
    }
  }
  (void)hipGetLastError();
  return v;
}

void P2PComm::abort() {
  if (aborted_) return;
  aborted_ = true;
  // Release every GPU waiter parked on this rank's flag block (a ready-wait for a dead sender, an ack-wait for a
  // dead receiver): overwrite all ready / ack words with a poison value above any sequence number, from a stream of
  // its own (the parked stream cannot run it). The released streams then copy stale arena bytes; the aborted_
  // state makes every later call and the engine's synchronize() raise, so nothing trusts them.
  // The poison write is polled for a bounded time rather than synchronized: if the new stream shares a hardware
  // queue with a parked one, it waits behind it, and abort() must still return (the caller is usually a watchdog
  // about to end the process).
  hipSetDevice(device_);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) {
    hipMemsetAsync(flags_, 0x7F, (size_t)2 * world_ * sizeof(uint64_t), s);
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q;
    while ((q = hipStreamQuery(s)) == hipErrorNotReady &&
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 5.0)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (q == hipSuccess) hipStreamDestroy(s);
  }
  (void)hipGetLastError();
}

P2PComm::~P2PComm() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (int p = 0; p < world_; ++p) {
    if (!opened_[p]) continue;
    hipIpcCloseMemHandle(peer_arena_[p]);
    hipIpcCloseMemHandle(peer_flags_[p]);
  }
  for (auto& t : tw_) {
    hipEventDestroy(t.ev[0]);
    hipEventDestroy(t.ev[1]);
  }
  if (rel_ev_) hipEventDestroy(rel_ev_);
  if (kflag_err_) hipFree(kflag_err_);
  hipFree(flags_);
  hipFree(arena_);
}

std::string P2PComm::handles() const {
  Handles h;
  FAN_HIP_CHECK(hipIpcGetMemHandle(&h.arena, arena_));
  FAN_HIP_CHECK(hipIpcGetMemHandle(&h.flags, flags_));
  if (std::getenv("FAN_P2P_DEBUG")) std::fprintf(stderr, "[p2p rank %d] IPC handles exported\n", rank_);
  device_identity(device_, h.host, sizeof(h.host), h.bus, sizeof(h.bus));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void P2PComm::connect(const std::vector<std::string>& all) {
  FAN_CHECK((int)all.size() == world_, "connect: need one handle blob per rank");
  FAN_HIP_CHECK(hipSetDevice(device_));
  char host[64], bus[32];
  device_identity(device_, host, sizeof(host), bus, sizeof(bus));
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    FAN_CHECK(all[p].size() == sizeof(Handles), "connect: bad handle blob");
    Handles h;
    std::memcpy(&h, all[p].data(), sizeof(h));
    if (std::strncmp(h.host, host, sizeof(host)) || std::strncmp(h.bus, bus, sizeof(bus))) cross_device_ = true;
    void* a = nullptr;
    void* f = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    FAN_HIP_CHECK(hipIpcOpenMemHandle(&a, h.arena, hipIpcMemLazyEnablePeerAccess));
    FAN_HIP_CHECK(hipIpcOpenMemHandle(&f, h.flags, hipIpcMemLazyEnablePeerAccess));
    if (std::getenv("FAN_P2P_DEBUG"))
      std::fprintf(stderr, "[p2p rank %d] opened peer %d's arena + flags (%s %s) in %.1f ms\n", rank_, p, h.host,
                   h.bus, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    peer_arena_[p] = reinterpret_cast<uint8_t*>(a);
    peer_flags_[p] = reinterpret_cast<uint64_t*>(f);
    opened_[p] = true;
  }
  // the command-processor release is unverified across devices (p2p_comm.h): peers on other GPUs get the in-kernel
  // system-scope release unless the user chose a mode
  if (cross_device_ && !std::getenv("FAN_P2P_RELEASE") && p2p_release_mode() == 3) set_p2p_release_mode(1);
}

void P2PComm::move(const std::vector<P2PCopy>& segs, hipStream_t s) {
  if (!sdma_) {
    launch_multi_copy(segs, s);
    return;
  }
  // copy engines: one command per contiguous run (segments whose source AND destination continue the previous one
  // are merged), so a round costs one command per peer rather than one per segment
  for (const P2PCopy& run : coalesce_copies(segs)) {
    FAN_HIP_CHECK(hipMemcpyAsync(run.dst, run.src, run.bytes, hipMemcpyDeviceToDeviceNoCU, s));
    nonkernel_pending_ = true;
  }
}

std::vector<P2PCopy> coalesce_copies(const std::vector<P2PCopy>& segs) {
  std::vector<P2PCopy> out;
  for (const P2PCopy& c : segs) {
    if (!c.bytes) continue;
    if (!out.empty()) {
      P2PCopy& b = out.back();
      if (static_cast<const uint8_t*>(b.src) + b.bytes == c.src && static_cast<uint8_t*>(b.dst) + b.bytes == c.dst) {
        b.bytes += c.bytes;
        continue;
      }
    }
    out.push_back(c);
  }
  return out;
}

void P2PComm::connect_local(const std::vector<P2PComm*>& ranks) {
  for (P2PComm* c : ranks) {
    FAN_CHECK((int)ranks.size() == c->world_, "connect_local: need every rank");
    for (P2PComm* d : ranks) {
      c->peer_arena_[d->rank_] = d->arena_;
      c->peer_flags_[d->rank_] = d->flags_;
    }
  }
}

void P2PComm::sendrecv(const std::vector<P2POp>& sends, const std::vector<P2POp>& recvs, hipStream_t s) {
  FAN_CHECK(!aborted_, "p2p transport aborted");
  const uint64_t q = ++seq_;
  const int par = (int)(q % depth_);
  // sends: per destination, in issue order, packed back to back into this rank's slot of the peer's arena.
  // WAR first (the receiver drained what we last put into this parity slot), then ONE copy launch for all
  // destinations (every link busy at once), then one ready flag per destination.
  std::vector<P2PCopy> out;
  std::vector<int> dests;
  for (int p = 0; p < world_; ++p) {
    size_t off = 0;
    bool any = false;
    for (const P2POp& op : sends) {
      if (op.peer != p || op.bytes == 0) continue;
      FAN_CHECK(p != rank_, "p2p: self-send");
      FAN_CHECK(peer_arena_[p] != nullptr, "p2p: peer not connected");
      if (!any) {
        any = true;
        dests.push_back(p);
      }
      FAN_CHECK(off + op.bytes <= payload_bytes(), "p2p: message larger than the arena slot (raise slot_bytes)");
      out.push_back({op.ptr, slot_ptr(peer_arena_[p], rank_, q) + off, op.bytes});
      bytes_to_peer_[p] += (int64_t)op.bytes;
      off += (op.bytes + 15) / 16 * 16;
    }
  }
  const RoundFlags sf = p2p_round_flags(rank_, world_, q, dests, {}, last_sent_[par]);
  wait_flags(s, flag_ptrs(sf.credit_waits), true);
  copy(out, s);
  release_before_flags(s);
  write_flags(s, flag_ptrs(sf.ready_writes));  // "ready from rank_" at each destination
  for (int p : dests) last_sent_[par][p] = q;
  // receives: wait for every source's ready flag, one copy-out launch, then acknowledge (frees the slots)
  std::vector<P2PCopy> in;
  std::vector<int> srcs;
  for (int src = 0; src < world_; ++src) {
    size_t off = 0;
    bool any = false;
    for (const P2POp& op : recvs) {
      if (op.peer != src || op.bytes == 0) continue;
      FAN_CHECK(src != rank_, "p2p: self-receive");
      if (!any) {
        any = true;
        srcs.push_back(src);
      }
      FAN_CHECK(off + op.bytes <= payload_bytes(), "p2p: message larger than the arena slot (raise slot_bytes)");
      in.push_back({slot_ptr(arena_, src, q) + off, op.ptr, op.bytes});
      off += (op.bytes + 15) / 16 * 16;
    }
  }
  const RoundFlags rf = p2p_round_flags(rank_, world_, q, {}, srcs, last_sent_[par]);
  wait_flags(s, flag_ptrs(rf.ready_waits), false);
  copy(in, s);
  write_flags(s, flag_ptrs(rf.ack_writes));
}

std::vector<int> P2PComm::others() const {
  std::vector<int> v;
  for (int p = 0; p < world_; ++p)
    if (p != rank_) v.push_back(p);
  return v;
}

std::vector<P2PComm::FlagOp> P2PComm::flag_ptrs(const std::vector<FlagRef>& refs) const {
  std::vector<FlagOp> out;
  for (const FlagRef& f : refs) out.push_back({(f.peer == rank_ ? flags_ : peer_flags_[f.peer]) + f.word, f.value});
  return out;
}

P2PComm::Round P2PComm::begin(hipStream_t s) { return begin_to(others(), s); }
void P2PComm::publish(const Round& r, hipStream_t s) { publish_to(r, others(), s); }
void P2PComm::wait(const Round& r, hipStream_t s) { wait_from(r, others(), s); }
void P2PComm::release(const Round& r, hipStream_t s) { release_from(r, others(), s); }

P2PComm::Round P2PComm::begin_to(const std::vector<int>& to, hipStream_t s) {
  FAN_CHECK(!aborted_, "p2p transport aborted");
  Round r{++seq_};
  for (int p : to)
    FAN_CHECK(p != rank_ && p >= 0 && p < world_ && peer_arena_[p] != nullptr, "p2p: bad or unconnected peer");
  // credit flow control: every peer acknowledged the previous message in the slot this round reuses
  wait_flags(s, flag_ptrs(p2p_round_flags(rank_, world_, r.seq, to, {}, last_sent_[r.seq % depth_]).credit_waits), true);
  return r;
}

void P2PComm::publish_to(const Round& r, const std::vector<int>& to, hipStream_t s) {
  const int par = (int)(r.seq % depth_);
  release_before_flags(s);
  write_flags(s, flag_ptrs(p2p_round_flags(rank_, world_, r.seq, to, {}, last_sent_[par]).ready_writes));
  for (int p : to) last_sent_[par][p] = r.seq;
}

void P2PComm::wait_from(const Round& r, const std::vector<int>& from, hipStream_t s) {
  wait_flags(s, flag_ptrs(p2p_round_flags(rank_, world_, r.seq, {}, from, last_sent_[r.seq % depth_]).ready_waits),
             false);
}

void P2PComm::release_from(const Round& r, const std::vector<int>& from, hipStream_t s) {
  write_flags(s, flag_ptrs(p2p_round_flags(rank_, world_, r.seq, {}, from, last_sent_[r.seq % depth_]).ack_writes));
}

void P2PComm::copy(const std::vector<P2PCopy>& segs, hipStream_t s) {
  bool aligned = true;
  for (const P2PCopy& c : segs)
    aligned = aligned && c.bytes % 16 == 0 && ((uintptr_t)c.src & 15) == 0 && ((uintptr_t)c.dst & 15) == 0;
  if (aligned) {
    launch_multi_copy(segs, s);
    return;
  }
  for (const P2PCopy& c : coalesce_copies(segs)) {
    FAN_HIP_CHECK(hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToDevice, s));
    nonkernel_pending_ = true;
  }
}

void P2PComm::all_to_all(const void* send, void* recv, size_t bpp, hipStream_t s) {
  std::vector<P2POp> sends, recvs;
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    sends.push_back({const_cast<uint8_t*>(static_cast<const uint8_t*>(send)) + p * bpp, bpp, p});
    recvs.push_back({static_cast<uint8_t*>(recv) + p * bpp, bpp, p});
  }
  if (bpp)
    FAN_HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(recv) + rank_ * bpp,
                                 static_cast<const uint8_t*>(send) + rank_ * bpp, bpp, hipMemcpyDeviceToDevice, s));
  sendrecv(sends, recvs, s);
}

void P2PComm::all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) {
  std::vector<P2POp> sends, recvs;
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    sends.push_back({const_cast<void*>(send), bytes, p});
    recvs.push_back({static_cast<uint8_t*>(recv) + p * bytes, bytes, p});
  }
  if (bytes)
    FAN_HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(recv) + rank_ * bytes, send, bytes, hipMemcpyDeviceToDevice, s));
  sendrecv(sends, recvs, s);
}

}  // namespace fan

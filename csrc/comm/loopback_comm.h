// Loopback communicator: N virtual ranks on ONE GPU, one host thread per rank.
//
// The stand-in for the reference's 3-NIC RTL testbench (readme.pdf §3.2-3.3: several DUT instances wired in
// a simulated ring): every collective is a host barrier + device-to-device copies between the ranks' buffers,
// so the C++ engine's multi-rank mesh / ring schedules run unchanged and can be checked bit-exactly on a
// single MI355X. Test infrastructure only (host-synchronous, not a fast path).
//
// Fault injection (test-only): drop_after(k) makes this rank stop delivering after k collectives, so peers
// exercise the engine's bounded waits / timeout diagnostics.
#pragma once
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

#include "comm/native_comm.h"

namespace fan {

class LoopbackFabric {
 public:
  explicit LoopbackFabric(int world, double timeout_s = 60.0);
  int world() const { return world_; }
  // Generation barrier with a timeout (throws instead of hanging a test).
  void barrier(int rank);
  std::vector<const void*> post;                // per rank: the buffer published for this collective
  std::vector<std::vector<P2POp>> sends;        // per rank: sends published for this round
  std::vector<char> lost;                       // per rank: this round's sends are lost in flight (fault injection)
  bool aborted = false;

 private:
  int world_;
  double timeout_s_;
  std::mutex m_;
  std::condition_variable cv_;
  int count_ = 0;
  uint64_t gen_ = 0;
};

class LoopbackComm : public Comm {
 public:
  LoopbackComm(std::shared_ptr<LoopbackFabric> f, int rank) : f_(std::move(f)), rank_(rank) {}
  int rank() const override { return rank_; }
  int world() const override { return f_->world(); }
  void sendrecv(const std::vector<P2POp>& sends, const std::vector<P2POp>& recvs, hipStream_t s) override;
  void all_to_all(const void* send, void* recv, size_t bytes_per_peer, hipStream_t s) override;
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override;
  std::string async_error() override { return f_->aborted ? "loopback fabric aborted" : ""; }
  void abort() override { f_->aborted = true; }
  const char* kind() const override { return "loopback"; }
  void drop_after(int64_t k) { drop_after_ = k; }
  // fault injection: the messages of this rank's k-th sendrecv round (0-based, counted over sendrecv calls) are lost
  // in flight — the receivers' buffers keep their stale contents, the schedule goes on (a silent loss, what
  // verify mode must catch)
  void lose_round(int64_t k) { lose_round_ = k; }
  int64_t collectives() const { return ops_; }

 private:
  bool dropped();
  std::shared_ptr<LoopbackFabric> f_;
  int rank_;
  int64_t ops_ = 0, drop_after_ = -1, lose_round_ = -1, rounds_ = 0;
};

}  // namespace fan

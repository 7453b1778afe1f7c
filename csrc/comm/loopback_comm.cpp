// Loopback communicator (virtual ranks on one GPU). See loopback_comm.h.
#include "comm/loopback_comm.h"

#include <chrono>
#include <string>

namespace fan {

LoopbackFabric::LoopbackFabric(int world, double timeout_s)
    : post(world, nullptr), sends(world), lost(world, 0), world_(world), timeout_s_(timeout_s) {
  FAN_CHECK(world >= 1, "loopback world must be >= 1");
}

void LoopbackFabric::barrier(int rank) {
  std::unique_lock<std::mutex> lk(m_);
  if (aborted) throw std::runtime_error("loopback fabric aborted (rank " + std::to_string(rank) + ")");
  const uint64_t g = gen_;
  if (++count_ == world_) {
    count_ = 0;
    ++gen_;
    cv_.notify_all();
    return;
  }
  const bool ok = cv_.wait_for(lk, std::chrono::duration<double>(timeout_s_), [&] { return gen_ != g || aborted; });
  if (!ok || gen_ == g) {
    aborted = true;
    cv_.notify_all();
    throw std::runtime_error("loopback collective timed out / aborted at rank " + std::to_string(rank) + " (" +
                             std::to_string(count_) + " of " + std::to_string(world_) + " ranks arrived)");
  }
}

bool LoopbackComm::dropped() {
  ++ops_;
  return drop_after_ >= 0 && ops_ > drop_after_;
}

void LoopbackComm::all_to_all(const void* send, void* recv, size_t bpp, hipStream_t s) {
  if (dropped()) throw std::runtime_error("fault injection: rank " + std::to_string(rank_) + " dropped all_to_all");
  const int N = world();
  FAN_HIP_CHECK(hipStreamSynchronize(s));
  f_->post[rank_] = send;
  f_->barrier(rank_);
  for (int p = 0; p < N; ++p)
    FAN_HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(recv) + p * bpp,
                                 static_cast<const uint8_t*>(f_->post[p]) + rank_ * bpp, bpp,
                                 hipMemcpyDeviceToDevice, s));
  FAN_HIP_CHECK(hipStreamSynchronize(s));
  f_->barrier(rank_);  // peers finished reading this rank's send buffer
}

void LoopbackComm::all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) {
  if (dropped()) throw std::runtime_error("fault injection: rank " + std::to_string(rank_) + " dropped all_gather");
  const int N = world();
  FAN_HIP_CHECK(hipStreamSynchronize(s));
  f_->post[rank_] = send;
  f_->barrier(rank_);
  for (int p = 0; p < N; ++p)
    FAN_HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(recv) + p * bytes, f_->post[p], bytes,
                                 hipMemcpyDeviceToDevice, s));
  FAN_HIP_CHECK(hipStreamSynchronize(s));
  f_->barrier(rank_);
}

void LoopbackComm::sendrecv(const std::vector<P2POp>& sends, const std::vector<P2POp>& recvs, hipStream_t s) {
  if (dropped()) throw std::runtime_error("fault injection: rank " + std::to_string(rank_) + " dropped sendrecv");
  const int N = world();
  FAN_HIP_CHECK(hipStreamSynchronize(s));
  f_->sends[rank_] = sends;
  f_->lost[rank_] = rounds_++ == lose_round_;
  f_->barrier(rank_);
  std::vector<int> taken(N, 0);
  for (const P2POp& r : recvs) {
    // the k-th receive from `peer` matches the k-th send of `peer` addressed to this rank (RCCL group order)
    const auto& ps = f_->sends.at(r.peer);
    int k = taken[r.peer]++;
    const P2POp* match = nullptr;
    for (const P2POp& o : ps)
      if (o.peer == rank_ && k-- == 0) {
        match = &o;
        break;
      }
    FAN_CHECK(match != nullptr, "loopback sendrecv: no matching send from peer");
    FAN_CHECK(match->bytes == r.bytes, "loopback sendrecv: size mismatch between send and recv");
    if (!f_->lost[r.peer]) FAN_HIP_CHECK(hipMemcpyAsync(r.ptr, match->ptr, r.bytes, hipMemcpyDeviceToDevice, s));
  }
  FAN_HIP_CHECK(hipStreamSynchronize(s));
  f_->barrier(rank_);
}

}  // namespace fan

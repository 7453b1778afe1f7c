// Native RCCL communicator (own ncclComm_t, independent of torch's ProcessGroup).
//
// The MI355X-native stand-in for the reference's NIC link layer + CSR driver (sw/mlp_mpi_example_f32.cpp:35-180,
// hw/all_reduce.sv ETH ports): point-to-point xGMI transfers between ring neighbours (ncclSend/ncclRecv in one
// group per round) and the direct full-mesh collectives that a fully connected 8-GPU xGMI node favours.
// Bootstrap: the 128-byte ncclUniqueId is exchanged through torch.distributed's store (no MPI).
#pragma once
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

#include "common/hip_common.h"

namespace fan {

#define FAN_NCCL_CHECK(expr)                                                                              \
  do {                                                                                                    \
    ncclResult_t _r = (expr);                                                                             \
    if (_r != ncclSuccess)                                                                                \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + __FILE__ + \
                               ":" + std::to_string(__LINE__) + ": " #expr);                              \
  } while (0)

struct P2POp {
  void* ptr;
  size_t bytes;
  int peer;
};

// What the all-reduce engine needs from a communicator. Implemented by NativeComm (RCCL over xGMI) and by
// LoopbackComm (virtual ranks on one GPU, csrc/comm/loopback_comm.h) so the engine's multi-rank schedules are
// testable on a single device.
class P2PComm;

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // One group with every send and recv of a round (ring round / multi-ring round). Several sends to the same
  // peer in one group are matched to that peer's receives in issue order.
  virtual void sendrecv(const std::vector<P2POp>& sends, const std::vector<P2POp>& recvs, hipStream_t s) = 0;
  virtual void all_to_all(const void* send, void* recv, size_t bytes_per_peer, hipStream_t s) = 0;
  virtual void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // Returns an empty string when healthy, else the async error text.
  virtual std::string async_error() = 0;
  virtual void abort() = 0;
  // Transports whose receive buffers the engine's kernels may write and read in place (direct peer stores):
  virtual P2PComm* direct() { return nullptr; }
  // Run-time echo of what this communicator actually reaches (the reference reads node_info back after
  // programming it, sw/mlp_mpi_example_f32.cpp:65-98): RCCL's own rank count (ncclCommCount), the P2P transport's
  // this rank + peers whose receive arenas are mapped, the loopback fabric's virtual ranks.
  virtual int ranks_seen() { return world(); }
  virtual const char* kind() const = 0;
};

class NativeComm : public Comm {
 public:
  NativeComm(const std::string& uid_bytes, int rank, int world, int device);
  ~NativeComm() override;
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void sendrecv(const std::vector<P2POp>& sends, const std::vector<P2POp>& recvs, hipStream_t s) override;
  void all_to_all(const void* send, void* recv, size_t bytes_per_peer, hipStream_t s) override;
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override;
  void all_reduce(void* buf, size_t count, int dtype /*0 f32, 1 bf16*/, hipStream_t s);
  void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, hipStream_t s);
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s);
  std::string async_error() override;
  void abort() override;
  int ranks_seen() override;
  const char* kind() const override { return "rccl"; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, world_ = 1;
  bool aborted_ = false;
};

std::string nccl_unique_id_bytes();
int nccl_version();

}  // namespace fan

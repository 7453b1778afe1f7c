// Native RCCL communicator. See native_comm.h.
#include "comm/native_comm.h"

#include <cstring>

namespace fan {

std::string nccl_unique_id_bytes() {
  ncclUniqueId id;
  FAN_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int nccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

NativeComm::NativeComm(const std::string& uid_bytes, int rank, int world, int device) : rank_(rank), world_(world) {
  FAN_CHECK(uid_bytes.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size");
  ncclUniqueId id;
  std::memcpy(&id, uid_bytes.data(), sizeof(id));
  FAN_HIP_CHECK(hipSetDevice(device));
  FAN_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
}

NativeComm::~NativeComm() {
  if (comm_ && !aborted_) ncclCommDestroy(comm_);
}

void NativeComm::sendrecv(const std::vector<P2POp>& sends, const std::vector<P2POp>& recvs, hipStream_t s) {
  FAN_NCCL_CHECK(ncclGroupStart());
  for (const auto& o : sends)
    if (o.bytes) FAN_NCCL_CHECK(ncclSend(o.ptr, o.bytes, ncclUint8, o.peer, comm_, s));
  for (const auto& o : recvs)
    if (o.bytes) FAN_NCCL_CHECK(ncclRecv(o.ptr, o.bytes, ncclUint8, o.peer, comm_, s));
  FAN_NCCL_CHECK(ncclGroupEnd());
}

void NativeComm::all_to_all(const void* send, void* recv, size_t bytes_per_peer, hipStream_t s) {
  FAN_NCCL_CHECK(ncclAllToAll(send, recv, bytes_per_peer, ncclUint8, comm_, s));
}

void NativeComm::all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) {
  FAN_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
}

static ncclDataType_t nd(int dtype) { return dtype == 0 ? ncclFloat32 : ncclBfloat16; }

void NativeComm::all_reduce(void* buf, size_t count, int dtype, hipStream_t s) {
  FAN_NCCL_CHECK(ncclAllReduce(buf, buf, count, nd(dtype), ncclSum, comm_, s));
}

void NativeComm::reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, hipStream_t s) {
  FAN_NCCL_CHECK(ncclReduceScatter(send, recv, recv_count, nd(dtype), ncclSum, comm_, s));
}

void NativeComm::broadcast(void* buf, size_t bytes, int root, hipStream_t s) {
  FAN_NCCL_CHECK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, s));
}

std::string NativeComm::async_error() {
  if (!comm_ || aborted_) return aborted_ ? "aborted" : "";
  ncclResult_t r = ncclSuccess;
  ncclCommGetAsyncError(comm_, &r);
  if (r == ncclSuccess || r == ncclInProgress) return "";
  return ncclGetErrorString(r);
}

int NativeComm::ranks_seen() {
  int n = -1;
  if (comm_ && !aborted_ && ncclCommCount(comm_, &n) != ncclSuccess) n = -1;
  return n;
}

void NativeComm::abort() {
  if (comm_ && !aborted_) {
    ncclCommAbort(comm_);
    aborted_ = true;
  }
}

}  // namespace fan

// Bindings for the native communicator (RCCL over xGMI).
#include "bindings_common.h"
#include "comm/native_comm.h"

namespace fan {

namespace {

void* ptr_of(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "comm buffers must be contiguous GPU tensors");
  return t.data_ptr();
}
size_t bytes_of(const at::Tensor& t) { return (size_t)t.numel() * t.element_size(); }

}  // namespace

void register_engine(pybind11::module_& m) {
  m.def("nccl_unique_id", []() { return pybind11::bytes(nccl_unique_id_bytes()); });
  m.def("nccl_version", &nccl_version);
  pybind11::class_<NativeComm>(m, "NativeComm")
      .def(pybind11::init([](pybind11::bytes uid, int rank, int world, int device) {
             return new NativeComm(std::string(uid), rank, world, device);
           }),
           pybind11::arg("uid"), pybind11::arg("rank"), pybind11::arg("world"), pybind11::arg("device"))
      .def_property_readonly("rank", &NativeComm::rank)
      .def_property_readonly("world", &NativeComm::world)
      .def("sendrecv",
           [](NativeComm& c, const std::vector<std::pair<at::Tensor, int>>& sends,
              const std::vector<std::pair<at::Tensor, int>>& recvs) {
             std::vector<P2POp> s, r;
             for (auto& p : sends) s.push_back({ptr_of(p.first), bytes_of(p.first), p.second});
             for (auto& p : recvs) r.push_back({ptr_of(p.first), bytes_of(p.first), p.second});
             c.sendrecv(s, r, fan_stream());
           })
      .def("all_to_all",
           [](NativeComm& c, const at::Tensor& send, at::Tensor& recv) {
             TORCH_CHECK(bytes_of(send) == bytes_of(recv) && bytes_of(send) % c.world() == 0, "all_to_all sizes");
             c.all_to_all(ptr_of(send), ptr_of(recv), bytes_of(send) / c.world(), fan_stream());
           })
      .def("all_gather",
           [](NativeComm& c, const at::Tensor& send, at::Tensor& recv) {
             TORCH_CHECK(bytes_of(recv) == bytes_of(send) * c.world(), "all_gather sizes");
             c.all_gather(ptr_of(send), ptr_of(recv), bytes_of(send), fan_stream());
           })
      .def("all_reduce",
           [](NativeComm& c, at::Tensor& buf) {
             TORCH_CHECK(buf.scalar_type() == at::kFloat || buf.scalar_type() == at::kBFloat16, "all_reduce dtype");
             c.all_reduce(ptr_of(buf), buf.numel(), buf.scalar_type() == at::kFloat ? 0 : 1, fan_stream());
           })
      .def("reduce_scatter",
           [](NativeComm& c, const at::Tensor& send, at::Tensor& recv) {
             TORCH_CHECK(send.numel() == recv.numel() * c.world(), "reduce_scatter sizes");
             c.reduce_scatter(ptr_of(send), ptr_of(recv), recv.numel(), recv.scalar_type() == at::kFloat ? 0 : 1,
                              fan_stream());
           })
      .def("broadcast", [](NativeComm& c, at::Tensor& buf, int root) { c.broadcast(ptr_of(buf), bytes_of(buf), root, fan_stream()); })
      .def("async_error", &NativeComm::async_error)
      .def("abort", &NativeComm::abort);
}

}  // namespace fan

// Python bindings of the fpga_ai_nic_amd native runtime (module fpga_ai_nic_amd._C).
//
// Only this translation unit includes torch headers; kernels live in their own .hip files and
// take raw pointers + a hipStream_t (the caller's current torch HIP stream).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#include "bfp/bfp_format.h"
#include "bindings_common.h"

namespace fan {
void register_gemm(pybind11::module_& m);
void register_nn(pybind11::module_& m);
void register_planner(pybind11::module_& m);
void register_engine(pybind11::module_& m);
}  // namespace fan

namespace {

using fan::DType;

int dtype_code(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return fan::kF32;
  if (t.scalar_type() == at::kBFloat16) return fan::kBF16;
  TORCH_CHECK(false, "expected float32 or bfloat16 tensor, got ", t.scalar_type());
}

void wire_pack(const at::Tensor& x, at::Tensor& out, int64_t shard_elems, int64_t codec) {
  FAN_T_CUDA_CONTIG(x);
  FAN_T_CUDA_CONTIG(out);
  TORCH_CHECK(out.scalar_type() == at::kByte, "packed buffer must be uint8");
  TORCH_CHECK(x.numel() % shard_elems == 0, "numel must be a multiple of shard_elems");
  const int n_shards = (int)(x.numel() / shard_elems);
  TORCH_CHECK((size_t)out.numel() >= fan::wire_shard_bytes((int)codec, shard_elems) * n_shards, "packed buffer too small");
  fan::launch_wire_pack((int)codec, dtype_code(x), x.data_ptr(), out.data_ptr(), (size_t)shard_elems, n_shards,
                        fan_stream());
}

// shard s of x encoded straight into dsts[s] (each a uint8 view, e.g. a peer's receive-arena slot); ends with a
// system-scope release (the direct P2P transport's producer kernel)
void wire_pack_to(const at::Tensor& x, const std::vector<at::Tensor>& dsts, int64_t shard_elems, int64_t codec) {
  FAN_T_CUDA_CONTIG(x);
  TORCH_CHECK(x.numel() == shard_elems * (int64_t)dsts.size(), "one destination per shard");
  TORCH_CHECK(dsts.size() <= (size_t)fan::kMaxPeers, "at most 16 destinations");
  fan::WirePtrs to{};
  for (size_t i = 0; i < dsts.size(); ++i) {
    TORCH_CHECK(dsts[i].is_cuda() && dsts[i].scalar_type() == at::kByte &&
                    (size_t)dsts[i].numel() >= fan::wire_shard_bytes((int)codec, shard_elems) &&
                    ((uintptr_t)dsts[i].data_ptr() & 15) == 0,
                "destination ", i, ": 16-B aligned uint8 buffer of one wire shard");
    to.p[i] = dsts[i].data_ptr<uint8_t>();
  }
  fan::launch_wire_pack_to((int)codec, dtype_code(x), x.data_ptr(), to, (size_t)shard_elems, (int)dsts.size(),
                           fan_stream());
}

void wire_pack_range(const at::Tensor& x, at::Tensor& out, int64_t shard_elems, int64_t begin, int64_t end,
                     int64_t codec) {
  FAN_T_CUDA_CONTIG(x);
  FAN_T_CUDA_CONTIG(out);
  TORCH_CHECK(out.scalar_type() == at::kByte, "packed buffer must be uint8");
  TORCH_CHECK(shard_elems > 0 && shard_elems % 256 == 0, "shard_elems must be a positive multiple of 256");
  TORCH_CHECK(0 <= begin && begin <= end && end <= x.numel() && begin % 16 == 0 && end % 16 == 0, "bad range");
  if (end == begin) return;
  const int64_t shards = (end - 1) / shard_elems + 1;
  TORCH_CHECK((int64_t)out.numel() >= (int64_t)fan::wire_shard_bytes((int)codec, shard_elems) * shards,
              "packed buffer too small");
  fan::launch_wire_pack_range((int)codec, dtype_code(x), x.data_ptr(), out.data_ptr(), (size_t)shard_elems,
                              (size_t)begin, (size_t)end, fan_stream());
}

void wire_unpack(const at::Tensor& packed, at::Tensor& out, int64_t shard_elems, int64_t codec) {
  FAN_T_CUDA_CONTIG(packed);
  FAN_T_CUDA_CONTIG(out);
  TORCH_CHECK(out.numel() % shard_elems == 0, "numel must be a multiple of shard_elems");
  const int n_shards = (int)(out.numel() / shard_elems);
  TORCH_CHECK((size_t)packed.numel() >= fan::wire_shard_bytes((int)codec, shard_elems) * n_shards, "packed buffer too small");
  fan::launch_wire_unpack((int)codec, dtype_code(out), packed.data_ptr(), out.data_ptr(), (size_t)shard_elems,
                          n_shards, fan_stream());
}

void wire_reduce(const at::Tensor& slots, int64_t n_slots, int64_t self_pos, const c10::optional<at::Tensor>& local,
                 const c10::optional<at::Tensor>& out_wire, const c10::optional<at::Tensor>& out_f32,
                 int64_t shard_elems, int64_t codec) {
  FAN_T_CUDA_CONTIG(slots);
  const size_t sb = fan::wire_shard_bytes((int)codec, shard_elems);
  // only slots other than self_pos are read (self_pos is replaced by the dense local operand)
  const int64_t last_read = (local && self_pos == n_slots - 1) ? n_slots - 2 : n_slots - 1;
  TORCH_CHECK((size_t)slots.numel() * slots.element_size() >= sb * (size_t)(last_read + 1), "slots buffer too small");
  const void* lp = nullptr;
  int ld = fan::kF32;
  if (local) {
    FAN_T_CUDA_CONTIG((*local));
    TORCH_CHECK(local->numel() >= shard_elems, "local operand too small");
    lp = local->data_ptr();
    ld = dtype_code(*local);
  }
  void* ow = nullptr;
  float* of = nullptr;
  if (out_wire) {
    FAN_T_CUDA_CONTIG((*out_wire));
    TORCH_CHECK((size_t)out_wire->numel() * out_wire->element_size() >= sb, "out_wire too small");
    ow = out_wire->data_ptr();
  }
  if (out_f32) {
    FAN_T_CUDA_CONTIG((*out_f32));
    TORCH_CHECK(out_f32->scalar_type() == at::kFloat && out_f32->numel() >= shard_elems, "bad out_f32");
    of = out_f32->data_ptr<float>();
  }
  fan::launch_wire_reduce((int)codec, ld, slots.data_ptr(), sb, (int)n_slots, (int)self_pos, lp, ow, of,
                          (size_t)shard_elems, fan_stream());
}

void wire_sgd(const at::Tensor& wire, int64_t shard_elems, int64_t n_shards, int64_t skip_shard, int64_t skip_period,
              at::Tensor& master,
              const c10::optional<at::Tensor>& lp, const c10::optional<at::Tensor>& mom, double lr, double grad_scale,
              double weight_decay, double momentum, bool nesterov, int64_t n_valid, int64_t codec) {
  FAN_T_CUDA_CONTIG(wire);
  FAN_T_CUDA_CONTIG(master);
  TORCH_CHECK(master.scalar_type() == at::kFloat, "master weights must be float32");
  TORCH_CHECK(master.numel() >= n_valid, "master too small");
  TORCH_CHECK((size_t)wire.numel() * wire.element_size() >= fan::wire_shard_bytes((int)codec, shard_elems) * n_shards,
              "wire buffer too small");
  fan::bf16_t* lpp = nullptr;
  float* mp = nullptr;
  if (lp) {
    FAN_T_CUDA_CONTIG((*lp));
    TORCH_CHECK(lp->scalar_type() == at::kBFloat16 && lp->numel() >= n_valid, "bad lp weights");
    lpp = reinterpret_cast<fan::bf16_t*>(lp->data_ptr());
  }
  if (mom) {
    FAN_T_CUDA_CONTIG((*mom));
    TORCH_CHECK(mom->scalar_type() == at::kFloat && mom->numel() >= n_valid, "bad momentum buffer");
    mp = mom->data_ptr<float>();
  }
  fan::SgdParams p{(float)lr, (float)grad_scale, (float)weight_decay, (float)momentum, nesterov ? 1 : 0};
  fan::launch_wire_sgd((int)codec, wire.data_ptr(), (size_t)shard_elems, (int)n_shards, (int)skip_shard, (int)skip_period,
                       master.data_ptr<float>(), lpp, mp, p, (size_t)n_valid, fan_stream());
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "fpga_ai_nic_amd native runtime: CDNA4 HIP kernels, BFP codec, ring planner, RCCL engine";
  m.attr("offload_arch") = "gfx950";
  m.def("wire_shard_bytes", [](int64_t codec, int64_t n_s) { return (int64_t)fan::wire_shard_bytes((int)codec, n_s); });
  m.def("wire_pack", &wire_pack, "encode dense f32/bf16 into the wire format (per shard)");
  m.def("wire_unpack", &wire_unpack, "decode wire format into dense f32/bf16");
  m.def("wire_pack_range", &wire_pack_range, "encode flat elements [begin, end) into the shard layout");
  m.def("wire_pack_to", &wire_pack_to, "encode shard s straight into dsts[s] (e.g. peers' receive slots)");
  m.def("p2p_release_mode", &fan::p2p_release_mode, "release form of peer-storing kernels: 1 block, 2 thread, 0 none");
  m.def("set_p2p_release_mode", &fan::set_p2p_release_mode);
  m.def("p2p_grid_cap", &fan::p2p_grid_cap, "workgroup cap of the peer-storing kernels");
  m.def("set_p2p_grid_cap", &fan::set_p2p_grid_cap);
  m.def("wire_reduce4", &fan::wire_reduce4, "owner reduce + SGD kernel: 4 values per lane (1) or 16 (0)");
  m.def("set_wire_reduce4", &fan::set_wire_reduce4);
  m.def("wire_reduce", &wire_reduce, "sum wire slots (+ dense local) -> wire and/or f32", pybind11::arg("slots"),
        pybind11::arg("n_slots"), pybind11::arg("self_pos"), pybind11::arg("local"), pybind11::arg("out_wire"),
        pybind11::arg("out_f32"), pybind11::arg("shard_elems"), pybind11::arg("codec"));
  m.def("wire_sgd", &wire_sgd, "fused decode + SGD weight update in place");
  fan::register_gemm(m);
  fan::register_nn(m);
  fan::register_planner(m);
  fan::register_engine(m);
}

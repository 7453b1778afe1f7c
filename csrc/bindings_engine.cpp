// Bindings for the native communicator (RCCL over xGMI).
#include "bindings_common.h"
#include "comm/engine.h"
#include "comm/loopback_comm.h"
#include "comm/native_comm.h"
#include "comm/p2p_comm.h"

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
  m.def("p2p_release_event_needed", &p2p_release_event_needed,
        "whether a P2P round records the system-scope release event before its flags (release mode, copy-engine bytes)");
  m.def(
      "p2p_round_flags",
      [](int rank, int world, uint64_t seq, const std::vector<int>& to, const std::vector<int>& from,
         const std::vector<uint64_t>& last_sent) {
        FAN_CHECK((int)last_sent.size() == world, "p2p_round_flags: last_sent needs one entry per rank");
        const RoundFlags r = p2p_round_flags(rank, world, seq, to, from, last_sent);
        auto conv = [](const std::vector<FlagRef>& v) {
          std::vector<std::tuple<int, int, uint64_t>> o;
          for (const FlagRef& f : v) o.emplace_back(f.peer, f.word, f.value);
          return o;
        };
        py::dict d;
        d["credit_waits"] = conv(r.credit_waits);
        d["ready_writes"] = conv(r.ready_writes);
        d["ready_waits"] = conv(r.ready_waits);
        d["ack_writes"] = conv(r.ack_writes);
        return d;
      },
      "the flag words one P2P round touches (peer, word, value): credit waits, ready writes, ready waits, acks -- "
      "the protocol the CP and kernel-flag arms both execute");
  m.def("p2p_coalesce_copies",
        [](const std::vector<std::tuple<uint64_t, uint64_t, uint64_t>>& segs) {
          std::vector<P2PCopy> in;
          for (const auto& t : segs)
            in.push_back({reinterpret_cast<const void*>(std::get<0>(t)), reinterpret_cast<void*>(std::get<1>(t)),
                          (size_t)std::get<2>(t)});
          std::vector<std::tuple<uint64_t, uint64_t, uint64_t>> out;
          for (const P2PCopy& c : coalesce_copies(in))
            out.emplace_back((uint64_t)reinterpret_cast<uintptr_t>(c.src), (uint64_t)reinterpret_cast<uintptr_t>(c.dst),
                             (uint64_t)c.bytes);
          return out;
        },
        "(src, dst, bytes) segments merged into the contiguous runs the copy-engine path issues (pure host logic)");
  pybind11::class_<Comm>(m, "Comm")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world", &Comm::world)
      .def("async_error", &Comm::async_error)
      .def("abort", &Comm::abort)
      .def("ranks_seen", &Comm::ranks_seen, "ranks this communicator reaches (RCCL: ncclCommCount)")
      .def_property_readonly("kind", [](const Comm& c) { return std::string(c.kind()); });
  pybind11::class_<LoopbackFabric, std::shared_ptr<LoopbackFabric>>(m, "LoopbackFabric")
      .def(pybind11::init<int, double>(), pybind11::arg("world"), pybind11::arg("timeout_s") = 60.0)
      .def_property_readonly("world", &LoopbackFabric::world)
      .def("comm", [](std::shared_ptr<LoopbackFabric> f, int rank) { return new LoopbackComm(f, rank); });
  pybind11::class_<LoopbackComm, Comm>(m, "LoopbackComm")
      .def("drop_after", &LoopbackComm::drop_after)
      .def("lose_round", &LoopbackComm::lose_round)
      .def_property_readonly("collectives", &LoopbackComm::collectives);
  pybind11::class_<P2PComm, Comm>(m, "P2PComm")
      .def(pybind11::init<int, int, int, size_t, int>(), pybind11::arg("rank"), pybind11::arg("world"),
           pybind11::arg("device"), pybind11::arg("slot_bytes") = (size_t)128 << 20, pybind11::arg("depth") = 2,
           pybind11::call_guard<pybind11::gil_scoped_release>())
      .def_property_readonly("depth", &P2PComm::depth, "arena slots per sender")
      .def("handles", [](P2PComm& c) { return pybind11::bytes(c.handles()); })
      .def("connect",
           [](P2PComm& c, const std::vector<pybind11::bytes>& all) {
             std::vector<std::string> v;
             for (auto& b : all) v.push_back(std::string(b));
             pybind11::gil_scoped_release nogil;  // a stuck IPC import must not block the run's watchdog thread
             c.connect(v);
           })
      .def_static("connect_local", &P2PComm::connect_local)
      .def_property_readonly("slot_bytes", &P2PComm::slot_bytes)
      .def_property_readonly("payload_bytes", &P2PComm::payload_bytes, "slot bytes messages may use (slot - trailer)")
      .def_property("sdma", &P2PComm::sdma, &P2PComm::set_sdma,
                    "pure copies (prepacked sends, forwards, arena -> scratch) on the copy engines instead of a CU kernel")
      .def_property_readonly("cross_device", &P2PComm::cross_device, "some peer's arena is on another GPU")
      .def_property_readonly("sequence", &P2PComm::sequence)
      .def_property_readonly("uncached", &P2PComm::uncached)
      .def_property_readonly("arena_memory", &P2PComm::arena_memory)
      .def("arena_view",
           [](P2PComm& c) {
             return at::from_blob(c.arena(), {(int64_t)c.arena_bytes()},
                                  at::TensorOptions().dtype(at::kByte).device(at::kCUDA, at::cuda::current_device()));
           },
           "diagnostics: this rank's receive arena as a uint8 tensor (no copy)")
      .def("set_timing", &P2PComm::set_timing, "time every flag wait with device events (stall counters)")
      .def_property("kernel_flags", &P2PComm::kernel_flags, &P2PComm::set_kernel_flags,
                    "flag writes / waits as kernels (system-scope release store / bounded spin + acquire) instead of "
                    "command-processor packets; switch between rounds only")
      .def("kernel_flag_error", &P2PComm::kernel_flag_error, "1 when a kernel-flag wait gave up after its bound")
      .def("stats",
           [](P2PComm& c) {
             P2PComm::Stats t;
             {
               pybind11::gil_scoped_release nogil;  // waits for the timed waits' events
               t = c.stats();
             }
             pybind11::dict d;
             d["ready_waits"] = t.ready_waits;
             d["credit_waits"] = t.credit_waits;
             d["timed_waits"] = t.timed_waits;
             d["ready_stall_ms"] = t.ready_stall_ms;
             d["credit_stall_ms"] = t.credit_stall_ms;
             d["bytes_to_peer"] = t.bytes_to_peer;
             d["kernel_flags"] = c.kernel_flags();
             d["kernel_flag_error"] = c.kernel_flag_error();
             return d;
           },
           "device-side stall counters: flag waits (ready / credit), their device time when timed, bytes per peer")
      .def("reset_stats", &P2PComm::reset_stats)
      .def("flags_snapshot", &P2PComm::flags_snapshot, pybind11::arg("timeout_s") = 2.0,
           "ready-from-src[world] + ack-from-dst[world] words (empty if the copy did not complete in time)")
      .def("all_to_all",
           [](P2PComm& c, const at::Tensor& send, at::Tensor& recv) {
             TORCH_CHECK(bytes_of(send) == bytes_of(recv) && bytes_of(send) % c.world() == 0, "all_to_all sizes");
             c.all_to_all(ptr_of(send), ptr_of(recv), bytes_of(send) / c.world(), fan_stream());
           })
      .def("all_gather",
           [](P2PComm& c, const at::Tensor& send, at::Tensor& recv) {
             TORCH_CHECK(bytes_of(recv) == bytes_of(send) * c.world(), "all_gather sizes");
             c.all_gather(ptr_of(send), ptr_of(recv), bytes_of(send), fan_stream());
           })
      .def("sendrecv", [](P2PComm& c, const std::vector<std::pair<at::Tensor, int>>& sends,
                          const std::vector<std::pair<at::Tensor, int>>& recvs) {
        std::vector<P2POp> s, r;
        for (auto& p : sends) s.push_back({ptr_of(p.first), bytes_of(p.first), p.second});
        for (auto& p : recvs) r.push_back({ptr_of(p.first), bytes_of(p.first), p.second});
        c.sendrecv(s, r, fan_stream());
      });
  pybind11::class_<NativeComm, Comm>(m, "NativeComm")
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

  namespace py = pybind11;
  py::class_<AllReduceEngine>(m, "AllReduceEngine")
      .def(py::init([](Comm* comm, int rank, int world, int codec, int algo, int rings, int64_t max_slice,
                       bool compat, double timeout_s, int priority, bool force_comm, int device, int verify,
                       int64_t chunk_elems, c10::optional<std::vector<std::vector<int>>> links, int ring_sub,
                       int shard_update) {
             EngineConfig c;
             c.codec = codec;
             c.algo = algo;
             c.rings = rings;
             c.max_slice_elems = max_slice;
             c.compat_owner_fp32 = compat;
             c.timeout_s = timeout_s;
             c.stream_priority = priority;
             c.force_comm = force_comm;
             c.verify = verify;
             c.chunk_elems = chunk_elems;
             c.ring_sub = ring_sub;
             c.shard_update = shard_update;
             if (links) {
               TORCH_CHECK((int)links->size() == world, "links: world x world expected");
               c.links.assign((size_t)world * world, 0);
               for (int a = 0; a < world; ++a) {
                 TORCH_CHECK((int)(*links)[a].size() == world, "links: world x world expected");
                 for (int b = 0; b < world; ++b) c.links[(size_t)a * world + b] = (*links)[a][b] != 0;
               }
             }
             return new AllReduceEngine(comm, rank, world, c, device);
           }),
           py::keep_alive<1, 2>(), py::arg("comm").none(true), py::arg("rank"), py::arg("world"), py::arg("codec"),
           py::arg("algo"), py::arg("rings"), py::arg("max_slice_elems"), py::arg("compat_owner_fp32"),
           py::arg("timeout_s"), py::arg("stream_priority"), py::arg("force_comm"), py::arg("device"),
           py::arg("verify") = -1, py::arg("chunk_elems") = 0, py::arg("links") = py::none(), py::arg("ring_sub") = 0,
           py::arg("shard_update") = -1)
      .def_property_readonly("ring_sub", &AllReduceEngine::ring_sub, "sub-slices per direct-ring hop message")
      .def_property_readonly("shard_update", &AllReduceEngine::shard_update,
                             "sharded weight update in force (owner reduce + SGD, all-gather of the bf16 weights)")
      .def("gather_owned",
           [](AllReduceEngine& e, at::Tensor& plane, int64_t n) {
             FAN_T_CUDA_CONTIG(plane);
             TORCH_CHECK(plane.scalar_type() == at::kFloat && plane.numel() >= e.layout(n).n_pad, "f32 bucket plane");
             py::gil_scoped_release nogil;
             e.gather_owned(plane.data_ptr<float>(), n);
           },
           "all-gather an owner-sharded f32 plane (master / momentum of a sharded-update engine) in place")
      .def("layout",
           [](AllReduceEngine& e, int64_t n, int64_t shard, int64_t chunks) {
             const EngineLayout L = e.layout(n, shard, chunks);
             return py::dict(py::arg("n") = L.n, py::arg("n_pad") = L.n_pad, py::arg("algo") = L.algo,
                             py::arg("shard") = L.shard, py::arg("slice") = L.slice, py::arg("blocks") = L.blocks,
                             py::arg("rings") = L.rings, py::arg("part") = L.part, py::arg("chunks") = L.chunks,
                             py::arg("sub") = L.sub);
           },
           py::arg("n"), py::arg("shard") = 0, py::arg("chunks") = 0)
      .def("wire_bytes", [](AllReduceEngine& e, int64_t n) { return e.wire_bytes(e.layout(n)); })
      .def_property_readonly("orders", &AllReduceEngine::orders)
      .def_property_readonly("inline", &AllReduceEngine::is_inline)
      .def_property_readonly("comm_kind",
                             [](AllReduceEngine& e) { return std::string(e.comm() ? e.comm()->kind() : "none"); })
      .def_property_readonly("comm_ranks", [](AllReduceEngine& e) { return e.comm() ? e.comm()->ranks_seen() : 1; },
                             "ranks the engine's communicator reaches (RCCL: ncclCommCount; P2P: mapped peers + 1)")
      .def_property_readonly("stream", [](AllReduceEngine& e) { return (uintptr_t)e.stream(); })
      .def("submit",
           [](AllReduceEngine& e, const at::Tensor& grad, at::Tensor& master, c10::optional<at::Tensor> lp,
              c10::optional<at::Tensor> mom, int64_t n_valid, double lr, double grad_scale, double wd,
              double momentum, bool nesterov, bool defer, bool update, c10::optional<at::Tensor> out_sum,
              c10::optional<at::Tensor> prepacked, int64_t prepacked_elems, int64_t layout_shard,
              int64_t layout_chunks, bool on_producer) {
             FAN_T_CUDA_CONTIG(grad);
             TORCH_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16,
                         "gradients must be f32 or bf16");
             const EngineLayout L = e.layout(n_valid, layout_shard, layout_chunks);
             TORCH_CHECK(grad.numel() >= L.n_pad, "gradient buffer has ", grad.numel(), " elements; layout needs ",
                         L.n_pad);
             if (update) {
               FAN_T_CUDA_CONTIG(master);
               TORCH_CHECK(master.scalar_type() == at::kFloat && master.numel() >= n_valid, "master: f32[n_valid]");
             }
             bf16_t* lpp = nullptr;
             float* momp = nullptr;
             float* outp = nullptr;
             if (lp && lp->defined()) {
               FAN_T_CUDA_CONTIG(*lp);
               TORCH_CHECK(lp->scalar_type() == at::kBFloat16 && lp->numel() >= n_valid, "lp: bf16[n_valid]");
               lpp = reinterpret_cast<bf16_t*>(lp->data_ptr());
             }
             if (mom && mom->defined()) {
               FAN_T_CUDA_CONTIG(*mom);
               TORCH_CHECK(mom->scalar_type() == at::kFloat && mom->numel() >= n_valid, "mom: f32[n_valid]");
               momp = mom->data_ptr<float>();
             }
             if (out_sum && out_sum->defined()) {
               FAN_T_CUDA_CONTIG(*out_sum);
               TORCH_CHECK(out_sum->scalar_type() == at::kFloat && out_sum->numel() >= L.n_pad,
                           "out_sum: f32[n_pad]");
               outp = out_sum->data_ptr<float>();
             }
             const uint8_t* pre = nullptr;
             if (prepacked && prepacked->defined()) {
               FAN_T_CUDA_CONTIG(*prepacked);
               TORCH_CHECK(e.prepack_shape(n_valid)[0] > 0, "this engine configuration cannot take prepacked input");
               const int64_t need = L.algo == 0
                                        ? L.chunks * e.world() * (int64_t)wire_shard_bytes(e.codec(), L.shard)
                                        : (int64_t)L.rings * L.blocks * e.world() * L.sub *
                                              (int64_t)wire_shard_bytes(e.codec(), L.slice / L.sub);
               TORCH_CHECK(prepacked->scalar_type() == at::kByte && prepacked->numel() >= need,
                           "prepacked wire buffer too small");
               pre = prepacked->data_ptr<uint8_t>();
             }
             SgdParams p{(float)lr, (float)grad_scale, (float)wd, (float)momentum, nesterov ? 1 : 0};
             return e.submit(grad.data_ptr(), grad.scalar_type() == at::kFloat ? kF32 : kBF16,
                             update ? master.data_ptr<float>() : nullptr, lpp, momp, n_valid, p, fan_stream(), defer,
                             update, outp, pre, prepacked_elems, layout_shard, layout_chunks, on_producer);
           },
           py::arg("grad"), py::arg("master"), py::arg("lp") = py::none(), py::arg("mom") = py::none(),
           py::arg("n_valid"), py::arg("lr"), py::arg("grad_scale") = 1.0, py::arg("weight_decay") = 0.0,
           py::arg("momentum") = 0.0, py::arg("nesterov") = false, py::arg("defer") = false,
           py::arg("update") = true, py::arg("out_sum") = py::none(), py::arg("prepacked") = py::none(),
           py::arg("prepacked_elems") = 0, py::arg("layout_shard") = 0, py::arg("layout_chunks") = 0,
           py::arg("on_producer") = false, py::call_guard<py::gil_scoped_release>())
      .def("prepack_shape", [](AllReduceEngine& e, int64_t n) {
        const auto s = e.prepack_shape(n);
        return py::make_tuple(s[0], s[1], s[2]);
      })
      .def_property_readonly("codec", &AllReduceEngine::codec)
      .def(
          "commit",
          [](AllReduceEngine& e, int slot, bool after_current, uint32_t seq) {
            e.commit(slot, after_current, after_current ? fan_stream() : nullptr, seq);
          },
          py::arg("slot"), py::arg("after_current") = true, py::arg("seq") = 0u,
          py::call_guard<py::gil_scoped_release>())
      .def(
          "wait_stream", [](AllReduceEngine& e, int slot, uint32_t seq) { e.wait_stream(slot, fan_stream(), seq); },
          py::arg("slot"), py::arg("seq") = 0u)
      .def_property("epilogue_on_producer", &AllReduceEngine::epilogue_on_producer,
                    &AllReduceEngine::set_epilogue_on_producer)
      .def("query", &AllReduceEngine::query, py::arg("slot"), py::arg("seq") = 0u)
      .def("done_word", &AllReduceEngine::done_word)
      .def("slot_seq", &AllReduceEngine::slot_seq)
      .def("synchronize", &AllReduceEngine::synchronize, py::arg("slot"), py::arg("timeout_s") = -1.0,
           py::arg("seq") = 0u, py::call_guard<py::gil_scoped_release>())
      .def("set_tracing", &AllReduceEngine::set_tracing, py::arg("on"), py::arg("capacity") = 1024)
      .def_property_readonly("tracing", &AllReduceEngine::tracing)
      .def(
          "trace_summary",
          [](AllReduceEngine& e) {
            TraceSummary t;
            {
              py::gil_scoped_release nogil;  // waits for the traced requests
              t = e.trace_summary();
            }
            py::dict d;
            d["requests"] = t.requests;
            d["dropped"] = t.dropped;
            d["logical_bytes"] = t.logical_bytes;
            d["wire_bytes"] = t.wire_bytes;
            d["pack_ms"] = t.ms[kTpPacked];
            d["exchange_ms"] = t.ms[kTpExchanged];
            d["reduce_ms"] = t.ms[kTpReduced];
            d["gather_ms"] = t.ms[kTpCommEnd];
            d["epilogue_ms"] = t.ms[kTpEpiEnd];
            d["comm_ms"] = t.comm_ms;
            d["total_ms"] = t.total_ms;
            d["hop_rounds"] = t.hop_rounds;
            d["hop_credit_ms"] = t.hop_credit_ms;
            d["hop_kernel_ms"] = t.hop_kernel_ms;
            d["hop_ready_ms"] = t.hop_ready_ms;
            d["hop_max_ms"] = t.hop_max_ms;
            return d;
          },
          "per-phase device time summed over the traced requests (pack / all-to-all / reduce / all-gather / "
          "epilogue; hw/all_reduce.sv:892-1085 per-state counters)")
      .def("latency_ms", &AllReduceEngine::latency_ms, py::call_guard<py::gil_scoped_release>())
      .def("set_timing", &AllReduceEngine::set_timing)
      .def("diagnostics", &AllReduceEngine::diagnostics)
      .def("debug_status", &AllReduceEngine::debug_status,
           "JSON snapshot: configuration, every slot, counters, comm error, P2P flags + stall counters")
      .def_property_readonly("verify", &AllReduceEngine::verify)
      .def("check_verify", &AllReduceEngine::check_verify,
           "verify mode: raise if any message so far failed its checksum / sequence check")
      .def("set_fault", &AllReduceEngine::set_fault, "test-only fault injection rules (FAN_FAULT grammar)")
      .def("counters",
           [](const AllReduceEngine& e) {
             const EngineCounters& c = e.counters();
             py::dict d;
             d["requests"] = c.requests;
             d["logical_bytes"] = c.logical_bytes;
             d["wire_bytes"] = c.wire_bytes;
             d["host_wait_s"] = c.host_wait_s;
             d["host_waits"] = c.host_waits;
             d["host_spins"] = c.host_spins;
             d["device_ms"] = c.device_ms;
             d["timed_requests"] = c.timed_requests;
             d["forced_commits"] = c.forced_commits;
             d["verified_rows"] = c.verified_rows;
             d["direct_rounds"] = c.direct_rounds;
             d["sharded_updates"] = c.sharded_updates;
             d["peer_bytes"] = c.peer_bytes;
             d["skipped_waits"] = e.skipped_waits();
             return d;
           },
           "perf counters (the NIC's latency / host-stall registers): requests, bytes, host wait, device time")
      .def("reset_counters", &AllReduceEngine::reset_counters)
      .def_property_readonly("scratch_bytes", &AllReduceEngine::scratch_bytes)
      .def_property_readonly("requests", &AllReduceEngine::requests);
}

}  // namespace fan

// Torch-facing bindings for the GEMM, NN and planner components.
#include "bindings_common.h"
#include "bfp/bfp_format.h"
#include "comm/planner.h"
#include "gemm/gemm.h"
#include "gemm/gemm_chain.h"
#include "gemm/gemm_group.h"
#include "nn/nn.h"

namespace fan {

namespace {

int dcode(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return kF32;
  if (t.scalar_type() == at::kBFloat16) return kBF16;
  TORCH_CHECK(false, "expected float32 or bfloat16 tensor");
}

// Row-major 2-D view helpers: returns leading dimension (elements) of a 2-D tensor with unit column stride.
int64_t ld_of(const at::Tensor& t) {
  TORCH_CHECK(t.dim() == 2, "expected a 2-D tensor");
  TORCH_CHECK(t.stride(1) == 1, "expected unit stride in the last dim");
  return t.stride(0);
}

// C = op(A) op(B) with fused epilogue.
//   a_t: if true, A is given as a [K][M] tensor (MN-contiguous), else [M][K]
//   b_t: if true, B is given as a [N][K] tensor (K-contiguous), else [K][N]
void gemm(const at::Tensor& A, bool a_t, const at::Tensor& B, bool b_t, at::Tensor& C, int64_t epilogue,
          const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& aux, bool accumulate,
          int64_t split_k, const c10::optional<at::Tensor>& workspace, int64_t tile_bm, int64_t tile_bn,
          const c10::optional<at::Tensor>& colsum, int64_t tile_waves, const c10::optional<at::Tensor>& wire,
          int64_t wire_shard, int64_t wire_own, int64_t wire_codec, int64_t wire_period, int64_t wire_off,
          const c10::optional<at::Tensor>& upd_master, const c10::optional<at::Tensor>& upd_lp,
          const c10::optional<at::Tensor>& upd_mom, double upd_lr, double upd_grad_scale, double upd_weight_decay,
          double upd_momentum, bool upd_nesterov, bool defer_colsum, bool defer_reduce) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm operands must be GPU tensors");
  TORCH_CHECK(A.scalar_type() == B.scalar_type(), "A and B dtype mismatch");
  GemmArgs g{};
  g.A = A.data_ptr();
  g.B = B.data_ptr();
  g.C = C.data_ptr();
  g.lda = ld_of(A);
  g.ldb = ld_of(B);
  g.ldc = ld_of(C);
  g.M = (int)(a_t ? A.size(1) : A.size(0));
  g.K = (int)(a_t ? A.size(0) : A.size(1));
  g.N = (int)(b_t ? B.size(0) : B.size(1));
  const int64_t kb = b_t ? B.size(1) : B.size(0);
  TORCH_CHECK(kb == g.K, "gemm: inner dimensions differ (", g.K, " vs ", kb, ")");
  TORCH_CHECK(C.size(0) == g.M && C.size(1) == g.N, "gemm: bad C shape");
  g.a_kcontig = !a_t;
  g.b_kcontig = b_t;
  g.epilogue = (int)epilogue;
  g.c_bf16 = C.scalar_type() == at::kBFloat16;
  g.accumulate = accumulate;
  g.split_k = (int)std::max<int64_t>(0, split_k);
  g.tile_bm = (int)tile_bm;
  g.tile_bn = (int)tile_bn;
  g.tile_waves = (int)tile_waves;
  g.defer_reduce = defer_reduce;
  TORCH_CHECK(!defer_reduce || (epilogue == kEpiBias && C.scalar_type() == at::kFloat && !colsum && !accumulate),
              "defer_reduce: the f32 bias epilogue only (the softmax folds the slabs)");
  if (colsum) {
    TORCH_CHECK(colsum->is_cuda() && colsum->is_contiguous() && colsum->scalar_type() == at::kFloat &&
                    colsum->numel() >= g.N,
                "colsum must be a contiguous f32 GPU tensor of >= N elements");
    g.colsum = colsum->data_ptr<float>();
  }
  if (bias) {
    TORCH_CHECK(bias->is_contiguous() && bias->numel() >= g.N, "bad bias");
    g.bias = bias->data_ptr();
  }
  if (aux) {
    TORCH_CHECK(aux->scalar_type() == C.scalar_type(), "aux dtype must match C");
    g.aux = aux->data_ptr();
    g.ldaux = ld_of(*aux);
  }
  if (workspace) g.workspace = workspace->data_ptr();
  if (epilogue == kEpiWire) {
    TORCH_CHECK(wire && wire->is_cuda() && wire->is_contiguous() && wire->scalar_type() == at::kByte,
                "wire epilogue needs a contiguous uint8 GPU wire buffer");
    TORCH_CHECK(wire_shard > 0 && wire_shard % 256 == 0, "wire_shard must be a positive multiple of 256");
    // with colsum the encoded bias segment follows C: flat M*ldc .. M*ldc + N - 1
    TORCH_CHECK(wire_off >= 0 && wire_off % 16 == 0, "wire_off must be a non-negative multiple of 16");
    const int64_t last = wire_off + (g.colsum ? (int64_t)g.M * g.ldc + g.N - 1 : (int64_t)(g.M - 1) * g.ldc + g.N - 1);
    const int64_t need = (last / wire_shard + 1) * (int64_t)wire_shard_bytes((int)wire_codec, (size_t)wire_shard);
    TORCH_CHECK(wire->numel() >= need, "wire buffer too small: ", wire->numel(), " < ", need);
    g.wire = wire->data_ptr<uint8_t>();
    g.wire_shard = wire_shard;
    g.wire_own = (int)wire_own;
    g.wire_period = (int)wire_period;
    g.wire_codec = (int)wire_codec;
    g.wire_off = wire_off;
    if (upd_master) {  // fused local update: the bucket planes cover every flat index the epilogue touches
      auto plane = [&](const at::Tensor& t, at::ScalarType st, const char* what) {
        TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == st && t.numel() > last &&
                        t.data_ptr() != nullptr && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
                    "fused update: ", what, " must be a contiguous, 16-B aligned GPU plane covering the bucket");
      };
      TORCH_CHECK(wire_own == -1, "fused update: no owner shard (single-rank engine)");
      TORCH_CHECK(wire_codec == kBfpRne, "fused update: rne codec only");
      plane(*upd_master, at::kFloat, "master");
      g.upd_master = upd_master->data_ptr<float>();
      if (upd_lp) {
        plane(*upd_lp, at::kBFloat16, "lp");
        g.upd_lp = reinterpret_cast<bf16_t*>(upd_lp->data_ptr());
      }
      if (upd_mom) {
        plane(*upd_mom, at::kFloat, "mom");
        g.upd_mom = upd_mom->data_ptr<float>();
      }
      g.upd = SgdParams{(float)upd_lr, (float)upd_grad_scale, (float)upd_weight_decay, (float)upd_momentum,
                        upd_nesterov ? 1 : 0};
      g.defer_colsum = defer_colsum && g.colsum != nullptr;
    }
  }
  if (A.scalar_type() == at::kBFloat16) {
    TORCH_CHECK(bias ? bias->scalar_type() == at::kBFloat16 : true, "bias must be bf16");
    const GemmPlan p = gemm_bf16_plan(g.M, g.N, g.K, g.split_k, g.tile_bm, g.tile_bn, g.tile_waves);
    // split-K slabs, then bias-gradient partials (at most split_k per tile row)
    const int64_t need = (p.split_k > 1 ? (int64_t)p.split_k * g.M * g.N : 0) +
                         (g.colsum && p.bm > 0 ? (int64_t)p.split_k * ((g.M + p.bm - 1) / p.bm) * g.N : 0);
    if (need > 0 || p.split_k > 1) {
      TORCH_CHECK(workspace && workspace->scalar_type() == at::kFloat && workspace->is_contiguous() &&
                      workspace->numel() >= need,
                  "gemm: split-K ", p.split_k, (g.colsum ? " with colsum" : ""), " needs an f32 workspace of ", need,
                  " elements");
    }
    TORCH_CHECK(gemm_bf16_supported(g), "gemm_bf16: unsupported shape M=", g.M, " N=", g.N, " K=", g.K,
                " split_k=", g.split_k);
    launch_gemm_bf16(g, fan_stream());
  } else {
    TORCH_CHECK(A.scalar_type() == at::kFloat, "gemm: A must be bf16 or f32");
    const int sk = gemm_f32_split(g.M, g.N, g.K, g.split_k);
    if (sk > 1) {
      const int64_t need = (int64_t)sk * g.M * g.N;
      TORCH_CHECK(workspace && workspace->scalar_type() == at::kFloat && workspace->is_contiguous() &&
                      workspace->numel() >= need,
                  "gemm_f32: split-K ", sk, " needs an f32 workspace of ", need, " elements");
    }
    TORCH_CHECK(gemm_f32_supported(g), "gemm_f32: unsupported shape M=", g.M, " N=", g.N, " K=", g.K);
    launch_gemm_f32(g, fan_stream());
  }
}

// Up to kGroupMax bwd-weight GEMMs C_i = X_i^T . dY_i (+ colsum_i = sum of dY_i's rows) in one dispatch, f32 out or
// BFP-encoded into one wire buffer at flat offsets offs[i] (the bias segment right after each C_i).
void gemm_wgrad_group(const std::vector<at::Tensor>& Xs, const std::vector<at::Tensor>& dYs,
                      const std::vector<at::Tensor>& Cs, const std::vector<at::Tensor>& colsums,
                      const std::vector<int64_t>& offs, at::Tensor& workspace, const c10::optional<at::Tensor>& wire,
                      int64_t wire_shard, int64_t wire_own, int64_t wire_codec, int64_t wire_period) {
  const size_t n = Xs.size();
  TORCH_CHECK(n >= 1 && n <= (size_t)kGroupMax && dYs.size() == n && Cs.size() == n && colsums.size() == n &&
                  (offs.empty() || offs.size() == n),
              "gemm_wgrad_group: 1..", kGroupMax, " problems, one X, dY, C, colsum (and wire offset) each");
  TORCH_CHECK(workspace.is_cuda() && workspace.scalar_type() == at::kFloat && workspace.is_contiguous(),
              "gemm_wgrad_group: f32 GPU workspace");
  std::vector<GemmArgs> g(n);
  int64_t ws_off = 0;
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor &X = Xs[i], &dY = dYs[i], &C = Cs[i], &cs = colsums[i];
    TORCH_CHECK(X.is_cuda() && dY.is_cuda() && C.is_cuda() && cs.is_cuda(), "gemm_wgrad_group: GPU tensors");
    TORCH_CHECK(X.scalar_type() == at::kBFloat16 && dY.scalar_type() == at::kBFloat16 &&
                    C.scalar_type() == at::kFloat && cs.scalar_type() == at::kFloat && cs.is_contiguous(),
                "gemm_wgrad_group: bf16 X / dY, f32 C / colsum");
    TORCH_CHECK(X.dim() == 2 && dY.dim() == 2 && X.size(0) == dY.size(0) && C.dim() == 2 && C.size(0) == X.size(1) &&
                    C.size(1) == dY.size(1) && cs.numel() >= dY.size(1),
                "gemm_wgrad_group: shapes (X [K][M], dY [K][N], C [M][N], colsum [N])");
    GemmArgs& a = g[i];
    a.A = X.data_ptr(); a.lda = ld_of(X);
    a.B = dY.data_ptr(); a.ldb = ld_of(dY);
    a.C = C.data_ptr(); a.ldc = ld_of(C);
    a.M = (int)X.size(1); a.N = (int)dY.size(1); a.K = (int)X.size(0);
    a.a_kcontig = false; a.b_kcontig = false; a.c_bf16 = false;
    a.colsum = cs.data_ptr<float>();
    a.epilogue = wire ? kEpiWire : kEpiNone;
    a.workspace = workspace.data_ptr<float>() + ws_off;
    ws_off += (gemm_wgrad_group_ws(a) + 3) / 4 * 4;
    if (wire) {
      TORCH_CHECK(wire->is_cuda() && wire->is_contiguous() && wire->scalar_type() == at::kByte,
                  "wire epilogue needs a contiguous uint8 GPU wire buffer");
      TORCH_CHECK(wire_shard > 0 && wire_shard % 256 == 0, "wire_shard must be a positive multiple of 256");
      const int64_t off = offs.empty() ? 0 : offs[i];
      TORCH_CHECK(off >= 0 && off % 16 == 0, "wire offsets must be non-negative multiples of 16");
      const int64_t last = off + (int64_t)a.M * a.ldc + a.N - 1;
      const int64_t need = (last / wire_shard + 1) * (int64_t)wire_shard_bytes((int)wire_codec, (size_t)wire_shard);
      TORCH_CHECK(wire->numel() >= need, "wire buffer too small: ", wire->numel(), " < ", need);
      a.wire = wire->data_ptr<uint8_t>();
      a.wire_shard = wire_shard;
      a.wire_own = (int)wire_own;
      a.wire_period = (int)wire_period;
      a.wire_codec = (int)wire_codec;
      a.wire_off = off;
    }
  }
  TORCH_CHECK(workspace.numel() >= ws_off, "gemm_wgrad_group: workspace of ", ws_off, " floats needed");
  TORCH_CHECK(gemm_wgrad_group_supported(g.data(), (int)n),
              "gemm_wgrad_group: unsupported (M % 256, N % 128, K % 64, aligned operands, at most ", 64 * kNumCU,
              " workgroups)");
  launch_gemm_wgrad_group(g.data(), (int)n, fan_stream());
}

// The GEMMs of one MLP pass as ONE persistent launch (gemm_chain.h). kind 0 (forward): A0 = X [M][K0], Bs[i] = W_i
// [K_i][N_i], Cs[i] = the layer outputs (bf16 hidden, the last bf16 or f32 logits), biases[i]; kind 1 (backward data):
// A0 = dZ [M][K0], Bs[i] = W [N_i][K_i] (K-contiguous), Cs[i] = dX outputs (bf16), auxes[i] = the ReLU-mask
// activations; epis[i]: each stage's epilogue (the chain checks it is one of its configurations). Stage i + 1 reads Cs[i]. counters: int32 GPU tensor of at least gemm_chain_words(n, M) elements,
// zero before the first call (the kernel leaves it zero). Returns false (nothing launched) when the chain does not
// take these shapes / layouts; dry_run: only that check.
bool gemm_chain(int64_t kind, const at::Tensor& A0, const std::vector<at::Tensor>& Bs, const std::vector<at::Tensor>& Cs,
                const std::vector<c10::optional<at::Tensor>>& biases,
                const std::vector<c10::optional<at::Tensor>>& auxes, const std::vector<int64_t>& epis,
                at::Tensor& counters, bool dry_run) {
  const int n = (int)Bs.size();
  TORCH_CHECK(n >= 1 && (int)Cs.size() == n && (int)biases.size() == n && (int)auxes.size() == n &&
                  (int)epis.size() == n,
              "gemm_chain: one B, C, bias, aux and epilogue entry per stage");
  if (n > gemm_chain_max_stages()) return false;
  std::vector<GemmArgs> g(n);
  for (int i = 0; i < n; ++i) {
    const at::Tensor& A = i == 0 ? A0 : Cs[i - 1];
    const at::Tensor& B = Bs[i];
    const at::Tensor& C = Cs[i];
    for (const at::Tensor* t : {&A, &B, &C})
      if (!t->is_cuda() || t->dim() != 2 || t->stride(1) != 1) return false;
    if (A.scalar_type() != at::kBFloat16 || B.scalar_type() != at::kBFloat16) return false;
    GemmArgs& a = g[i];
    a.A = A.data_ptr();
    a.B = B.data_ptr();
    a.C = C.data_ptr();
    a.lda = A.stride(0);
    a.ldb = B.stride(0);
    a.ldc = C.stride(0);
    a.M = (int)A.size(0);
    a.K = (int)A.size(1);
    a.N = (int)(kind == kChainBwdData ? B.size(0) : B.size(1));
    if ((kind == kChainBwdData ? B.size(1) : B.size(0)) != a.K || C.size(0) != a.M || C.size(1) != a.N) return false;
    a.a_kcontig = true;
    a.b_kcontig = kind == kChainBwdData;
    a.c_bf16 = C.scalar_type() == at::kBFloat16;
    if (!a.c_bf16 && C.scalar_type() != at::kFloat) return false;
    a.split_k = 1;
    if (kind == kChainFwd) {
      if (!biases[i] || biases[i]->scalar_type() != at::kBFloat16 || biases[i]->numel() < a.N) return false;
      a.bias = biases[i]->data_ptr();
      a.epilogue = (int)epis[i];
    } else {
      if (!auxes[i] || auxes[i]->scalar_type() != at::kBFloat16 || auxes[i]->dim() != 2 ||
          auxes[i]->stride(1) != 1 || auxes[i]->size(0) != a.M || auxes[i]->size(1) != a.N)
        return false;
      a.aux = auxes[i]->data_ptr();
      a.ldaux = auxes[i]->stride(0);
      a.epilogue = (int)epis[i];
    }
  }
  if (!gemm_chain_supported(g.data(), n, (int)kind)) return false;
  TORCH_CHECK(counters.is_cuda() && counters.scalar_type() == at::kInt && counters.is_contiguous() &&
                  counters.numel() >= gemm_chain_counter_words(n, g[0].M),
              "gemm_chain: counters must be a contiguous int32 GPU tensor of gemm_chain_words(n, M) elements");
  if (dry_run) return true;
  launch_gemm_chain(g.data(), n, (int)kind, reinterpret_cast<unsigned*>(counters.data_ptr()), fan_stream());
  return true;
}

int64_t gemm_wgrad_group_ws_floats(const std::vector<std::pair<int64_t, int64_t>>& mn) {
  int64_t w = 0;
  for (const auto& p : mn) w += ((p.first / 256) * p.second + 3) / 4 * 4;
  return w;
}

pybind11::tuple gemm_plan(int64_t M, int64_t N, int64_t K, int64_t split_k, int64_t tile_bm, int64_t tile_bn,
                          int64_t tile_waves) {
  GemmPlan p = gemm_bf16_plan((int)M, (int)N, (int)K, (int)split_k, (int)tile_bm, (int)tile_bn, (int)tile_waves);
  return pybind11::make_tuple(p.bm, p.bn, p.split_k, p.waves);
}

bool gemm_supported(int64_t M, int64_t N, int64_t K, bool bf16, int64_t split_k) {
  GemmArgs g{};
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = g.ldb = 64;
  g.ldc = N;
  g.split_k = (int)split_k;
  g.workspace = (void*)16;
  return bf16 ? gemm_bf16_supported(g) : gemm_f32_supported(g);
}

void softmax_xent(const at::Tensor& logits, const at::Tensor& labels, at::Tensor& dlogits, at::Tensor& loss_rows,
                  double grad_scale) {
  TORCH_CHECK(logits.is_cuda() && labels.is_cuda() && dlogits.is_cuda() && loss_rows.is_cuda(), "GPU tensors");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous(), "labels must be int32");
  TORCH_CHECK(loss_rows.scalar_type() == at::kFloat, "loss_rows must be f32");
  const int M = (int)logits.size(0), Cc = (int)logits.size(1);
  TORCH_CHECK(dlogits.size(0) == M && dlogits.size(1) == Cc, "dlogits shape");
  launch_softmax_xent(dcode(logits), logits.data_ptr(), ld_of(logits), labels.data_ptr<int32_t>(), dcode(dlogits),
                      dlogits.data_ptr(), ld_of(dlogits), loss_rows.data_ptr<float>(), M, Cc, (float)grad_scale,
                      fan_stream());
}

void softmax_xent_slabs(const at::Tensor& ws, int64_t sk, const at::Tensor& bias, at::Tensor& logits,
                        const at::Tensor& labels, at::Tensor& dlogits, at::Tensor& loss_rows, double grad_scale) {
  TORCH_CHECK(ws.is_cuda() && bias.is_cuda() && logits.is_cuda() && labels.is_cuda() && dlogits.is_cuda() &&
                  loss_rows.is_cuda(), "GPU tensors");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && logits.scalar_type() == at::kFloat &&
                  bias.scalar_type() == at::kBFloat16 && bias.is_contiguous(), "f32 slabs / logits, bf16 bias");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && loss_rows.scalar_type() == at::kFloat,
              "int32 labels, f32 loss rows");
  const int M = (int)logits.size(0), Cc = (int)logits.size(1);
  TORCH_CHECK(dlogits.size(0) == M && dlogits.size(1) == Cc && bias.numel() >= Cc, "shapes");
  TORCH_CHECK(sk >= 1 && ws.numel() >= sk * (int64_t)M * Cc, "workspace holds sk slabs of M x C");
  launch_softmax_xent_slabs(ws.data_ptr<float>(), (int)sk, reinterpret_cast<const bf16_t*>(bias.data_ptr()),
                            logits.data_ptr<float>(), ld_of(logits), labels.data_ptr<int32_t>(), dcode(dlogits),
                            dlogits.data_ptr(), ld_of(dlogits), loss_rows.data_ptr<float>(), M, Cc,
                            (float)grad_scale, fan_stream());
}

void col_sum(const at::Tensor& x, at::Tensor& out, double scale, bool accumulate, at::Tensor& workspace) {
  TORCH_CHECK(x.is_cuda() && out.is_cuda() && workspace.is_cuda(), "GPU tensors");
  const int M = (int)x.size(0), N = (int)x.size(1);
  TORCH_CHECK(out.numel() >= N && out.is_contiguous(), "out too small");
  TORCH_CHECK(workspace.scalar_type() == at::kFloat && (size_t)workspace.numel() >= col_sum_workspace_floats(M, N),
              "workspace too small");
  launch_col_sum(dcode(x), x.data_ptr(), ld_of(x), M, N, dcode(out), out.data_ptr(), (float)scale, accumulate,
                 workspace.data_ptr<float>(), fan_stream());
}

}  // namespace

void register_gemm(pybind11::module_& m) {
  m.def("gemm", &gemm, "MFMA GEMM with fused epilogue", pybind11::arg("A"), pybind11::arg("a_t"), pybind11::arg("B"),
        pybind11::arg("b_t"), pybind11::arg("C"), pybind11::arg("epilogue") = 0, pybind11::arg("bias") = pybind11::none(),
        pybind11::arg("aux") = pybind11::none(), pybind11::arg("accumulate") = false, pybind11::arg("split_k") = 1,
        pybind11::arg("workspace") = pybind11::none(), pybind11::arg("tile_bm") = 0, pybind11::arg("tile_bn") = 0,
        pybind11::arg("colsum") = pybind11::none(), pybind11::arg("tile_waves") = 0,
        pybind11::arg("wire") = pybind11::none(), pybind11::arg("wire_shard") = 0, pybind11::arg("wire_own") = -1,
        pybind11::arg("wire_codec") = 1, pybind11::arg("wire_period") = 0, pybind11::arg("wire_off") = 0,
        pybind11::arg("upd_master") = pybind11::none(), pybind11::arg("upd_lp") = pybind11::none(),
        pybind11::arg("upd_mom") = pybind11::none(), pybind11::arg("upd_lr") = 0.0,
        pybind11::arg("upd_grad_scale") = 1.0, pybind11::arg("upd_weight_decay") = 0.0,
        pybind11::arg("upd_momentum") = 0.0, pybind11::arg("upd_nesterov") = false,
        pybind11::arg("defer_colsum") = false, pybind11::arg("defer_reduce") = false);
  m.def("gemm_supported", &gemm_supported);
  m.def("gemm_flush_colsum", []() { return gemm_flush_colsum(fan_stream()); },
        "launch the bias-gradient reduces queued on the current stream by defer_colsum GEMMs; returns how many");
  m.def("gemm_pending_colsum", []() { return gemm_pending_colsum(fan_stream()); },
        "bias-gradient reduces queued on the current stream");
  m.def("gemm_wgrad_group", &gemm_wgrad_group,
        "up to 8 bwd-weight GEMMs (+ fused bias gradients, f32 or BFP wire epilogue) in one dispatch",
        pybind11::arg("Xs"), pybind11::arg("dYs"), pybind11::arg("Cs"), pybind11::arg("colsums"),
        pybind11::arg("offs"), pybind11::arg("workspace"), pybind11::arg("wire") = pybind11::none(),
        pybind11::arg("wire_shard") = 0, pybind11::arg("wire_own") = -1, pybind11::arg("wire_codec") = 1,
        pybind11::arg("wire_period") = 0);
  m.def("gemm_wgrad_group_ws", &gemm_wgrad_group_ws_floats, "f32 workspace elements for a group of (M, N) problems");
  m.def("gemm_chain", &gemm_chain, "the GEMMs of one MLP pass as one persistent launch (row-panel hand-offs)",
        pybind11::arg("kind"), pybind11::arg("A0"), pybind11::arg("Bs"), pybind11::arg("Cs"), pybind11::arg("biases"),
        pybind11::arg("auxes"), pybind11::arg("epis"), pybind11::arg("counters"), pybind11::arg("dry_run") = false);
  m.def("gemm_chain_words", &gemm_chain_counter_words, "int32 words of a layer-chain counter block",
        pybind11::arg("n"), pybind11::arg("M"));
  m.def("gemm_set_prio", [](int on) { gemm_prio_flag().store(on); },
        "4-wave pipelined GEMM waves at s_setprio 2 (another stream's kernels issue in their stalls)");
  m.def("gemm_prio", []() { return gemm_prio_flag().load(); });
  m.def("gemm_set_ovl", [](int on) { gemm_ovl_flag().store(on); },
        "256x256 bf16 plans on the persistent loop with overlapped tile transitions (pl4_run OVL)");
  m.def("gemm_ovl", []() { return gemm_ovl_flag().load(); });
  m.def("gemm_set_reduce4", [](int on) { gemm_reduce4_flag().store(on); },
        "split-K wire / fused-update reduce: 4 values per lane (1) or one 16-value group per lane (0)");
  m.def("gemm_reduce4", []() { return gemm_reduce4_flag().load(); });
  m.def("gemm_f32_split", &gemm_f32_split, "f32 GEMM split-K factor (split_k <= 0: automatic)", pybind11::arg("M"),
        pybind11::arg("N"), pybind11::arg("K"), pybind11::arg("split_k") = 0);
  m.def("gemm_set_main_loop", [](int mode) { gemm_main_loop_flag().store(mode); },
        "256x256 GEMM tiles: 0 one-role, 2 pipelined (4 or 8 waves by layout / K), 3 pipelined 4-wave, "
        "5 pipelined 8-wave");
  m.def("gemm_main_loop", []() { return gemm_main_loop_flag().load(); });
  m.def("gemm_set_persist", [](int cap) { gemm_persist_flag().store(cap); },
        "grid cap of the persistent 4-wave GEMM kernel (<= 0: one workgroup per tile)");
  m.def("gemm_persist", []() { return gemm_persist_flag().load(); });
  m.def("gemm_set_stamp_buffer", [](const c10::optional<at::Tensor>& t) {
          gemm_set_stamp_buffer(t ? t->data_ptr() : nullptr);
        },
        "diagnostic builds only: int64 GPU buffer [8 wg][8 waves][64 K-tiles][5] for the GEMM loop's s_memtime stamps");
  m.def("gemm_plan", &gemm_plan, "bf16 GEMM tile/split-K plan (bm, bn, split_k, waves); bm == 0: unsupported",
        pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("K"), pybind11::arg("split_k") = 0,
        pybind11::arg("tile_bm") = 0, pybind11::arg("tile_bn") = 0, pybind11::arg("tile_waves") = 0);
  m.attr("EPI_NONE") = (int)kEpiNone;
  m.attr("EPI_BIAS") = (int)kEpiBias;
  m.attr("EPI_BIAS_RELU") = (int)kEpiBiasRelu;
  m.attr("EPI_RELU_MASK") = (int)kEpiReluMask;
  m.attr("EPI_WIRE") = (int)kEpiWire;
}

void register_nn(pybind11::module_& m) {
  m.def("softmax_xent", &softmax_xent, "fused softmax + cross-entropy fwd/bwd");
  m.def("softmax_xent_slabs", &softmax_xent_slabs,
        "softmax + cross-entropy over the classifier GEMM's unreduced split-K slabs (+ bias; logits written)");
  m.def("col_sum", &col_sum, "bias-gradient column sum");
  m.def("col_sum_workspace_floats", [](int64_t M, int64_t N) { return (int64_t)col_sum_workspace_floats((int)M, (int)N); });
}

void register_planner(pybind11::module_& m) {
  m.def("ring_geometry", [](int64_t n, int world, int64_t max_slice) {
    auto g = ring_geometry(n, world, max_slice);
    return pybind11::make_tuple(g.n, g.slice_elems, g.blocks, g.n_pad);
  });
  m.def("ring_plan", [](int world, int position, int64_t blocks) {
    auto rounds = ring_plan(world, position, blocks);
    std::vector<std::vector<int32_t>> out;
    out.reserve(rounds.size());
    for (auto& r : rounds) out.push_back({r.send_slice, r.send_src, r.recv_slice, r.recv_full, r.owned});
    return out;
  });
  m.def(
      "ring_orders",
      [](int world, int max_rings, c10::optional<std::vector<std::vector<int>>> links) {
        if (!links) return ring_orders(world, max_rings);
        std::vector<char> l((size_t)world * world, 0);
        TORCH_CHECK((int)links->size() == world, "links: world rows expected");
        for (int a = 0; a < world; ++a) {
          TORCH_CHECK((int)(*links)[a].size() == world, "links: world columns expected");
          for (int b = 0; b < world; ++b) l[(size_t)a * world + b] = (*links)[a][b] != 0;
        }
        return ring_orders(world, max_rings, &l);
      },
      pybind11::arg("world"), pybind11::arg("max_rings"), pybind11::arg("links") = pybind11::none(),
      "arc-disjoint directed Hamiltonian rings over the (optional) link matrix links[a][b]: a can send to b");
}

}  // namespace fan

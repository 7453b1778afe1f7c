"""End-to-end numerics of the training path on the GPU: the bf16 HIP MLP (hand-written MFMA GEMMs, softmax-xent kernel,
BFP-rne round trip of every gradient group + SGD fused into the bwd-weight GEMM epilogue, C++ engine) trained for 10
steps against an fp32 ``torch.autograd`` + SGD reference started from the same weights on the same GPU.

Two checks, with bounds derived from the formats (the measured values are printed):
* per step, from the SAME weights (the reference is re-seeded from the HIP model's bf16 compute weights before each
  step): the HIP update of every layer vs the fp32 autograd update. BFP rne: a 16-value group is re-expressed as 8-bit
  mantissas under its max exponent E with 2^(E-127) <= max|group|, so the step is 2^(E-133) <= 2^-6 max|group| and
  one element's rounding error is at most 2^-7 max|group| (SURVEY.md Appendix A's 2^-6 is truncation's). Over a
  layer the error norm is <= 2^-7 sqrt(16 sum_g max_g^2) <= 2^-5 ||update|| (max_g^2 <= the group's sum of squares).
  The bf16 operands of the HIP GEMMs (activations, dZ; f32 accumulation, ~2^-9 relative each) add at most 2^-7:
  per-step update error <= 2^-5 + 2^-7 relative, and the step's loss within 1e-4 relative (same weights, same f32
  loss; only bf16 rounding of the logits' inputs differs);
* over a 10-step trajectory: ||dW_hip - dW_ref|| <= (2^-5 + 2^-7) * sum_t ||update_t|| (the per-step errors add up at
  most along the path). The losses track within one step of the reference's decrease: the HIP forward computes with
  bf16 copies of the f32 master weights, which swallow an update smaller than half a bf16 ulp (2^-9 relative) until
  the master has accumulated enough of them — the loss lags, then catches up (the master weights do not).
The batch is the same every step (the net memorises it), so the loss falls and the updates stay aligned. A wrong
update (sign, scale, a missing layer, a stale weight copy) is off by >= 50 % of the update, far outside all of these.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SIZES = [1024, 4096, 4096, 1024]
MB, STEPS, LR = 512, 10, 0.1
UPDATE_BOUND = 2.0 ** -5 + 2.0 ** -7  # BFP rne worst case + bf16 roundings (per step / per unit of update path)
UPDATE_NET_BOUND = 0.15               # relative to the net update of the trajectory (catches any gross error)
LOSS_SAME_WEIGHTS_REL = 1e-4


def _ref_step(W, b, x, y):
    """One fp32 autograd step from (W, b): (loss, per-layer update [dW | db])."""
    Ws = [w.clone().requires_grad_(True) for w in W]
    bs = [v.clone().requires_grad_(True) for v in b]
    h = x.float()
    for i in range(len(Ws)):
        h = h @ Ws[i] + bs[i]
        if i + 1 < len(Ws):
            h = torch.relu(h)
    loss = F.cross_entropy(h, y.long())
    gs = torch.autograd.grad(loss, Ws + bs)
    L = len(Ws)
    return float(loss.detach()), [torch.cat([(-LR * gs[i]).flatten(), -LR * gs[L + i]]) for i in range(L)]


def _reference(W0, b0, batches):
    """fp32 autograd + plain SGD (w -= lr * g) on the same batches."""
    Ws = [w.clone().requires_grad_(True) for w in W0]
    bs = [b.clone().requires_grad_(True) for b in b0]
    losses, path = [], [0.0] * len(Ws)
    for x, y in batches:
        h = x.float()
        for i in range(len(Ws)):
            h = h @ Ws[i] + bs[i]
            if i + 1 < len(Ws):
                h = torch.relu(h)
        loss = F.cross_entropy(h, y.long())
        losses.append(float(loss.item()))
        gs = torch.autograd.grad(loss, Ws + bs)
        with torch.no_grad():
            for i in range(len(Ws)):
                path[i] += float(LR * torch.cat([gs[i].flatten(), gs[len(Ws) + i]]).norm())
            for p, g in zip(Ws + bs, gs):
                p -= LR * g
    return [w.detach() for w in Ws], [b.detach() for b in bs], losses, path


def test_bf16_hip_training_tracks_fp32_autograd():
    from fpga_ai_nic_amd import _ext
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import ThreadFabric

    _ext.require()
    dev = torch.device("cuda", 0)
    eng = make_engine(ThreadFabric(1).transport(0), "bfp", rounding="rne", impl="native")
    m = MLP(SIZES, dtype=torch.bfloat16, device=dev, seed=7, pad_fn=lambda n: eng.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=LR)
    assert tr.prepack and tr.fused_update, "expected the production path: GEMM-encoded wire + fused update"
    # the reference starts from the weights the HIP model computes with (its bf16 copy, as f32)
    W0 = [l.w.float().clone() for l in m.layers]
    b0 = [l.b.float().clone() for l in m.layers]
    for l in m.layers:  # the f32 masters too, so both runs start from identical values
        l.master[: l.n].copy_(l.lp[: l.n].float())
    g = torch.Generator().manual_seed(11)
    x = (torch.rand(MB, SIZES[0], generator=g) * 2 - 1).to(dev, torch.bfloat16)
    y = torch.randint(0, SIZES[-1], (MB,), generator=g, dtype=torch.int32).to(dev)
    batches = [(x, y)] * STEPS
    hip_losses = []
    for x, y in batches:
        hip_losses.append(float(tr.step(x, y).float().mean().item()))
    tr.finish()
    torch.cuda.synchronize()
    assert tr.fused_updates == STEPS * m.L
    Wr, br, ref_losses, path = _reference(W0, b0, batches)
    # per step from the same weights: 3 more HIP steps, each against a reference step from the HIP compute weights
    step_err, step_loss = [], []
    for _ in range(3):
        Wm = [l.w_master.clone() for l in m.layers]
        bm = [l.b_master.clone() for l in m.layers]
        rl, upd = _ref_step([l.w.float() for l in m.layers], [l.b.float() for l in m.layers], x, y)
        hl = float(tr.step(x, y).float().mean().item())
        tr.finish()
        torch.cuda.synchronize()
        step_loss.append(abs(hl - rl) / rl)
        for i, l in enumerate(m.layers):
            dh = torch.cat([(l.w_master - Wm[i]).flatten(), l.b_master - bm[i]])
            step_err.append(float((dh - upd[i]).norm() / upd[i].norm()))

    # within one step of the reference's decrease (bf16 compute weights lag the f32 masters, see above)
    lag = [abs(a - b) - max(abs(ref_losses[max(t - 1, 0)] - ref_losses[t]), 1e-4 * b)
           for t, (a, b) in enumerate(zip(hip_losses, ref_losses))]
    upd_net, upd_path = [], []
    for i, l in enumerate(m.layers):
        dh = torch.cat([(l.w_master - W0[i]).flatten(), l.b_master - b0[i]])
        dr = torch.cat([(Wr[i] - W0[i]).flatten(), br[i] - b0[i]])
        err = float((dh - dr).norm())
        upd_net.append(err / float(dr.norm()))
        upd_path.append(err / path[i])
    print(f"\nloss hip {['%.5f' % v for v in hip_losses]}\nloss ref {['%.5f' % v for v in ref_losses]}\n"
          f"trajectory: update error / net update per layer {['%.4f' % v for v in upd_net]}; / update path length "
          f"{['%.4f' % v for v in upd_path]}\nper step from the same weights: update rel error "
          f"{['%.4f' % v for v in step_err]}, loss rel diff {['%.1e' % v for v in step_loss]}")
    assert all(math.isfinite(v) for v in hip_losses)
    assert ref_losses[-1] < ref_losses[0] - 0.01 and hip_losses[-1] < hip_losses[0] - 0.01, "loss did not fall"
    assert max(step_err) <= UPDATE_BOUND, step_err
    assert max(step_loss) <= LOSS_SAME_WEIGHTS_REL, step_loss
    assert max(upd_path) <= UPDATE_BOUND, upd_path
    assert max(upd_net) <= UPDATE_NET_BOUND, upd_net
    assert max(lag) <= 0, (lag, hip_losses, ref_losses)

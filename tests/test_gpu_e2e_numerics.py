"""End-to-end numerics of the training path on the GPU: the bf16 HIP MLP (hand-written MFMA GEMMs, softmax-xent kernel,
BFP-rne round trip of every gradient group + SGD fused into the bwd-weight GEMM epilogue, C++ engine) trained against
PyTorch references on the same GPU, from the same weights.

Three checks (measured values printed):
1. per step vs a bf16-EMULATING fp32 reference with the codec oracle: the reference rounds to bf16 exactly where the
   HIP step does (activations after bias + ReLU, the softmax gradient, each dZ after the ReLU mask; weights are the
   model's bf16 copy; every GEMM accumulates in f32) and applies SGD with the gradient taken through the bit-exact BFP
   oracle (ops/bfp_oracle.quantize, 16-value groups of the flat [W | b] bucket). What is left is summation order
   inside the f32 GEMMs (~1e-6 relative) and the rare element it moves across a bf16 or BFP rounding boundary: each
   layer's update within 1e-2 relative, the loss within 1e-5.
2. per step vs plain fp32 torch.autograd from the same bf16 weights: BFP rne moves a gradient element by at most half
   a step, 2^-7 max|group| (the group's step is 2^(E-133) <= 2^-6 max|group|; SURVEY.md Appendix A's 2^-6 is
   truncation's), so over a layer the update error is <= 2^-7 sqrt(16 sum_g max_g^2) <= 2^-5 ||update|| (max_g^2 <= the
   group's sum of squares); the bf16 roundings of check 1 add the rest (bound 2^-6 for them: activations and dZ at
   2^-9 relative, compounded over two backward GEMM levels and the ReLU masks they can flip): <= 2^-5 + 2^-6.
3. a 10-step trajectory vs fp32 autograd + SGD: the accumulated update error <= (2^-5 + 2^-6) x the update path
   length, <= 15 % of the net update, and each step's loss within one step's decrease of the reference's (the HIP
   forward computes with bf16 copies of the f32 master weights, which swallow updates below half a bf16 ulp until the
   master has accumulated enough of them: the loss lags, then catches up; the masters do not lag).
The batch is the same every step (the net memorises it), so the loss falls and the updates stay aligned. A wrong
update (sign, scale, a missing layer, a stale weight copy) is off by >= 50 % of the update in every check.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SIZES = [1024, 4096, 4096, 1024]
MB, STEPS, LR = 512, 10, 0.1
EMUL_BOUND = 1e-2                     # check 1: update vs the bf16-emulating reference + BFP oracle
EMUL_LOSS = 1e-5
FP32_BOUND = 2.0 ** -5 + 2.0 ** -6    # checks 2 and 3: BFP rne worst case + bf16 roundings
UPDATE_NET_BOUND = 0.15
LOSS_SAME_WEIGHTS_REL = 1e-4


def _bf16(t):
    return t.to(torch.bfloat16).float()


def _fp32_step(W, b, x, y):
    """One fp32 autograd step from (W, b): (loss, per-layer update -lr [dW | db])."""
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


def _emul_step(W, b, x, y):
    """The HIP step's arithmetic in torch: bf16 rounding points as in models/mlp.py + csrc, BFP round trip by the
    oracle. Returns (loss, per-layer update -lr q([dW | db]))."""
    from fpga_ai_nic_amd.ops import bfp_oracle as O

    L = len(W)
    act = [x.float()]
    for i in range(L):
        z = act[i] @ W[i] + b[i]
        act.append(_bf16(torch.relu(z)) if i + 1 < L else z)  # logits stay f32
    logits = act[L]
    loss = F.cross_entropy(logits, y.long())
    p = torch.softmax(logits, dim=1)
    p[torch.arange(MB), y.long()] -= 1.0
    dz = _bf16(p / MB)
    ups = [None] * L
    for i in reversed(range(L)):
        dW = act[i].t() @ dz
        db = dz.sum(0)
        g = torch.cat([dW.flatten(), db]).cpu().numpy().astype(np.float32)
        ups[i] = -LR * torch.from_numpy(O.quantize(g, "bfp_rne")).to(x.device)
        if i > 0:
            dz = _bf16((dz @ W[i].t()) * (act[i] > 0))
    return float(loss), ups


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
    for l in m.layers:  # the f32 masters start at the bf16 values the HIP forward computes with
        l.master[: l.n].copy_(l.lp[: l.n].float())
    W0 = [l.w_master.clone() for l in m.layers]
    b0 = [l.b_master.clone() for l in m.layers]
    g = torch.Generator().manual_seed(11)
    x = (torch.rand(MB, SIZES[0], generator=g) * 2 - 1).to(dev, torch.bfloat16)
    y = torch.randint(0, SIZES[-1], (MB,), generator=g, dtype=torch.int32).to(dev)

    # 3. trajectory: 10 HIP steps vs 10 fp32 autograd + SGD steps from the same start
    hip_losses = []
    for _ in range(STEPS):
        hip_losses.append(float(tr.step(x, y).float().mean().item()))
    tr.finish()
    torch.cuda.synchronize()
    assert tr.fused_updates == STEPS * m.L
    Wr, br, ref_losses, path = [w.clone() for w in W0], [v.clone() for v in b0], [], [0.0] * m.L
    for _ in range(STEPS):
        rl, upd = _fp32_step(Wr, br, x, y)
        ref_losses.append(rl)
        for i in range(m.L):
            path[i] += float(upd[i].norm())
            k = Wr[i].numel()
            Wr[i] += upd[i][:k].view_as(Wr[i])
            br[i] += upd[i][k:]
    upd_net, upd_path = [], []
    for i, l in enumerate(m.layers):
        dh = torch.cat([(l.w_master - W0[i]).flatten(), l.b_master - b0[i]])
        dr = torch.cat([(Wr[i] - W0[i]).flatten(), br[i] - b0[i]])
        err = float((dh - dr).norm())
        upd_net.append(err / float(dr.norm()))
        upd_path.append(err / path[i])
    lag = [abs(a - b) - max(abs(ref_losses[max(t - 1, 0)] - ref_losses[t]), 1e-4 * b)
           for t, (a, b) in enumerate(zip(hip_losses, ref_losses))]

    # 1 + 2. three more HIP steps, each against both references from the model's current bf16 compute weights
    emul_err, emul_loss, fp32_err, fp32_loss = [], [], [], []
    for _ in range(3):
        Wm = [l.w_master.clone() for l in m.layers]
        bm = [l.b_master.clone() for l in m.layers]
        Wl = [l.w.float().clone() for l in m.layers]
        bl = [l.b.float().clone() for l in m.layers]
        el, eupd = _emul_step(Wl, bl, x, y)
        rl, rupd = _fp32_step(Wl, bl, x, y)
        hl = float(tr.step(x, y).float().mean().item())
        tr.finish()
        torch.cuda.synchronize()
        emul_loss.append(abs(hl - el) / el)
        fp32_loss.append(abs(hl - rl) / rl)
        for i, l in enumerate(m.layers):
            dh = torch.cat([(l.w_master - Wm[i]).flatten(), l.b_master - bm[i]])
            emul_err.append(float((dh - eupd[i]).norm() / eupd[i].norm()))
            fp32_err.append(float((dh - rupd[i]).norm() / rupd[i].norm()))

    print(f"\nloss hip {['%.5f' % v for v in hip_losses]}\nloss ref {['%.5f' % v for v in ref_losses]}\n"
          f"trajectory: update error / net update per layer {['%.4f' % v for v in upd_net]}; / update path length "
          f"{['%.4f' % v for v in upd_path]}\n"
          f"per step vs bf16-emulating reference + BFP oracle: update rel error {['%.2e' % v for v in emul_err]}, "
          f"loss {['%.1e' % v for v in emul_loss]}\n"
          f"per step vs fp32 autograd: update rel error {['%.4f' % v for v in fp32_err]}, "
          f"loss {['%.1e' % v for v in fp32_loss]}")
    assert all(math.isfinite(v) for v in hip_losses)
    assert ref_losses[-1] < ref_losses[0] - 0.01 and hip_losses[-1] < hip_losses[0] - 0.01, "loss did not fall"
    assert max(emul_err) <= EMUL_BOUND, emul_err
    assert max(emul_loss) <= EMUL_LOSS, emul_loss
    assert max(fp32_err) <= FP32_BOUND, fp32_err
    assert max(fp32_loss) <= LOSS_SAME_WEIGHTS_REL, fp32_loss
    assert max(upd_path) <= FP32_BOUND, upd_path
    assert max(upd_net) <= UPDATE_NET_BOUND, upd_net
    assert max(lag) <= 0, (lag, hip_losses, ref_losses)

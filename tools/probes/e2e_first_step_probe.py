"""Probe: the first training steps of the bf16 HIP MLP vs fp32 autograd, per layer (tests/test_gpu_e2e_numerics.py).

Prints, for fused / unfused update and GEMM tuning on / off, each step's loss and each layer's update error relative
to the fp32 reference's update of that step (both from the same weights each step: the reference is re-seeded from the
HIP weights before every step, so the per-step error does not accumulate)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.models.mlp import MLP  # noqa: E402
from fpga_ai_nic_amd.ops import gemm_tune  # noqa: E402
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import ThreadFabric  # noqa: E402

SIZES = [1024, 4096, 4096, 1024]
MB, LR, STEPS = 512, 0.1, 4


def ref_step(W, b, x, y):
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
    return float(loss), [torch.cat([(-LR * gs[i]).flatten(), -LR * gs[L + i]]) for i in range(L)]


def run(fused, tune):
    gemm_tune.reset(enabled=tune)
    dev = torch.device("cuda", 0)
    eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
    m = MLP(SIZES, dtype=torch.bfloat16, device=dev, seed=7, pad_fn=lambda n: eng.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=LR, fused_update=fused)
    for l in m.layers:
        l.master[: l.n].copy_(l.lp[: l.n].float())
    g = torch.Generator().manual_seed(11)
    x = (torch.rand(MB, SIZES[0], generator=g) * 2 - 1).to(dev, torch.bfloat16)
    y = torch.randint(0, SIZES[-1], (MB,), generator=g, dtype=torch.int32).to(dev)
    for s in range(STEPS):
        W = [l.w_master.clone() for l in m.layers]
        b = [l.b_master.clone() for l in m.layers]
        Wl = [l.w.float().clone() for l in m.layers]
        bl = [l.b.float().clone() for l in m.layers]
        rl, upd = ref_step(Wl, bl, x, y)
        hl = float(tr.step(x, y).float().mean())
        tr.finish()
        torch.cuda.synchronize()
        errs = []
        for i, l in enumerate(m.layers):
            dh = torch.cat([(l.w_master - W[i]).flatten(), l.b_master - b[i]])
            errs.append(float((dh - upd[i]).norm() / upd[i].norm()))
        print(f"fused={int(fused)} tune={int(tune)} step {s}: loss hip {hl:.5f} ref {rl:.5f}  update rel err per "
              f"layer {['%.4f' % e for e in errs]}", flush=True)


if __name__ == "__main__":
    for fused in (True, False):
        for tune in (True, False):
            run(fused, tune)

"""Row-panel split of the last-issued bucket (DataParallelTrainer ``panels``): layer 0's dW is computed in row panels,
each encoded straight into its chunk of the wire buffer and submitted as a request of its own while the next panel's
GEMM runs. N virtual ranks on one GPU (LoopbackFabric, one host thread and stream per rank): the split schedule
trains bit-identically to the unsplit schedule (the same panels submitted as ONE request of the same chunked
layout), the replicas stay bit-identical, and the loss goes down."""
import threading

import numpy as np
import pytest
import torch

from fpga_ai_nic_amd import _ext
from fpga_ai_nic_amd.models.mlp import MLP
from fpga_ai_nic_amd.ops import gemm_tune
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce

pytestmark = pytest.mark.gpu
SIZES = [256, 512, 256, 128]


def _train(N, submit, steps=3, momentum=False):
    C = _ext.require()
    fabric = C.LoopbackFabric(N, 60.0)
    engines = [NativeAllReduce(None, codec="bfp_rne", algo="mesh", comm=fabric.comm(r)) for r in range(N)]
    out, errs = [None] * N, [None] * N

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                eng = engines[r]
                m = MLP(SIZES, dtype=torch.bfloat16, device="cuda", seed=7, momentum=momentum,
                        pad_fn=lambda n: eng.layout(n).n_pad)
                tr = DataParallelTrainer(m, eng, lr=0.05, momentum=0.9 if momentum else 0.0, panels=4,
                                         panel_submit=submit)
                assert tr.panel_plans and tr.panel_plans[0]["chunks"] >= 2, tr.panel_plans
                g = torch.Generator().manual_seed(1000 + r)
                x = (torch.rand(128, SIZES[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
                y = torch.randint(0, SIZES[-1], (128,), generator=g, dtype=torch.int32).cuda()
                losses = [float(tr.step(x, y).float().mean().item()) for _ in range(steps)]
                tr.finish()
                s.synchronize()
                out[r] = (torch.cat([l.master[: l.n].cpu() for l in m.layers]).numpy(), losses,
                          len(eng.C.orders), eng.counters()["requests"])
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(180)
    assert not any(t.is_alive() for t in ts), "virtual rank thread hung"
    assert not any(errs), errs
    return out


@pytest.mark.parametrize("N", [2, 4, 8])
def test_panel_split_bit_identical_to_unsplit(N):
    gemm_tune.reset(enabled=False)  # static GEMM plans: both schedules run the same kernels
    try:
        split = _train(N, "split")
        whole = _train(N, "whole")
    finally:
        gemm_tune.reset()
    for r in range(N):
        assert np.array_equal(split[r][0], split[0][0]), f"replica {r} diverged (split)"
        assert np.array_equal(whole[r][0], whole[0][0]), f"replica {r} diverged (whole)"
    assert np.array_equal(split[0][0], whole[0][0]), "split schedule differs from the unsplit one"
    # 3 steps x (2 unsplit layers + 4 panels) vs 3 x (2 + 1) requests
    assert split[0][3] == 3 * 6 and whole[0][3] == 3 * 3, (split[0][3], whole[0][3])
    losses = split[0][1]
    assert np.all(np.isfinite(losses)) and losses[-1] < losses[0]


def test_panel_split_with_momentum_replicas_identical():
    gemm_tune.reset(enabled=False)
    try:
        out = _train(2, "split", steps=4, momentum=True)
    finally:
        gemm_tune.reset()
    assert np.array_equal(out[0][0], out[1][0])

"""mlp_mpi modes 'F' / 'B' (the reference's commented-out paths, sw:543-680) and the fuse_type -> epilogue
mapping (sw:479-489), on CPU."""
import io

import pytest
import torch

from fpga_ai_nic_amd.cli import mlp_mpi
from fpga_ai_nic_amd.models.mlp import MLP
from fpga_ai_nic_amd.utils import metrics

ARGS = ["32", "32", "32", "64", "96", "48", "--device", "cpu", "--dtype", "f32", "--warmup", "1"]


@pytest.mark.parametrize("kind,label", [("F", "PERFDUMP,FP,"), ("B", "PERFDUMP,BP,"), ("A", "PERFDUMP,BP,")])
def test_modes_report(kind, label):
    out = io.StringIO()
    mlp_mpi.run(["2", "16", "3", kind] + ARGS, out=out)
    text = out.getvalue()
    assert label in text
    g = float([l for l in text.splitlines() if l.startswith("GFLOP")][0].split("=")[1])
    assert g == pytest.approx(metrics.mlp_gflop([64, 96, 48], 16, kind), rel=1e-4)


def test_gflop_formulas():
    s, mb = [2048] * 3, 100
    f = 2 * mb * 2048 * 2048 / 1e9
    assert metrics.mlp_gflop(s, mb, "F") == pytest.approx(2 * f)
    assert metrics.mlp_gflop(s, mb, "B") == pytest.approx(2 * f + f)
    assert metrics.mlp_gflop(s, mb, "A") == pytest.approx(3 * f + 2 * f)


def _reference_forward(m: MLP, x):
    """Plain fp32 PyTorch forward with the model's epilogue settings."""
    h = x
    for i, l in enumerate(m.layers):
        h = h @ l.w_master + (l.b_master if m.bias else 0)
        if m._relu_at(i):
            h = torch.relu(h)
    return h


@pytest.mark.parametrize("bias,relu", [(False, "none"), (True, "none"), (False, "all"), (True, "all"),
                                       (True, "hidden")])
def test_fuse_variants_forward_and_grad(bias, relu):
    torch.manual_seed(0)
    m = MLP([16, 32, 8], dtype=torch.float32, seed=3, bias=bias, relu=relu)
    if not bias:
        assert all(torch.count_nonzero(l.b_master) == 0 for l in m.layers)
    x = torch.randn(12, 16)
    y = torch.randint(0, 8, (12,), dtype=torch.int32)
    logits = m.forward(x).clone()
    assert torch.allclose(logits, _reference_forward(m, x), atol=1e-5)
    # gradients vs autograd of the same network (mean softmax cross-entropy)
    ws = [l.w_master.clone().requires_grad_(True) for l in m.layers]
    bs = [l.b_master.clone().requires_grad_(True) for l in m.layers]
    h = x
    for i in range(m.L):
        h = h @ ws[i] + (bs[i] if bias else 0)
        if m._relu_at(i):
            h = torch.relu(h)
    torch.nn.functional.cross_entropy(h, y.long()).backward()
    m.loss_backward(y, grad_scale=1.0 / 12)
    for i in reversed(range(m.L)):
        m.backward_weight(i)
        m.backward_data(i)
    for i, l in enumerate(m.layers):
        assert torch.allclose(l.gw, ws[i].grad, atol=1e-5)
        if bias:
            assert torch.allclose(l.gb, bs[i].grad, atol=1e-5)
        else:
            assert torch.count_nonzero(l.gb) == 0


def test_check_env_and_norm_dumps(monkeypatch):
    monkeypatch.setenv("CHECK", "0")  # reference quirk: thread count printed only when CHECK is 0
    out = io.StringIO()
    mlp_mpi.run(["2", "16", "3", "A"] + ARGS + ["--dump-norms", "--verify-fwd"], out=out)
    text = out.getvalue()
    assert "Threads:" in text
    assert text.count("L1 of layer's") == 2
    line = [l for l in text.splitlines() if l.startswith("VERIFY fwd")][0]
    linf = float(line.split("linf_abs=")[1].split()[0])
    assert linf < 1e-4
    monkeypatch.setenv("CHECK", "1")
    out = io.StringIO()
    mlp_mpi.run(["1", "16", "3", "A"] + ARGS, out=out)
    assert "Threads:" not in out.getvalue()


def test_matdiff():
    import numpy as np

    r = np.array([1.0, -2.0, 3.0])
    d = metrics.matdiff(r, r + np.array([0.0, 0.5, 0.0]))
    assert d["l1_ref"] == 6.0 and d["linf_abs"] == 0.5 and abs(d["l2_rel"] - 0.5 / np.sqrt(14)) < 1e-12

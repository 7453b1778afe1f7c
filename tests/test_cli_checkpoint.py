"""mlp_mpi CLI (reference positional signature + report format) and checkpoint/resume."""
import io
import os

import numpy as np
import pytest
import torch

from fpga_ai_nic_amd.cli import mlp_mpi
from fpga_ai_nic_amd.models.mlp import MLP
from fpga_ai_nic_amd.utils import checkpoint, metrics


def test_cli_report_format(tmp_path):
    out = io.StringIO()
    ck = str(tmp_path / "ck")
    res = mlp_mpi.run(["3", "64", "0", "A", "32", "32", "32", "128", "256", "128", "--device", "cpu", "--dtype",
                       "f32", "--warmup", "1", "--profile", "--checkpoint", ck, "--metrics-jsonl",
                       str(tmp_path / "m.jsonl")], out=out)
    text = out.getvalue()
    for key in ("Setting Up (Common)", "PARAMS: N:64", "SIZE Filter       0 (128x256)", "GFLOP  =", "fp time =",
                "GFLOPS  =", "PERFDUMP,BP,", "SAMPLES/S =", "FC time compute/loss", "Bwdupd compute FIRST"):
        assert key in text, key
    perf = [l for l in text.splitlines() if l.startswith("PERFDUMP")][0].split(",")
    assert perf[4] == "64" and perf[5:7] == ["128", "256"]
    assert np.isfinite(res["loss"])
    assert os.path.exists(ck + ".safetensors") and os.path.exists(tmp_path / "m.jsonl")


def test_gflop_formula_matches_reference():
    # sw/mlp_mpi_example_f32.cpp:794-798 for the run.sh workload: 10 x 2048^2, global MB 5376
    g = metrics.mlp_gflop([2048] * 11, 5376)
    assert g == pytest.approx((9 * 6 + 4) * 5376 * 2048 * 2048 / 1e9)
    assert g == pytest.approx(1307.8, rel=1e-3)


def test_cli_rejects_bad_type():
    with pytest.raises(SystemExit):
        mlp_mpi.run(["1", "8", "0", "Z", "1", "1", "1", "16", "16", "--device", "cpu"])


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_checkpoint_roundtrip_reference_layout(tmp_path, dtype):
    m = MLP([64, 128, 32], dtype=torch.float32, seed=5)
    p = str(tmp_path / "c")
    checkpoint.save(p, m, iteration=7, dtype=dtype, meta={"bn": 32})
    # raw .bin image: layer 0 weight is C0 x C1 row-major, exactly the reference's fil_libxsmm[0]
    w0 = checkpoint.read_raw_layer(p, "fc0.weight")
    assert w0.shape == (64, 128)
    tol = 0 if dtype == "f32" else 1e-2
    assert np.abs(w0 - m.layers[0].w_master.numpy()).max() <= tol
    m2 = MLP([64, 128, 32], dtype=torch.float32, seed=99)
    info = checkpoint.load(p, m2)
    assert info["iteration"] == 7 and info["bn"] == 32
    assert torch.allclose(m2.layers[1].b_master, m.layers[1].b_master, atol=tol)


def test_resume_continues_training(tmp_path):
    ck = str(tmp_path / "r")
    r1 = mlp_mpi.run(["2", "32", "0", "A", "1", "1", "1", "64", "64", "--device", "cpu", "--dtype", "f32",
                      "--warmup", "0", "--checkpoint", ck], out=io.StringIO())
    r2 = mlp_mpi.run(["2", "32", "0", "A", "1", "1", "1", "64", "64", "--device", "cpu", "--dtype", "f32",
                      "--warmup", "0", "--resume", ck], out=io.StringIO())
    assert r2["loss"] < r1["loss"]

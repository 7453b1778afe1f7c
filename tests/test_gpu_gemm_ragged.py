"""MFMA GEMMs on shapes that are not multiples of the tile (edge tiles zero-filled from a zero page, predicated
stores): every operand layout, split-K (ragged K splits included), both dtypes, the fused epilogues — against an
fp64 reference of the same (bf16-rounded) inputs with a PER-ELEMENT bound.

Shapes: the reference workload's per-rank batch at 4 and 8 ranks (global MB 5376 / 4 = 1344, / 8 = 672,
sw/run.sh:16), its commented 448-row sweep (sw/run.sh:24-29) and widths that are not multiples of 128 (the
reference's libxsmm falls back to whole dimensions, sw/mlp_mpi_example_f32.cpp:498-506).

Bound: the kernels accumulate exact products in f32, so |C - C64| <= c * sum_k |a_mk b_kn| (c = 2e-5 covers
the f32 summation error with a wide margin at K <= 4096; a layout / indexing bug misplaces whole products and
breaks it by orders of magnitude); bf16 outputs add their rounding, 2^-8 relative."""
import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(Cout, ref, absprod, what, out_bf16=False):
    bound = 2e-5 * absprod + 1e-6
    if out_bf16:
        bound = bound + ref.abs() * 2.0 ** -8
    err = (Cout.double() - ref).abs()
    bad = (err > bound) | ~torch.isfinite(Cout.double())
    assert not bool(bad.any()), (f"{what}: {int(bad.sum())} elements out of bound, worst err "
                                 f"{float(err.max()):.3g} (bound there {float(bound.flatten()[int(err.argmax())]):.3g})")


def _operands(M, N, K, dt, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    A = torch.randn(M, K, generator=g).to(dt).to(DEV)
    B = torch.randn(K, N, generator=g).to(dt).to(DEV)
    ref = A.double() @ B.double()
    absprod = A.double().abs() @ B.double().abs()
    return A, B, ref, absprod


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M", [672, 1344, 1000])
def test_ragged_all_layouts(C, dt, M):
    for N in (1000, 2048):
        for K in (200, 672):
            A, B, ref, absprod = _operands(M, N, K, dt, M + N + K)
            for a_t in (False, True):
                for b_t in (False, True):
                    Ain = A.t().contiguous() if a_t else A
                    Bin = B.t().contiguous() if b_t else B
                    splits = (None, 1, 3)
                    for sk in splits:
                        Cout = torch.full((M, N), float("nan"), device=DEV)
                        G.gemm(Ain, a_t, Bin, b_t, Cout, split_k=sk)
                        _check(Cout, ref, absprod, f"{dt} M={M} N={N} K={K} a_t={a_t} b_t={b_t} split_k={sk}")


@pytest.mark.parametrize("tile", [(128, 128), (128, 256), (256, 128), (256, 256)])
def test_ragged_forced_tiles(C, tile):
    """Every tile shape on an edge in all three dimensions (M, N, K = 1000, 1000, 456: partial tiles in M and N,
    a partial last K-tile), split into 2 ragged K ranges as well."""
    M, N, K = 1000, 1000, 456
    A, B, ref, absprod = _operands(M, N, K, torch.bfloat16, 17)
    for a_t in (False, True):
        for b_t in (False, True):
            Ain = A.t().contiguous() if a_t else A
            Bin = B.t().contiguous() if b_t else B
            for sk in (1, 2):
                Cout = torch.full((M, N), float("nan"), device=DEV)
                G.gemm(Ain, a_t, Bin, b_t, Cout, split_k=sk, tile=tile)
                _check(Cout, ref, absprod, f"tile={tile} a_t={a_t} b_t={b_t} split_k={sk}")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_ragged_epilogues(C, dt):
    """Layer-shaped products of a 672-row batch through 1000-wide layers: forward with bias + ReLU, bwd-data with
    the ReLU mask, bwd-weight with the fused bias gradient (bf16) — every output element in range, nothing past
    the edge written."""
    MB, Cin, Cout_ = 672, 1000, 1000
    g = torch.Generator(device="cpu").manual_seed(3)
    X = torch.randn(MB, Cin, generator=g).to(dt).to(DEV)
    W = (torch.randn(Cin, Cout_, generator=g) / Cin ** 0.5).to(dt).to(DEV)
    b = torch.randn(Cout_, generator=g).to(dt).to(DEV)
    out_dt = dt
    # forward: relu(X W + b)
    Y = torch.full((MB + 8, Cout_), 7.0, device=DEV, dtype=out_dt)  # guard rows past the edge
    G.gemm(X, False, W, False, Y[:MB], G.EPI_BIAS_RELU, bias=b)
    ref = torch.relu(X.double() @ W.double() + b.double())
    absprod = X.double().abs() @ W.double().abs() + b.double().abs()
    _check(Y[:MB].float(), ref, absprod, "fwd bias+relu", out_bf16=out_dt == torch.bfloat16)
    assert torch.all(Y[MB:] == 7.0), "forward wrote past the edge"
    # bwd-data: (dZ W^T) * (act > 0)
    dZ = torch.randn(MB, Cout_, generator=g).to(dt).to(DEV)
    act = torch.randn(MB, Cin, generator=g).to(dt).to(DEV)
    dX = torch.empty(MB, Cin, device=DEV, dtype=out_dt)
    G.linear_bwd_data(dZ, W, dX, relu_input=act)
    ref = (dZ.double() @ W.double().t()) * (act.double() > 0)
    absprod = dZ.double().abs() @ W.double().abs().t()
    _check(dX.float(), ref, absprod, "bwd-data relu-mask", out_bf16=out_dt == torch.bfloat16)
    # bwd-weight: X^T dZ (+ bias gradient fused in bf16)
    dW = torch.empty(Cin, Cout_, device=DEV)
    db = torch.full((Cout_ + 8,), float("nan"), device=DEV)
    G.linear_bwd_weight(act, dZ, dW, bias_grad=db[:Cout_])
    ref = act.double().t() @ dZ.double()
    absprod = act.double().abs().t() @ dZ.double().abs()
    _check(dW, ref, absprod, "bwd-weight")
    _check(db[:Cout_], dZ.double().sum(0), dZ.double().abs().sum(0), "bias gradient")
    assert torch.isnan(db[Cout_:]).all(), "bias gradient written past the edge"


@pytest.mark.parametrize("in_dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Cc", [10, 1000, 1003])
def test_softmax_xent_any_width(C, in_dt, Cc):
    from fpga_ai_nic_amd.ops import nn as NN

    torch.manual_seed(Cc)
    M = 333
    x = (torch.randn(M, Cc, device=DEV) * 3).to(in_dt)
    y = torch.randint(0, Cc, (M,), device=DEV, dtype=torch.int32)
    d = torch.empty(M, Cc, device=DEV, dtype=torch.float32)
    loss = torch.empty(M, device=DEV)
    NN.softmax_xent(x, y, d, loss, 0.5)
    xf = x.double()
    ref_loss = torch.nn.functional.cross_entropy(xf, y.long(), reduction="none")
    assert (loss.double() - ref_loss).abs().max().item() < 1e-4 * (1 + ref_loss.abs().max().item())
    p = torch.softmax(xf, 1)
    p[torch.arange(M), y.long()] -= 1
    assert (d.double() - p * 0.5).abs().max().item() < 1e-5


@pytest.mark.parametrize("N", [10, 100, 1000, 1003])
def test_col_sum_any_width(C, N):
    from fpga_ai_nic_amd.ops import nn as NN

    torch.manual_seed(N)
    x = torch.randn(777, N, device=DEV)
    out = torch.full((N,), float("nan"), device=DEV)
    NN.col_sum(x, out, 1.0)
    ref = x.double().sum(0)
    assert (out.double() - ref).abs().max().item() < 1e-5 * x.abs().sum(0).max().item()


def test_mlp_mpi_reference_workload_per_rank_shape_f32(C):
    """The per-rank shape of the 8-GPU reference workload (global MB 5376 / 8 ranks = 672 rows, 10 x 2048 f32
    layers; sw/run.sh:16) trains on one GPU through the mlp_mpi entry point."""
    import io

    import numpy as np

    from fpga_ai_nic_amd.cli import mlp_mpi

    out = io.StringIO()
    res = mlp_mpi.run(["3", "672", "0", "A", "32", "32", "32"] + ["2048"] * 11 + ["--dtype", "f32", "--warmup", "1"],
                      out=out)
    assert "PERFDUMP,BP," in out.getvalue()
    assert np.isfinite(res["loss"])


def test_mlp_ragged_widths_bf16_trains(C):
    """A bf16 MLP whose widths and batch are not tile multiples (1000-wide layers, 10 classes, 448 rows) trains
    through the native engine: loss decreases over a few steps."""
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import ThreadFabric

    eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
    m = MLP([1000, 1000, 1000, 16], dtype=torch.bfloat16, device=DEV, seed=3, pad_fn=lambda n: eng.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=0.5)
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(448, 1000, generator=g) * 2 - 1).to(DEV, torch.bfloat16)
    y = torch.randint(0, 16, (448,), generator=g, dtype=torch.int32).to(DEV)
    losses = [tr.step(x, y).float().mean().item() for _ in range(8)]
    tr.finish()
    assert all(l == l for l in losses) and losses[-1] < losses[0]

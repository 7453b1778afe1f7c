"""1-bit ReLU masks (ops/gemm.py EPI_BIAS_RELU_BITS / EPI_RELU_BITS, csrc/gemm/gemm_bf16_kernel.h epi8_bf16): the
forward GEMM writes its ReLU output's mask bits beside the bf16 activation, the bwd-data GEMM reads them instead of
the activation. Both must be bit-identical to the activation-reading schedule (EPI_BIAS_RELU + EPI_RELU_MASK), on
every kernel the planner picks (256x256 persistent, 224x128, 128x128, the one-role kernel on a ragged shape), and a
training step of the MLP must not change (opt-in: FAN_RELU_BITS=1, measured slower on the flagship step)."""
import os

import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def test_mask_bits_shapes():
    """Whole-wave, unsplit static plans only (the MLP's 8192-row layers); others keep the activation (the 1792-row
    layers' plans are tuned on the device)."""
    assert G.mask_bits_supported(8192, 4096, 1024) and G.mask_bits_supported(8192, 4096, 4096)
    assert not G.mask_bits_supported(2048, 1024, 4096)  # 32 tiles: split-K
    assert not G.mask_bits_supported(8192, 4100, 1024)  # N % 8


@pytest.mark.parametrize("M,K,N", [(8192, 1024, 4096), (8192, 4096, 4096)])
def test_forward_bits_and_bwd_data_match_the_activation_schedule(M, K, N):
    torch.manual_seed(M + N)
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    G.linear_fwd(x, w, b, ref, relu=True)
    out = torch.full_like(ref, 3.0)
    bits = torch.full((M, N // 8), 0xA5, device="cuda", dtype=torch.uint8)
    assert G.mask_bits_supported(M, N, K)
    G.linear_fwd(x, w, b, out, relu=True, mask_out=bits)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(bits, G.pack_mask_bits(ref > 0))
    # bwd-data of the next layer (dX = dZ . W2^T masked by the activation)
    C2 = K  # (the MLP's next layer: a whole-wave unsplit bwd-data plan)
    dz = (torch.randn(M, C2, device="cuda") * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(N, C2, device="cuda") * N ** -0.5).to(torch.bfloat16)
    dref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    G.linear_bwd_data(dz, w2, dref, relu_input=ref)
    dx = torch.full_like(dref, 3.0)
    G.linear_bwd_data(dz, w2, dx, relu_bits=bits)
    torch.cuda.synchronize()
    assert torch.equal(dx, dref)


def test_mlp_step_identical_with_and_without_mask_bits(monkeypatch):
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import ThreadFabric

    res = {}
    for bits in ("0", "1"):
        monkeypatch.setenv("FAN_RELU_BITS", bits)
        torch.manual_seed(5)
        engine = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
        sizes = [1024, 4096, 4096, 1024]  # the flagship (whole-wave unsplit plans at 8192 rows)
        model = MLP(sizes, dtype=torch.bfloat16, device=torch.device("cuda"), pad_fn=lambda n: engine.layout(n).n_pad)
        tr = DataParallelTrainer(model, engine, lr=0.05)
        g = torch.Generator(device="cuda").manual_seed(9)
        x = torch.randn(8192, sizes[0], device="cuda", generator=g).to(torch.bfloat16)
        y = torch.randint(0, sizes[-1], (8192,), device="cuda", dtype=torch.int32, generator=g)
        for _ in range(3):
            tr.step(x, y)
        tr.finish()
        torch.cuda.synchronize()
        assert (model.mask[1] is not None) == (bits == "1") and (model.mask[2] is not None) == (bits == "1")
        res[bits] = [l.master.clone() for l in model.layers]
    for a, b in zip(res["0"], res["1"]):
        assert torch.equal(a, b)

"""The 256x256 persistent 4-wave GEMM loop on a ring of four 32-k half-stages (gemm_pl4h_kernel) against the
two-stage loop it replaces (gemm_pl4_kernel): the MFMAs run in the same k order, so every layout, epilogue, split-K
and the fused bias gradient must give the SAME BITS; and a few training steps of the flagship MLP (GEMM-encoded
wire + update fused into the bwd-weight epilogue) must leave bit-identical weights. Both loops are also checked
against an fp64 reference (bound as in tests/test_gpu_kernels.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def C():
    from fpga_ai_nic_amd import _ext

    C = _ext.require()
    saved = C.gemm_half_stage()
    yield C
    C.gemm_set_half_stage(saved)


def _both(C, fn):
    outs = []
    for half in (0, 1):
        C.gemm_set_half_stage(half)
        outs.append(fn())
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("a_t,b_t", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("K", [64, 192, 320, 1024])
@pytest.mark.parametrize("epi", ["none", "bias_relu", "relu_mask"])
def test_half_stage_loop_bit_identical(C, a_t, b_t, K, epi):
    from fpga_ai_nic_amd.ops import gemm as G

    M, N = 512, 768
    g = torch.Generator(device="cuda").manual_seed(K + 7 * a_t + 3 * b_t)
    A = (torch.rand(*((K, M) if a_t else (M, K)), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(*((N, K) if b_t else (K, N)), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    bias = (torch.rand(N, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
    aux = (torch.rand(M, N, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
    dt = torch.float32 if epi == "none" else torch.bfloat16
    e = {"none": G.EPI_NONE, "bias_relu": G.EPI_BIAS_RELU, "relu_mask": G.EPI_RELU_MASK}[epi]

    def run():
        out = torch.empty(M, N, device="cuda", dtype=dt)
        G.gemm(A, a_t, B, b_t, out, e, bias=bias if epi == "bias_relu" else None,
               aux=aux if epi == "relu_mask" else None, tile=(256, 256), split_k=1)
        return out

    o2, o4 = _both(C, run)
    assert torch.equal(o2, o4), (o2 - o4).abs().max()
    ref = (A.double().t() if a_t else A.double()) @ (B.double().t() if b_t else B.double())
    if epi == "bias_relu":
        ref = torch.relu(ref + bias.double())
    elif epi == "relu_mask":
        ref = ref * (aux.double() > 0)
    tol = 2e-2 * ref.abs().max().item() if dt == torch.bfloat16 else 1e-4 * ref.abs().max().item()
    assert (o4.double() - ref).abs().max().item() <= tol


@pytest.mark.parametrize("split_k", [1, 2])
def test_half_stage_split_k_and_bias_gradient_bit_identical(C, split_k):
    from fpga_ai_nic_amd.ops import gemm as G

    M, N, K = 512, 1024, 2048  # bwd-weight: X^T dZ, both operands MN-contiguous, with the fused column sum of dZ
    g = torch.Generator(device="cuda").manual_seed(5)
    X = (torch.rand(K, M, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    dZ = (torch.rand(K, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)

    def run():
        out = torch.empty(M, N, device="cuda")
        cs = torch.empty(N, device="cuda")
        G.gemm(X, True, dZ, False, out, G.EPI_NONE, colsum=cs, tile=(256, 256), split_k=split_k)
        return out, cs

    (o2, c2), (o4, c4) = _both(C, run)
    assert torch.equal(o2, o4) and torch.equal(c2, c4)
    assert torch.allclose(c4.double(), dZ.double().sum(0), rtol=1e-4, atol=1e-3)


def test_half_stage_training_bit_identical(C):
    """The flagship step (fwd bias+ReLU, bwd-data with the ReLU mask, bwd-weight with the wire encode and the
    update fused into its epilogue) trains to the same bits on either loop."""
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.ops import gemm_tune
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import ThreadFabric

    sizes = [1024, 2048, 2048, 512]
    g = torch.Generator().manual_seed(3)
    x = (torch.rand(1024, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    y = torch.randint(0, sizes[-1], (1024,), generator=g, dtype=torch.int32).cuda()
    weights = []
    gemm_tune.reset(enabled=False)  # the static plans on both runs (a timing-driven choice could differ)
    try:
        for half in (0, 1):
            C.gemm_set_half_stage(half)
            eng = make_engine(ThreadFabric(1).transport(0), "bfp", rounding="rne", impl="native")
            m = MLP(sizes, dtype=torch.bfloat16, device="cuda", seed=9, pad_fn=lambda n: eng.layout(n).n_pad)
            tr = DataParallelTrainer(m, eng, lr=0.05)
            for _ in range(3):
                tr.step(x, y)
            tr.finish()
            torch.cuda.synchronize()
            weights.append([l.master.clone() for l in m.layers])
    finally:
        gemm_tune.reset()
    for w2, w4 in zip(*weights):
        assert torch.equal(w2, w4)

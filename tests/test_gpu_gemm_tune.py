"""On-device GEMM plan tuner (fpga_ai_nic_amd/ops/gemm_tune.py): the first call of a shape times the candidate
plans in place and keeps the fastest; the result is the same product (vs an fp64 reference), later calls reuse the
decision, and calls that cannot be re-run (accumulate, output aliasing an input, HIP-graph capture) are never
tuned."""
import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import gemm_tune

pytestmark = pytest.mark.gpu


def _ref(A, B, a_t, b_t):
    a = (A.t() if a_t else A).double()
    b = (B.t() if b_t else B).double()
    return a @ b


@pytest.mark.parametrize("M,N,K,a_t,b_t", [(1792, 4096, 1024, False, False), (1792, 1024, 2048, False, True),
                                           (1024, 1536, 1792, True, False)])
def test_tuned_plan_same_product(M, N, K, a_t, b_t):
    T = gemm_tune.reset(enabled=True)
    torch.manual_seed(0)
    A = (torch.rand((K, M) if a_t else (M, K), device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand((N, K) if b_t else (K, N), device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda")
    G.gemm(A, a_t, B, b_t, C)
    torch.cuda.synchronize()
    assert len(T.log) == 1, "first call of a shape tunes it"
    d = T.log[0]
    assert d["chosen_us"] <= d["static_us"]
    err = (C.double() - _ref(A, B, a_t, b_t)).abs().max().item()
    assert err < 2e-2 * K ** 0.5 / 8, err
    C2 = torch.empty_like(C)
    G.gemm(A, a_t, B, b_t, C2)  # cached decision, same plan -> bit-identical
    torch.cuda.synchronize()
    assert len(T.log) == 1 and torch.equal(C, C2)


def test_whole_wave_static_plans_are_kept():
    """A static plan that fills whole waves of the 256 CUs (chosen by in-step A/B) is not re-tuned."""
    T = gemm_tune.reset(enabled=True)
    A = (torch.rand(8192, 1024, device="cuda") - 0.5).to(torch.bfloat16)
    B = (torch.rand(1024, 4096, device="cuda") - 0.5).to(torch.bfloat16)
    C = torch.empty(8192, 4096, device="cuda")
    G.gemm(A, False, B, False, C)  # 256x256 tiles: 512 workgroups = 2 waves
    torch.cuda.synchronize()
    assert T.log == [] and len(T.plans) == 1
    gemm_tune.reset()


def test_untunable_calls_use_the_static_plan():
    T = gemm_tune.reset(enabled=True)
    A = (torch.rand(1792, 1024, device="cuda") - 0.5).to(torch.bfloat16)
    B = (torch.rand(1024, 2048, device="cuda") - 0.5).to(torch.bfloat16)
    C = torch.zeros(1792, 2048, device="cuda")
    G.gemm(A, False, B, False, C, accumulate=True)  # C += A.B cannot be re-run
    G.gemm(A, False, B, False, C, split_k=1, tile=(128, 128))  # explicit plan
    torch.cuda.synchronize()
    assert T.log == []
    gemm_tune.reset(enabled=False)
    G.gemm(A, False, B, False, C)
    assert gemm_tune.tuner().log == []
    gemm_tune.reset()

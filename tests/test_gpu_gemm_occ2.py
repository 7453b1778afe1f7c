"""Two workgroups per CU (csrc/gemm/gemm_bf16_kernel.h gemm_pl2h_kernel, FAN_GEMM_OCC2 / C.gemm_set_occ2): the
unsplit 256x256 plans run as 256x128 tiles with two independent workgroups per CU. Same k order as the default
kernel: outputs bit-identical for every epilogue and layout it takes (forward bias + ReLU, bwd-data ReLU mask, plain
f32, persistent and one-tile-per-workgroup grids)."""
import pytest
import torch

from fpga_ai_nic_amd import _ext
from fpga_ai_nic_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,kind", [(8192, 4096, 1024, "fwd"), (8192, 4096, 4096, "bwdd"),
                                        (4096, 4096, 2048, "f32"), (2048, 2048, 512, "fwd")])
@pytest.mark.parametrize("persist", [256, 0])
def test_occ2_bit_identical(M, N, K, kind, persist):
    C = _ext.require()
    torch.manual_seed(M + N + K)
    A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    if kind == "bwdd":
        B = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)  # W [N][K]: K-contiguous B
        aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    else:
        B = (torch.randn(K, N, device="cuda") * K ** -0.5).to(torch.bfloat16)
    bias = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    odt = torch.float32 if kind == "f32" else torch.bfloat16

    def run():
        out = torch.full((M, N), 5.0, device="cuda", dtype=odt)
        if kind == "fwd":
            G.gemm(A, False, B, False, out, G.EPI_BIAS_RELU, bias=bias, tile=(256, 256), split_k=1)
        elif kind == "bwdd":
            G.gemm(A, False, B, True, out, G.EPI_RELU_MASK, aux=aux, tile=(256, 256), split_k=1)
        else:
            G.gemm(A, False, B, False, out, G.EPI_NONE, tile=(256, 256), split_k=1)
        torch.cuda.synchronize()
        return out

    saved = C.gemm_persist()
    try:
        C.gemm_set_persist(persist)
        C.gemm_set_occ2(0)
        ref = run()
        C.gemm_set_occ2(1)
        got = run()
    finally:
        C.gemm_set_occ2(0)
        C.gemm_set_persist(saved)
    assert torch.equal(got, ref)
    r = A.float() @ (B.float().t() if kind == "bwdd" else B.float())
    if kind == "fwd":
        r = torch.relu(r + bias.float())
    elif kind == "bwdd":
        r = r * (aux.float() > 0)
    assert (got.float() - r).abs().max() <= 2e-2 * r.abs().max() + 1e-3

"""Overlapped tile transitions of the persistent 256x256 GEMM (csrc/gemm/gemm_bf16_kernel.h pl4_run OVL,
FAN_GEMM_OVL / C.gemm_set_ovl): the epilogue stages through rows of its own, the next tile's first K-tiles are
fetched under the last k-step, and vmcnt waits let the epilogue's stores drain under the next tile. Same arithmetic:
bit-identical to the default kernel for the bf16 epilogues it takes, with 1, 2, 4 and uneven tile counts per
workgroup (persistent grid caps), and a K of exactly two K-tiles. (The transposed-accumulator epilogue and the
two-barrier DMA split that rode on this loop in round 5 measured no faster and were removed in round 6.)"""
import pytest
import torch

from fpga_ai_nic_amd import _ext
from fpga_ai_nic_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,kind,cap", [(8192, 4096, 1024, "fwd", 256), (8192, 4096, 4096, "bwdd", 256),
                                            (6144, 4096, 512, "fwd", 256), (4096, 4096, 128, "none", 64),
                                            (8192, 8192, 256, "bwdd", 256), (2048, 2048, 1024, "fwd", 24)])
def test_ovl_bit_identical(M, N, K, kind, cap):
    C = _ext.require()
    torch.manual_seed(M + N + K)
    A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    if kind == "bwdd":
        B = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    else:
        B = (torch.randn(K, N, device="cuda") * K ** -0.5).to(torch.bfloat16)
    bias = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)

    def run():
        out = torch.full((M, N), 5.0, device="cuda", dtype=torch.bfloat16)
        if kind == "fwd":
            G.gemm(A, False, B, False, out, G.EPI_BIAS_RELU, bias=bias, tile=(256, 256), split_k=1)
        elif kind == "bwdd":
            G.gemm(A, False, B, True, out, G.EPI_RELU_MASK, aux=aux, tile=(256, 256), split_k=1)
        else:
            G.gemm(A, False, B, False, out, G.EPI_NONE, tile=(256, 256), split_k=1)
        torch.cuda.synchronize()
        return out

    saved = C.gemm_persist(), C.gemm_ovl()
    try:
        C.gemm_set_persist(cap)
        C.gemm_set_ovl(0)
        ref = run()
        C.gemm_set_ovl(1)
        got = run()
        got2 = run()
    finally:
        C.gemm_set_persist(saved[0])
        C.gemm_set_ovl(saved[1])
    assert torch.equal(got, ref) and torch.equal(got2, ref)

"""CPU reference path of the GEMM epilogues (ops/gemm.py, the gloo / CPU training path)."""
import torch

from fpga_ai_nic_amd.ops import gemm as G


def test_cpu_epilogues_match_torch():
    torch.manual_seed(1)
    M, K, N = 32, 48, 64
    x, w, b = torch.randn(M, K), torch.randn(K, N), torch.randn(N)
    out = torch.empty(M, N)
    G.gemm(x, False, w, False, out, G.EPI_BIAS_RELU, bias=b)
    ref = torch.relu(x @ w + b)
    assert torch.allclose(out, ref)
    dz, w2 = torch.randn(M, 24), torch.randn(N, 24)
    d = torch.empty(M, N)
    G.gemm(dz, False, w2, True, d, G.EPI_RELU_MASK, aux=out)
    assert torch.allclose(d, (dz @ w2.t()) * (out > 0))


def test_wgrad_group_needs_gpu_bf16_shapes():
    x, y = torch.zeros(64, 256), torch.zeros(64, 128)
    assert not G.wgrad_group_supported([(x, y)])  # CPU f32 tensors: the grouped launch is a GPU kernel
    assert not G.wgrad_group_supported([])

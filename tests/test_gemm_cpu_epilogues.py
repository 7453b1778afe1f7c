"""CPU reference path of the GEMM epilogues (ops/gemm.py, the gloo / CPU training path) and the 1-bit ReLU mask
plane layout the GPU kernels share (bit n % 8 of byte n / 8, csrc/gemm/gemm_bf16_kernel.h epi8_bf16)."""
import torch

from fpga_ai_nic_amd.ops import gemm as G


def test_mask_bits_round_trip_and_layout():
    torch.manual_seed(0)
    m = torch.rand(7, 64) > 0.5
    bits = G.pack_mask_bits(m)
    assert bits.shape == (7, 8) and bits.dtype == torch.uint8
    assert torch.equal(G.unpack_mask_bits(bits, 64).bool(), m)
    # column 8k + j is bit j of byte k
    one = torch.zeros(1, 16, dtype=torch.bool)
    one[0, 11] = True
    assert G.pack_mask_bits(one).tolist() == [[0, 1 << 3]]


def test_cpu_bits_epilogues_match_the_activation_epilogues():
    torch.manual_seed(1)
    M, K, N = 32, 48, 64
    x, w, b = torch.randn(M, K), torch.randn(K, N), torch.randn(N)
    ref = torch.empty(M, N)
    G.gemm(x, False, w, False, ref, G.EPI_BIAS_RELU, bias=b)
    out, bits = torch.empty(M, N), torch.zeros(M, N // 8, dtype=torch.uint8)
    G.gemm(x, False, w, False, out, G.EPI_BIAS_RELU_BITS, bias=b, aux=bits)
    assert torch.equal(out, ref) and torch.equal(bits, G.pack_mask_bits(ref > 0))
    dz, w2 = torch.randn(M, 24), torch.randn(N, 24)
    d_ref, d_bits = torch.empty(M, N), torch.empty(M, N)
    G.gemm(dz, False, w2, True, d_ref, G.EPI_RELU_MASK, aux=ref)
    G.gemm(dz, False, w2, True, d_bits, G.EPI_RELU_BITS, aux=bits)
    assert torch.equal(d_ref, d_bits)


def test_wgrad_group_needs_gpu_bf16_shapes():
    x, y = torch.zeros(64, 256), torch.zeros(64, 128)
    assert not G.wgrad_group_supported([(x, y)])  # CPU f32 tensors: the grouped launch is a GPU kernel
    assert not G.wgrad_group_supported([])

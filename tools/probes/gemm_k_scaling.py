"""Probe: fixed vs per-K cost of the MFMA GEMM at the MLP's 8192 x 4096 output (what the K=1024 layers pay beyond
their main loop). Times M=8192, N=4096, K in {256 .. 4096} for the bf16-out bias+ReLU epilogue (fwd0), the ReLU-mask
epilogue (bwd-data of layer 2) and a plain f32-out product, next to torch.matmul, interleaved in one process on
random operands, and fits t(K) = fixed + K * per_k per arm (least squares): fixed is the tile prologue + epilogue +
launch cost the K=1024 layers cannot amortise."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402


def t_us(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    M, N = 8192, 4096
    Ks = [256, 512, 1024, 2048, 4096]
    torch.manual_seed(0)
    res = {}
    for K in Ks:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        Bt = B.t().contiguous()  # [N][K]: the bwd-data layout (both operands K-contiguous)
        bias = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16)
        aux = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16)
        Cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Cf = torch.empty(M, N, device="cuda", dtype=torch.float32)
        arms = {
            "bias_relu_bf16": lambda: G.gemm(A, False, B, False, Cb, G.EPI_BIAS_RELU, bias=bias),
            "relu_mask_bf16_nt": lambda: G.gemm(A, False, Bt, True, Cb, G.EPI_RELU_MASK, aux=aux),
            "plain_f32": lambda: G.gemm(A, False, B, False, Cf, G.EPI_NONE),
            "torch_matmul": lambda: torch.matmul(A, B),
            "torch_matmul_nt": lambda: torch.matmul(A, Bt.t()),
        }
        tm = {k: [] for k in arms}
        for _ in range(5):
            for k, fn in arms.items():
                tm[k].append(t_us(fn))
        res[K] = {k: statistics.median(v) for k, v in tm.items()}
        print(json.dumps({"K": K, **{k: round(v, 2) for k, v in res[K].items()},
                          "plan": G._ext.require().gemm_plan(M, N, K, 0)}), flush=True)
    for arm in res[Ks[0]]:
        xs, ys = Ks, [res[k][arm] for k in Ks]
        mx, my = statistics.mean(xs), statistics.mean(ys)
        b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        a = my - b * mx
        print(json.dumps({"arm": arm, "fixed_us": round(a, 2), "us_per_1k_K": round(b * 1024, 2),
                          "tflops_main_loop": round(2 * M * N * 1024 / (b * 1024) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

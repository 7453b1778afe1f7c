"""Probe: what the library's NT GEMM (both operands K-contiguous) does at the MLP's bwd-data shape that the pl4 kernel
does not — run under rocprofv3 --kernel-trace, the library kernel's name (macro tile, MFMA shape, wave layout, global
read / LDS options), grid, workgroup size, LDS and register counts land in the trace next to the pl4 kernel's.
M=8192 N=4096 K=4096 bf16, bf16 output, no epilogue on either side."""
import json
import os
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
    M, N, K = 8192, 4096, 4096
    torch.manual_seed(0)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    Bt = ((torch.rand(N, K, device="cuda") * 2 - 1)).to(torch.bfloat16)
    B = Bt.t().contiguous()
    Cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16)
    arms = {"pl4_nt": lambda: G.gemm(A, False, Bt, True, Cb, G.EPI_NONE),
            "pl4_nt_mask": lambda: G.gemm(A, False, Bt, True, Cb, G.EPI_RELU_MASK, aux=aux),
            "pl4_nn": lambda: G.gemm(A, False, B, False, Cb, G.EPI_NONE),
            "lib_nt": lambda: torch.matmul(A, Bt.t()),
            "lib_nn": lambda: torch.matmul(A, B)}
    res = {k: [] for k in arms}
    for _ in range(5):
        for k, fn in arms.items():
            res[k].append(t_us(fn))
    print(json.dumps({k: round(sorted(v)[2], 2) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()

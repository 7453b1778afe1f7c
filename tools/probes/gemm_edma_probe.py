"""Probe: the overlapped 256x256 loop with two barriers per K-tile and the operand DMA spread over both k-steps
(pl4_run EDMA, C.gemm_set_edma) against the one-barrier schedule, on the flagship's bf16 GEMM shapes (forward
bias+ReLU NN, bwd-data ReLU-mask NT; M=8192 N=4096, K 1024 and 4096), interleaved in one process, plus the library's
NT GEMM at the same shape for reference. Prints one JSON line per shape."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
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
    C = _ext.require()
    torch.manual_seed(0)
    M, N = 8192, 4096
    for K in (1024, 4096):
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = ((torch.rand(K, N, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        Bt = B.t().contiguous()
        bias = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16)
        aux = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        shapes = {"fwd_nn": lambda: G.gemm(A, False, B, False, out, G.EPI_BIAS_RELU, bias=bias),
                  "bwdd_nt": lambda: G.gemm(A, False, Bt, True, out, G.EPI_RELU_MASK, aux=aux)}
        res = {}
        for name, fn in shapes.items():
            tm = {0: [], 1: []}
            for _ in range(7):
                for e in (0, 1):
                    C.gemm_set_edma(e)
                    tm[e].append(t_us(fn))
            C.gemm_set_edma(0)
            res[name] = {"off": round(statistics.median(tm[0]), 2), "edma": round(statistics.median(tm[1]), 2)}
        res["lib_nt"] = round(statistics.median([t_us(lambda: torch.matmul(A, Bt.t())) for _ in range(5)]), 2)
        print(json.dumps({"M": M, "N": N, "K": K, **res}), flush=True)


if __name__ == "__main__":
    main()

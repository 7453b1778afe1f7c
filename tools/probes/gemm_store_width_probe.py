"""Probe: the bf16 GEMM epilogue's store width, A/B in one process. The epilogue writes 8 columns (16 B) per lane when
C, bias and the activation are 16-B aligned (store_tile, epi8_bf16) and 4 columns (8 B) otherwise; a C view offset
by 8 bytes forces the 8-B path with the same kernel, shape and operands. Also checks both paths give the same
bits. Shapes: the flagship's bf16-output GEMMs (fwd with bias + ReLU, bwd-data with the ReLU mask).
(Historical: the run in profiles/r4_gemm_store_width_ab.jsonl predates the removal of the 8-B path — keeping both
spilled VGPRs — so today a misaligned C is staged through an aligned copy by ops/gemm.py and "us_8B" times that.)"""
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
    torch.manual_seed(0)
    M = 8192
    cases = [("fwd_bias_relu", 4096, 1024), ("fwd_bias_relu", 4096, 4096), ("bwdd_relu_mask", 4096, 4096),
             ("bwdd_relu_mask", 4096, 1024)]
    for name, N, K in cases:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        if name.startswith("fwd"):
            B = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)
            bias = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16)
            run = lambda C: G.gemm(A, False, B, False, C, G.EPI_BIAS_RELU, bias=bias)  # noqa: E731
        else:
            B = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)  # W stored [N][K]: the NT layout
            aux = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16)
            run = lambda C: G.gemm(A, False, B, True, C, G.EPI_RELU_MASK, aux=aux)  # noqa: E731
        buf = torch.empty(M * N + 8, device="cuda", dtype=torch.bfloat16)
        C16 = buf[:M * N].view(M, N)      # 16-B aligned: 8 columns per store
        C8 = buf[4:4 + M * N].view(M, N)  # 8-B offset: the 4-column path
        run(C16)
        ref = C16.clone()
        run(C8)
        same = bool(torch.equal(C8, ref))
        w, n = [], []
        for _ in range(5):
            w.append(t_us(lambda: run(C16)))
            n.append(t_us(lambda: run(C8)))
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "us_16B": round(statistics.median(w), 2),
                          "us_8B": round(statistics.median(n), 2), "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()

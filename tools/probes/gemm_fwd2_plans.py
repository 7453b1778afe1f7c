"""Probe: the flagship's classifier forward (8192 x 1024 x 4096, f32 out + bias) and the other whole-wave shapes the
tuner keeps static (worth_tuning: only partial last waves are tuned): every candidate plan, timed in place."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402
from fpga_ai_nic_amd.ops import gemm_tune  # noqa: E402


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
    Cx = _ext.require()
    T = gemm_tune.tuner()
    torch.manual_seed(0)
    cases = [("fwd2_bias_f32", 8192, 1024, 4096, False, False, G.EPI_BIAS, torch.float32),
             ("fwd0_bias_relu", 8192, 4096, 1024, False, False, G.EPI_BIAS_RELU, torch.bfloat16),
             ("bwdd2_relu_mask_nt", 8192, 4096, 1024, False, True, G.EPI_RELU_MASK, torch.bfloat16)]
    for name, M, N, K, a_t, b_t, epi, odt in cases:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(*((N, K) if b_t else (K, N)), device="cuda") * 2 - 1).to(torch.bfloat16)
        bias = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16)
        aux = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=odt)
        static = tuple(Cx.gemm_plan(M, N, K, 0, 0, 0, 0))[:3]
        res = {}
        for bm, bn, sk in T.candidates(Cx, M, N, K, a_kcontig=True, colsum=False):
            fn = lambda: G.gemm(A, False, B, b_t, C, epi, bias=bias if epi in (G.EPI_BIAS, G.EPI_BIAS_RELU) else None,  # noqa: E731
                                aux=aux if epi == G.EPI_RELU_MASK else None, tile=(bm, bn), split_k=sk)
            res[f"{bm}x{bn}/sk{sk}"] = round(statistics.median(t_us(fn) for _ in range(5)), 2)
        best = min(res, key=res.get)
        print(json.dumps({"gemm": name, "static": "%dx%d/sk%d" % static, "static_us": res.get("%dx%d/sk%d" % static),
                          "best": best, "best_us": res[best], "plans": res}), flush=True)


if __name__ == "__main__":
    main()

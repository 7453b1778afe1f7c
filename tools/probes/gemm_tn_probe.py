"""Probe: the bwd-weight (TN) GEMMs of the flagship, dW = X^T dZ with the batch (8192) as the reduction dimension and
both operands MN-contiguous, per tile / split-K plan, against torch.matmul on the same operands. Shapes (M = fan-in,
N = fan-out): 4096x4096 (layer 1), 1024x4096 (layer 0), 4096x1024 (layer 2); plus K-scaling of 4096x4096 (fixed vs
per-K cost). One JSON line per shape: us per plan, the static plan, torch's us."""
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


def med(fn, reps=5):
    return statistics.median(t_us(fn) for _ in range(reps))


def main():
    Cx = _ext.require()
    torch.manual_seed(0)
    shapes = [(4096, 4096, 8192), (1024, 4096, 8192), (4096, 1024, 8192),
              (4096, 4096, 2048), (4096, 4096, 4096), (4096, 4096, 16384)]
    T = gemm_tune.tuner()
    for M, N, K in shapes:
        X = (torch.rand(K, M, device="cuda") * 2 - 1).to(torch.bfloat16)   # activations [batch][fan-in]
        dZ = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)  # [batch][fan-out]
        C = torch.empty(M, N, device="cuda", dtype=torch.float32)
        cs = torch.empty(N, device="cuda", dtype=torch.float32)
        static = tuple(Cx.gemm_plan(M, N, K, 0, 0, 0, 0))[:3]
        plans = T.candidates(Cx, M, N, K, a_kcontig=False, colsum=True)
        res = {}
        for p in plans:
            bm, bn, sk = p
            res[f"{bm}x{bn}/sk{sk}"] = round(med(lambda: G.gemm(X, True, dZ, False, C, G.EPI_NONE, tile=(bm, bn),
                                                                 split_k=sk, colsum=cs)), 2)
        tm = round(med(lambda: torch.matmul(X.t(), dZ)), 2)
        best = min(res, key=res.get)
        fl = 2.0 * M * N * K
        print(json.dumps({"M": M, "N": N, "K": K, "static": "%dx%d/sk%d" % static, "best": best,
                          "best_us": res[best], "static_us": res.get("%dx%d/sk%d" % static),
                          "torch_us": tm, "best_tflops": round(fl / res[best] / 1e6, 1),
                          "torch_tflops": round(fl / tm / 1e6, 1), "plans": res}), flush=True)


if __name__ == "__main__":
    main()

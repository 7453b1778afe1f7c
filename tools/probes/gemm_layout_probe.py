"""Probe: the MFMA GEMM's four operand layouts on the same FLOPs. For each shape (M, N, K) and each (a_t, b_t), time
C[M][N] (f32) = op(A) op(B) with the 256x256 single-pass plan, next to torch.matmul on the same operand views.
a_t: A stored [K][M] (MN-contiguous, the bwd-weight X); b_t: B stored [N][K] (K-contiguous, the bwd-data W).
Separates "the TN main loop is slower" from "this shape is slower"."""
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
    quick = "--quick" in sys.argv  # counter passes: one shape, NN and TN only, few launches, no torch.matmul
    shapes = [(4096, 4096, 8192)] if quick else [(4096, 4096, 8192), (8192, 4096, 4096), (4096, 4096, 4096)]
    for M, N, K in shapes:
        out = {"M": M, "N": N, "K": K}
        C = torch.empty(M, N, device="cuda", dtype=torch.float32)
        for a_t in (False, True):
            for b_t in ((False,) if quick else (False, True)):
                A = (torch.rand(*((K, M) if a_t else (M, K)), device="cuda") * 2 - 1).to(torch.bfloat16)
                B = (torch.rand(*((N, K) if b_t else (K, N)), device="cuda") * 2 - 1).to(torch.bfloat16)
                Av = A.t() if a_t else A
                Bv = B.t() if b_t else B
                reps = 1 if quick else 5
                ours = statistics.median(t_us(lambda: G.gemm(A, a_t, B, b_t, C, G.EPI_NONE, tile=(256, 256),
                                                             split_k=1), 3 if quick else 20) for _ in range(reps))
                tm = 0.0 if quick else statistics.median(t_us(lambda: torch.matmul(Av, Bv)) for _ in range(5))
                tag = ("T" if a_t else "N") + ("T" if b_t else "N")
                out[tag] = {"us": round(ours, 2), "torch_us": round(tm, 2),
                            "tflops": round(2.0 * M * N * K / ours / 1e6, 1)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

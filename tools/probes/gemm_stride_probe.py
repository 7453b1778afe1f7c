"""Probe: does the operands' row stride change the 256x256 main loop's speed? At the MLP's shapes every K-contiguous
operand row is 8 KiB (K = 4096 bf16), so in one K-tile every workgroup reads the same 128-B column slice of its rows:
addresses equal modulo 8 KiB. If the L2 channel selection leaves such addresses on few channels, rows padded by a
few cache lines spread them and the loop gets faster. Arms (M=8192 N=4096 K=4096 and K=1024, bf16 out): our NT
(bwd-data layout) and NN (forward layout) with row pitches padded by 0 / 64 / 128 / 256 elements, and the library's
NT kernel (torch.matmul) for reference. Interleaved, median of 5 x 20 launches, us."""
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


def padded(rows, cols, pad):
    t = ((torch.rand(rows, cols + pad, device="cuda") * 2 - 1)).to(torch.bfloat16)
    return t[:, :cols]


def main():
    torch.manual_seed(0)
    M, N = 8192, 4096
    out = []
    for K in (4096, 1024):
        arms = {}
        for pad in (0, 64, 128, 256):
            A = padded(M, K, pad)          # [M][K] K-contiguous
            Bt = padded(N, K, pad)         # [N][K] K-contiguous (NT)
            B = padded(K, N, pad)          # [K][N] N-contiguous (NN)
            C = torch.empty(M, N + pad, device="cuda", dtype=torch.bfloat16)[:, :N]
            arms[f"nt_pad{pad}"] = (lambda A=A, Bt=Bt, C=C: G.gemm(A, False, Bt, True, C, G.EPI_NONE))
            arms[f"nn_pad{pad}"] = (lambda A=A, B=B, C=C: G.gemm(A, False, B, False, C, G.EPI_NONE))
        A0 = padded(M, K, 0)
        Bt0 = padded(N, K, 0)
        arms["lib_nt"] = lambda: torch.matmul(A0, Bt0.t())
        res = {k: [] for k in arms}
        for _ in range(5):
            for k, fn in arms.items():
                res[k].append(t_us(fn))
        rec = {"M": M, "N": N, "K": K, **{k: round(sorted(v)[2], 2) for k, v in res.items()}}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    path = os.environ.get("PROBE_OUT")
    if path:
        with open(path, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()

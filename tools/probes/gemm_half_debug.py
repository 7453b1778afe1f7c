"""Debug probe for the half-stage GEMM loop: one 256x256 tile, K = 64 / 128, compares against fp64 partial
products to see which part of the result is wrong."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402

C = _ext.require()
torch.manual_seed(0)
for K in (64, 128):
    for a_t, b_t in ((False, False), (False, True)):
        M = N = 256
        A = (torch.rand(*((K, M) if a_t else (M, K)), device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(*((N, K) if b_t else (K, N)), device="cuda") * 2 - 1).to(torch.bfloat16)
        Ad = (A.double().t() if a_t else A.double())
        Bd = (B.double().t() if b_t else B.double())
        ref = Ad @ Bd
        outs = {}
        for half in (0, 1):
            C.gemm_set_half_stage(half)
            o = torch.zeros(M, N, device="cuda")
            G.gemm(A, a_t, B, b_t, o, G.EPI_NONE, tile=(256, 256), split_k=1)
            torch.cuda.synchronize()
            outs[half] = o.double()
        e0 = (outs[0] - ref).abs().max().item()
        e1 = (outs[1] - ref).abs()
        print(f"K={K} a_t={a_t} b_t={b_t}: pl4 err {e0:.2e}, pl4h err {e1.max().item():.2e}", flush=True)
        # per 16x16 block max error of pl4h
        blk = e1.view(16, 16, 16, 16).amax(dim=(1, 3))
        print("  wrong 16x16 blocks:", int((blk > 1e-3).sum().item()), "of 256", flush=True)
        print("  block err rows 0..15 (col block 0..15):")
        for i in range(16):
            print("   ", " ".join("x" if v > 1e-3 else "." for v in blk[i].tolist()))
        # candidate: only one k half accumulated
        for nm, (k0, k1) in {"k0-31": (0, 32), "k32-63": (32, 64)}.items():
            part = Ad[:, k0:k1] @ Bd[k0:k1, :]
            print(f"  vs {nm} only: {(outs[1] - part).abs().max().item():.2e}", flush=True)
        # candidate: k halves of A swapped relative to B
        if K == 64:
            sw = Ad[:, 32:64] @ Bd[0:32, :] + Ad[:, 0:32] @ Bd[32:64, :]
            print(f"  vs swapped halves: {(outs[1] - sw).abs().max().item():.2e}", flush=True)

"""Probe: one layer's bwd-data + bwd-weight as ONE grouped dispatch (gemm_bwd_pair: workgroups [0, g0) run the
bwd-data tiles, [g0, g0 + g1) the bwd-weight tiles) vs the two GEMMs back to back, at the flagship's MB 8192 shapes.
Checks the grouped results bit-identical to the separate launches of the same tiles, then times (median of 5 x 20
launches, interleaved)."""
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
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    C = _ext.require()
    M = 8192
    torch.manual_seed(0)
    dev = "cuda"
    out = []
    for name, cin, cout, cfgs in (  # cfgs: (bwd-weight tile width, bwd-data workgroups, bwd-weight workgroups)
            ("layer2", 4096, 1024, [(128, 128, 128), (128, 160, 96), (128, 96, 160), (256, 192, 64)]),
            ("layer1", 4096, 4096, [(256, 128, 128), (128, 128, 128), (256, 120, 136), (256, 136, 120),
                                    (128, 112, 144)])):
        X = (torch.rand(M, cin, device=dev) * 2 - 1).to(torch.bfloat16)
        dZ = ((torch.rand(M, cout, device=dev) * 2 - 1) * 0.01).to(torch.bfloat16)
        W = ((torch.rand(cin, cout, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16)
        dX = torch.empty(M, cin, device=dev, dtype=torch.bfloat16)
        dW = torch.empty(cin, cout, device=dev, dtype=torch.float32)
        dX2 = torch.empty_like(dX)
        dW2 = torch.empty_like(dW)

        def bd():
            G.gemm(dZ, False, W, True, dX, G.EPI_RELU_MASK, aux=X, tile=(256, 256), split_k=1)

        arms = {"bd": bd}
        for bn in (256, 128):
            arms[f"bw{bn}"] = (lambda bn=bn: G.gemm(X, True, dZ, False, dW, G.EPI_NONE, tile=(256, bn), split_k=1))
        arms["bw_default"] = lambda: G.gemm(X, True, dZ, False, dW, G.EPI_NONE)
        arms["seq_default"] = lambda: (bd(), arms["bw_default"]())
        for bn, g0, g1 in cfgs:
            arms[f"pair_bw{bn}_{g0}_{g1}"] = (lambda bn=bn, g0=g0, g1=g1: C.gemm_bwd_pair(dZ, W, X, dX2, dW2, bn, g0, g1))
        # exactness: grouped vs separate launches of the same tiles
        exact = {}
        for bn, g0, g1 in cfgs:
            bd()
            G.gemm(X, True, dZ, False, dW, G.EPI_NONE, tile=(256, bn), split_k=1)
            dX2.zero_()
            dW2.zero_()
            C.gemm_bwd_pair(dZ, W, X, dX2, dW2, bn, g0, g1)
            torch.cuda.synchronize()
            exact[f"{bn}_{g0}_{g1}"] = bool(torch.equal(dX, dX2) and torch.equal(dW, dW2))
        tm = {k: [] for k in arms}
        for _ in range(5):
            for k, fn in arms.items():
                tm[k].append(t_us(fn))
        rec = {"layer": name, "M": M, "cin": cin, "cout": cout, "exact": exact,
               **{k: round(statistics.median(v), 2) for k, v in tm.items()}}
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()

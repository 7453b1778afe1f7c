"""Layer-chain GEMM vs per-GEMM launches on the flagship forward / backward-data shapes (tools for docs/ROUND6.md).

Times (CUDA events, median of rounds, each round `iters` back-to-back passes): the per-GEMM launches of the same tiles,
the whole chain, and one-stage chains (the chain machinery without hand-offs: dynamic tickets, panel order). Env
switches of the chain launcher (FAN_CHAIN_ACQ / FAN_CHAIN_ORDER / FAN_CHAIN_ASC1) are read once per process, so the
variants run as separate invocations: python tools/probes/chain_probe.py [--label x] >> out.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
os.environ["FAN_GEMM_CHAIN"] = "1"

import torch  # noqa: E402

from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20, rounds=7):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) * 1000 / iters)
    return round(statistics.median(out), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="default")
    ap.add_argument("--mb", type=int, default=8192)
    a = ap.parse_args()
    M, sizes = a.mb, [1024, 4096, 4096, 1024]
    torch.manual_seed(0)
    x = (torch.randn(M, sizes[0], device="cuda") * 0.5).to(torch.bfloat16)
    ws = [(torch.randn(i, o, device="cuda") * i ** -0.5).to(torch.bfloat16) for i, o in zip(sizes[:-1], sizes[1:])]
    bs = [(torch.randn(o, device="cuda") * 0.1).to(torch.bfloat16) for o in sizes[1:]]
    outs = [torch.empty(M, 4096, device="cuda", dtype=torch.bfloat16),
            torch.empty(M, 4096, device="cuda", dtype=torch.bfloat16), torch.empty(M, 1024, device="cuda")]
    epis = [G.EPI_BIAS_RELU, G.EPI_BIAS_RELU, G.EPI_BIAS]
    tiles = [(256, 256), (256, 256), (256, 128)]
    ins = [x, outs[0], outs[1]]
    rec = {"label": a.label, "M": M, "env": {k: v for k, v in os.environ.items() if k.startswith("FAN_CHAIN")}}

    def per_gemm(idx):
        def f():
            for i in idx:
                G.gemm(ins[i], False, ws[i], False, outs[i], epis[i], bias=bs[i], tile=tiles[i], split_k=1)
        return f

    def chain(idx, key):
        def f():
            assert G.linear_chain(G.CHAIN_FWD, ins[idx[0]], [ws[i] for i in idx], [outs[i] for i in idx],
                                  biases=[bs[i] for i in idx], epis=[epis[i] for i in idx], key=key)
        return f

    rec["fwd_per_gemm_us"] = [timeit(per_gemm([i])) for i in range(3)]
    rec["fwd_per_gemm_sum_us"] = timeit(per_gemm([0, 1, 2]))
    rec["fwd_chain_us"] = timeit(chain([0, 1, 2], "p3"))
    rec["fwd_chain_1stage_us"] = [timeit(chain([i], f"p1_{i}")) for i in range(3)]
    rec["fwd_chain_2stage_01_us"] = timeit(chain([0, 1], "p01"))
    # backward data: dH2 = dY . W3^T (mask H2), dH1 = dH2 . W2^T (mask H1)
    dy = (torch.randn(M, 1024, device="cuda") * 0.1).to(torch.bfloat16)
    d2, d1 = torch.empty(M, 4096, device="cuda", dtype=torch.bfloat16), torch.empty(M, 4096, device="cuda",
                                                                                      dtype=torch.bfloat16)

    def bwd_per():
        G.gemm(dy, False, ws[2], True, d2, G.EPI_RELU_MASK, aux=outs[1], tile=(256, 256), split_k=1)
        G.gemm(d2, False, ws[1], True, d1, G.EPI_RELU_MASK, aux=outs[0], tile=(256, 256), split_k=1)

    def bwd_chain():
        assert G.linear_chain(G.CHAIN_BWD_DATA, dy, [ws[2], ws[1]], [d2, d1], auxes=[outs[1], outs[0]], key="pb")

    rec["bwd_per_gemm_us"] = timeit(bwd_per)
    rec["bwd_chain_us"] = timeit(bwd_chain)
    rec["chain_error"] = G.chain_error()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

"""Persistent 4-wave GEMM (grid capped at one workgroup per CU, each looping over its tiles) vs one workgroup per
tile, on the MLP's 2-round shapes at MB 8192 (8192x4096 outputs: 512 tiles of 256x256) and the 1-round ones.
One process, arms interleaved per round, median of rounds."""
from __future__ import annotations

import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402


def t(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    Cx = G._ext.require()
    mb, bf = 8192, torch.bfloat16
    shapes = [("fwd0", mb, 4096, 1024, False, G.EPI_BIAS_RELU), ("fwd1", mb, 4096, 4096, False, G.EPI_BIAS_RELU),
              ("bwdd1", mb, 4096, 4096, True, G.EPI_RELU_MASK), ("bwdd2", mb, 4096, 1024, True, G.EPI_RELU_MASK),
              ("fwd2", mb, 1024, 4096, False, G.EPI_BIAS)]
    cap0 = Cx.gemm_persist()
    for name, M, N, K, b_t, epi in shapes:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(bf)
        B = ((torch.rand(N, K, device="cuda") if b_t else torch.rand(K, N, device="cuda")) * 2 - 1).to(bf)
        C = torch.empty(M, N, device="cuda", dtype=bf)
        kw = {"bias": (torch.rand(N, device="cuda") - 0.5).to(bf)} if epi != G.EPI_RELU_MASK else \
            {"aux": (torch.rand(M, N, device="cuda") - 0.5).to(bf)}
        res = {}
        for _ in range(7):
            for cap in (256, 0):
                Cx.gemm_set_persist(cap)
                res.setdefault(cap, []).append(t(lambda: G.gemm(A, False, B, b_t, C, epi, **kw)))
        Cx.gemm_set_persist(cap0)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "plan": Cx.gemm_plan(M, N, K, 0),
                          "persistent_us": round(statistics.median(res[256]), 2),
                          "one_wg_per_tile_us": round(statistics.median(res[0]), 2)}), flush=True)


if __name__ == "__main__":
    main()

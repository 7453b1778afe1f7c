#!/usr/bin/env python3
"""GEMM micro-benchmark: the framework's MFMA kernels vs torch.matmul (hipBLASLt) on the MLP's shapes.

Interleaved rounds in one process (guide §5.4 rule 24), random operands (rule 25), median of rounds.
Prints one JSON line per shape.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402

def mlp_shapes(mb: int):
    """(name, M, N, K, a_t, b_t, epilogue) of one MLP 1024-4096-4096-1024 step at minibatch ``mb``."""
    return [
        ("fwd0", mb, 4096, 1024, False, False, G.EPI_BIAS_RELU),
        ("fwd1", mb, 4096, 4096, False, False, G.EPI_BIAS_RELU),
        ("fwd2", mb, 1024, 4096, False, False, G.EPI_BIAS),
        ("bwdw2", 4096, 1024, mb, True, False, G.EPI_NONE),
        ("bwdw1", 4096, 4096, mb, True, False, G.EPI_NONE),
        ("bwdw0", 1024, 4096, mb, True, False, G.EPI_NONE),
        ("bwdd2", mb, 4096, 1024, False, True, G.EPI_RELU_MASK),
        ("bwdd1", mb, 4096, 4096, False, True, G.EPI_RELU_MASK),
        ("sq4k", 4096, 4096, 4096, False, True, G.EPI_NONE),
        ("sq8k", 8192, 8192, 8192, False, True, G.EPI_NONE),
    ]


MLP_SHAPES = mlp_shapes(2048)


def ref_shapes(mb: int = 5376, c: int = 2048):
    """The reference run.sh workload (10 x 2048^2 f32 FC layers, MB 5376): one layer's three GEMMs, plus the
    same products with every operand K-contiguous (what a transposed-weight path would run)."""
    return [
        ("ref_fwd", mb, c, c, False, False, G.EPI_NONE),
        ("ref_bwdd", mb, c, c, False, True, G.EPI_NONE),
        ("ref_bwdw", c, c, mb, True, False, G.EPI_NONE),
        ("ref_fwd_kk", mb, c, c, False, True, G.EPI_NONE),
        ("ref_bwdw_kk", c, c, mb, False, True, G.EPI_NONE),
    ]


def ragged_shapes():
    """Shapes that are not tile multiples: the reference workload's per-rank batch at 8 / 4 ranks (global MB 5376,
    sw/run.sh:16) and its 448-row sweep (sw/run.sh:24-29) on 2048-wide layers, plus 1000-wide layers."""
    out = []
    for mb in (672, 1344, 448):
        out += [(f"r{mb}_fwd", mb, 2048, 2048, False, False, G.EPI_NONE),
                (f"r{mb}_bwdd", mb, 2048, 2048, False, True, G.EPI_NONE),
                (f"r{mb}_bwdw", 2048, 2048, mb, True, False, G.EPI_NONE)]
    out += [("w1000_fwd", 8192, 1000, 1000, False, False, G.EPI_NONE),
            ("w1000_bwdw", 1000, 1000, 8192, True, False, G.EPI_NONE)]
    return out


def bert_shapes(tokens: int):
    """BERT-base encoder-layer backward GEMMs (BASELINE config 5) at ``tokens`` rows per GPU."""
    import sys as _s
    import os as _o
    _s.path.insert(0, _o.path.dirname(_o.path.dirname(_o.path.abspath(__file__))))
    from fpga_ai_nic_amd.models import bert

    return [(name, M, N, K, a_t, b_t, G.EPI_NONE) for name, M, N, K, a_t, b_t in bert.layer_backward_gemms(tokens)]


def time_fn(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--shapes", default="")
    ap.add_argument("--sweep", action="store_true", help="time every tile/split-K plan per shape")
    ap.add_argument("--sweep-wire", action="store_true",
                    help="bwd-weight shapes: sweep with the BFP wire epilogue the training step runs (split plans then "
                         "include splitk_reduce_wire instead of the f32 reduce)")
    ap.add_argument("--mb", type=int, default=2048, help="MLP minibatch of the shape set")
    ap.add_argument("--set", default="mlp", choices=["mlp", "bert", "ref", "ragged"])
    ap.add_argument("--loops", default="",
                    help="also time these 256x256 main loops (0 one-role, 1 staggered, 2 pipelined), e.g. 0,2")
    ap.add_argument("--epi-arms", action="store_true",
                    help="bwd-weight shapes: also time the fused bias-gradient (colsum) and BFP wire epilogues")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    shapes = (mlp_shapes(a.mb) if a.set == "mlp" else bert_shapes(a.mb) if a.set == "bert" else
              ragged_shapes() if a.set == "ragged" else ref_shapes())
    for name, M, N, K, a_t, b_t, epi in shapes:
        if a.shapes and name not in a.shapes.split(","):
            continue
        if a.dtype == "f32" and K > 8192:
            continue
        A = (torch.rand(K, M, device="cuda") * 2 - 1).to(dt) if a_t else (torch.rand(M, K, device="cuda") * 2 - 1).to(dt)
        B = (torch.rand(N, K, device="cuda") * 2 - 1).to(dt) if b_t else (torch.rand(K, N, device="cuda") * 2 - 1).to(dt)
        out_dt = torch.float32 if epi == G.EPI_NONE else dt
        C = torch.empty(M, N, device="cuda", dtype=out_dt)
        bias = (torch.rand(N, device="cuda") - 0.5).to(dt)
        aux = (torch.rand(M, N, device="cuda") - 0.5).to(out_dt)
        kw = {}
        if epi in (G.EPI_BIAS, G.EPI_BIAS_RELU):
            kw["bias"] = bias
        if epi == G.EPI_RELU_MASK:
            kw["aux"] = aux
        Am = A.t() if a_t else A
        Bm = B.t() if b_t else B

        def mine():
            G.gemm(A, a_t, B, b_t, C, epi, **kw)

        def ref():
            r = torch.matmul(Am, Bm)
            if epi in (G.EPI_BIAS, G.EPI_BIAS_RELU):
                r = r + bias
            if epi == G.EPI_BIAS_RELU:
                r = torch.relu_(r)
            return r

        def ref_mm_only():
            torch.matmul(Am, Bm)

        wire_sweep = a.sweep_wire and a_t and not b_t
        if wire_sweep:
            from fpga_ai_nic_amd.ops import wire as W

            shard_w = (M * N + N + 255) // 256 * 256
            wbuf_s = torch.empty(W.shard_bytes("bfp_rne", shard_w), dtype=torch.uint8, device="cuda")
            wt_s = (wbuf_s, shard_w, -1, W.codec_id("bfp_rne"))
        if a.sweep and dt == torch.bfloat16:
            res = {}
            tiles = ((256, 256), (256, 128), (128, 256), (128, 128)) + (((224, 128),) if not a_t else ())
            for tile in tiles:
                for waves in (8, 4) if tile[0] != 224 else (4,):
                    for sk in (1, 2, 3, 4, 6, 8):
                        if M % tile[0] or N % tile[1] or K % (64 * sk):
                            continue
                        t3 = tile + (waves,)
                        fn = lambda t=t3, s=sk: G.gemm(A, a_t, B, b_t, C, epi, split_k=s, tile=t, **kw)  # noqa: E731
                        fn()
                        torch.cuda.synchronize()
                        ref_out = ref().float() * ((aux > 0) if epi == G.EPI_RELU_MASK else 1)
                        ok = (C.float() - ref_out).abs().max().item() < 1.0
                        if wire_sweep:  # the plan is checked above with the f32 epilogue; time the wire one
                            fn = lambda t=t3, s=sk: G.gemm(A, a_t, B, b_t, C, G.EPI_WIRE, split_k=s, tile=t,  # noqa: E731
                                                           wire=wt_s)
                        res[f"{tile[0]}x{tile[1]}w{waves}/s{sk}"] = round(
                            statistics.median(time_fn(fn, a.iters) for _ in range(3)), 2) if ok else "WRONG"
            valid = {k: v for k, v in res.items() if v != "WRONG"}
            best = min(valid, key=valid.get) if valid else None
            print(json.dumps({"shape": name, "epi": "wire" if wire_sweep else epi, "sweep_us": res, "best": best,
                              "auto_plan": G._ext.require().gemm_plan(M, N, K)}), flush=True)
        mine(); ref(); torch.cuda.synchronize()
        err = (C.float() - (ref().float() * ((aux > 0) if epi == G.EPI_RELU_MASK else 1))).abs().max().item()
        tm, tr, tmm = [], [], []
        Cx = G._ext.require()
        loops = [int(x) for x in a.loops.split(",") if x]
        tloop = {m: [] for m in loops}
        mode0 = Cx.gemm_main_loop()
        arms = {}
        if a.epi_arms and a_t and not b_t and dt == torch.bfloat16:
            from fpga_ai_nic_amd.ops import wire as W

            cs = torch.empty(N, device="cuda")
            shard = (M * N + N + 255) // 256 * 256
            wbuf = torch.empty(W.shard_bytes("bfp_rne", shard), dtype=torch.uint8, device="cuda")
            wt = (wbuf, shard, -1, W.codec_id("bfp_rne"))
            arms = {"colsum": lambda: G.gemm(A, a_t, B, b_t, C, epi, colsum=cs),
                    "wire": lambda: G.gemm(A, a_t, B, b_t, C, G.EPI_WIRE, wire=wt),
                    "wire_colsum": lambda: G.gemm(A, a_t, B, b_t, C, G.EPI_WIRE, colsum=cs, wire=wt)}
        tarm = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                tarm[k].append(time_fn(fn, a.iters))
            for mode in loops:  # same plan, other main loop (256x256 tiles only differ)
                Cx.gemm_set_main_loop(mode)
                tloop[mode].append(time_fn(mine, a.iters))
                Cx.gemm_set_main_loop(mode0)
            tm.append(time_fn(mine, a.iters))
            tr.append(time_fn(ref, a.iters))
            tmm.append(time_fn(ref_mm_only, a.iters))
        flop = 2.0 * M * N * K
        m, r, rm = statistics.median(tm), statistics.median(tr), statistics.median(tmm)
        plan = G._ext.require().gemm_plan(M, N, K, 0) if dt == torch.bfloat16 else None
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "a_t": a_t, "b_t": b_t, "epi": epi,
                          "dtype": a.dtype, "plan": plan,
                          "mine_us": round(m, 2), "mine_tflops": round(flop / m / 1e6, 1),
                          "torch_fused_us": round(r, 2), "torch_matmul_only_us": round(rm, 2),
                          "torch_matmul_tflops": round(flop / rm / 1e6, 1), "speedup_vs_torch_fused": round(r / m, 3),
                          "max_abs_err": err,
                          **({"loop_us": {str(k): round(statistics.median(v), 2) for k, v in tloop.items()}}
                             if loops else {}),
                          **({"epi_arms_us": {k: round(statistics.median(v), 2) for k, v in tarm.items()}}
                             if arms else {})}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""BASELINE config 5: BERT-base layer gradients (bf16) — backward MFMA GEMMs on the compute stream overlapped
with the compressed all-reduce (+ fused SGD) of each layer's gradient bucket on the side HIP stream.

Measures (median of rounds): t_compute (backward GEMMs only), t_comm (all-reduce of all buckets only),
t_overlap (both, issued the way a trainer does: bucket i's all-reduce right after layer i's backward) and
overlap efficiency = (t_compute + t_comm - t_overlap) / min(t_compute, t_comm).

1 GPU:  python bench/bert_overlap.py
N GPUs: torchrun --nproc-per-node N --master-addr 127.0.0.1 bench/bert_overlap.py
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpga_ai_nic_amd.models import bert  # noqa: E402
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402
from fpga_ai_nic_amd.parallel.dp import make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import ThreadFabric, TorchDistTransport  # noqa: E402
from fpga_ai_nic_amd.utils import dist as D  # noqa: E402


def measure(eng, dev, world, tokens=4096, layers=12, rounds=5, only=""):
    """Config 5 on an engine: the BERT-base layers' backward GEMMs (compute stream) and each layer bucket's
    all-reduce + fused SGD (the engine's stream), as compute only, comm only and both; medians over ``rounds``
    (max over ranks). Also called by bench.py at world > 1 (``extra.config5``)."""
    buckets = bert.gradient_buckets(layers)
    bufs = []
    for b in buckets:
        L = eng.layout(b.numel)
        g = (torch.randn(L.n_pad, device=dev) * 1e-3).to(torch.bfloat16)
        g[b.numel:] = 0
        w = torch.randn(L.n_pad, device=dev) * 0.02
        bufs.append((b, g, w, w.to(torch.bfloat16)))
    T = tokens
    gemms = []
    for name, M, N, K, a_t, b_t in bert.layer_backward_gemms(T):
        A = torch.randn(K, M, device=dev).to(torch.bfloat16) if a_t else torch.randn(M, K, device=dev).to(torch.bfloat16)
        B = torch.randn(N, K, device=dev).to(torch.bfloat16) if b_t else torch.randn(K, N, device=dev).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if "wgrad" in name else torch.bfloat16)
        gemms.append((A, a_t, B, b_t, C))

    def layer_bwd():
        for A, a_t, B, b_t, C in gemms:
            G.gemm(A, a_t, B, b_t, C)

    def comm(b, g, w, lp):
        return eng.allreduce_sgd(g, w, lp, n_valid=b.numel, lr=1e-4, grad_scale=1.0 / world, name=b.name)

    def run(do_compute, do_comm):
        D.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hs = []
        for li, (b, g, w, lp) in enumerate(bufs):
            if do_compute and b.name.startswith("layer"):
                layer_bwd()
            if do_comm:
                hs.append(comm(b, g, w, lp))
        for h in hs:
            h.wait()
        torch.cuda.synchronize()
        return D.max_over_ranks(time.perf_counter() - t0)

    kinds = {"compute": (True, False), "comm": (False, True), "overlap": (True, True)}
    run(*kinds[only or "overlap"])  # warmup (GEMM plan tuning, engine scratch): in --only mode of that kind only
    res = {"compute": [], "comm": [], "overlap": []}
    for _ in range(rounds):
        for k, (dc, dm) in kinds.items():
            if not only or only == k:
                res[k].append(run(dc, dm))
                if only:  # a clear idle gap between rounds, so a trace can be cut into them
                    time.sleep(0.01)
    if only:
        for k in res:
            res[k] = res[k] or [0.0]
    tc, tm, to = (statistics.median(res[k]) * 1e3 for k in ("compute", "comm", "overlap"))
    eff = (tc + tm - to) / min(tc, tm) if min(tc, tm) > 0 else 0.0
    flops = bert.layer_backward_flops(T) * layers
    return {"tokens_per_gpu": T, "params": bert.num_params(layers), "t_compute_ms": round(tc, 3),
            "t_comm_ms": round(tm, 3), "t_overlap_ms": round(to, 3), "overlap_efficiency": round(eff, 3),
            "bwd_gemm_tflops": round(flops / (tc / 1e3) / 1e12, 1) if tc > 0 else None,
            "comm_algo_bw_GBps": round(bert.num_params(layers) * 4 / (tm / 1e3) / 1e9, 1) if tm > 0 else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096, help="batch x seq rows per GPU (e.g. 8 x 512)")
    ap.add_argument("--compress", default="bfp", choices=["bfp", "raw", "rccl"])
    ap.add_argument("--algo", default="mesh", choices=["mesh", "ring"])
    ap.add_argument("--rings", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--engine", default="native", choices=["python", "native"])
    ap.add_argument("--only", default="", choices=["", "compute", "comm", "overlap"],
                    help="profiling: run only rounds of this kind (one kernel trace per kind, for tools/overlap_report.py)")
    a = ap.parse_args()
    rank, world, _, dev = D.init_distributed()
    transport = TorchDistTransport() if world > 1 else ThreadFabric(1).transport(0)
    if a.engine == "native" and a.compress != "rccl":
        from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce

        codec = {"bfp": "bfp_rne", "raw": "raw_f32"}[a.compress]
        # world 1: keep the side stream (no inline) so the overlap is real even on one GPU
        eng = NativeAllReduce(transport, codec=codec, algo=a.algo, rings=a.rings, side_stream=(world == 1))
    else:
        eng = make_engine(transport, a.compress, algo=a.algo, rings=a.rings)
        if world == 1:  # force the side-stream path so the overlap is real even on one GPU
            eng.inline = False
            eng.stream = torch.cuda.Stream(priority=-1)
    r = measure(eng, dev, world, tokens=a.tokens, layers=a.layers, rounds=a.rounds, only=a.only)
    if rank == 0:
        print(json.dumps({"bench": "bert_base_bwd_overlap", "n_gpus": world, "compress": a.compress,
                          "engine": a.engine, "algo": a.algo, **r, "only": a.only or None}), flush=True)
    D.cleanup()


if __name__ == "__main__":
    main()

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


def _offsets(bucket):
    """tensor name -> (flat offset in the bucket, shape)"""
    off, out = 0, {}
    for nm, shp in bucket.tensors:
        k = 1
        for d in shp:
            k *= d
        out[nm] = (off, shp)
        off += k
    return out


# (linear, tensor prefix inside the layer bucket, fin, fout) in backward order
_LINEARS = (("ffn_out", "output.dense", bert.FFN, bert.HIDDEN), ("ffn_in", "intermediate.dense", bert.HIDDEN, bert.FFN),
            ("attn_out", "attention.output.dense", bert.HIDDEN, bert.HIDDEN),
            ("qkv", "attention.self.qkv", bert.HIDDEN, 3 * bert.HIDDEN))


def measure(eng, dev, world, tokens=4096, layers=12, rounds=5, only="", last_on_producer=True, group_wgrad=None):
    """Config 5 on an engine: a BERT-base backward whose gradients ARE the all-reduce's input. Per encoder layer (last
    first) the four projections' bwd-data GEMM (bf16 dX) and bwd-weight GEMM run on the compute stream; each
    bwd-weight GEMM writes its dW — and, fused, its bias gradient — straight into the layer's gradient bucket, BFP-
    encoded by the GEMM epilogue into the engine's wire buffer when the engine takes producer-encoded input (the
    MLP's dp.py path; otherwise f32 into the bucket and the engine encodes). The LayerNorm gradients (no GEMM) are
    encoded after the layer's GEMMs, and the bucket's all-reduce + fused SGD is issued right after that, on the
    engine's stream, consuming exactly what the GEMMs produced. The pooler bucket is issued first and the embedding
    bucket last, where a real backward produces them (their producers — the pooler's tiny GEMM, the embedding
    scatter-add — are modelled as the encode of their buckets). Timed as compute only (GEMMs + encodes), comm only
    (the all-reduces of the encoded buckets) and both; medians over ``rounds`` (max over ranks). Also called by
    bench.py (``extra.config5``)."""
    from fpga_ai_nic_amd import _ext

    C = _ext.require()
    buckets = bert.gradient_buckets(layers)
    T = tokens
    acts = {}  # per projection: X [T, fin] (ReLU-free layer input) and dY [T, fout], shared by every layer
    for name, _, fin, fout in _LINEARS:
        acts[name] = ((torch.rand(T, fin, device=dev) * 2 - 1).to(torch.bfloat16),
                      ((torch.rand(T, fout, device=dev) * 2 - 1) * 1e-2).to(torch.bfloat16),
                      ((torch.rand(fin, fout, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16),
                      torch.empty(T, fin, device=dev, dtype=torch.bfloat16))
    bufs = []
    prepacked_buckets = 0
    for b in buckets:
        L = eng.layout(b.numel)
        g = torch.randn(L.n_pad, device=dev) * 1e-3
        g[b.numel:] = 0
        w = torch.randn(L.n_pad, device=dev) * 0.02
        tgt = eng.prepack_target(g, b.numel) if getattr(eng, "prepack", False) else None
        prepacked_buckets += tgt is not None
        bufs.append((b, g, w, w.to(torch.bfloat16), L, tgt, _offsets(b)))

    def encode_range(g, tgt, lo, hi):
        if tgt is not None and hi > lo:
            C.wire_pack_range(g, tgt[0], tgt[1], lo, hi, tgt[3])

    def produce(bi):
        """bucket bi's gradient, produced into the bucket (and its wire buffer)"""
        b, g, _, _, L, tgt, offs = bufs[bi]
        if not b.name.startswith("layer"):
            encode_range(g, tgt, 0, b.numel)
            return
        pre = f"encoder.layer.{b.name[5:]}."
        probs = []
        for name, tn, fin, fout in _LINEARS:
            X, dY, W, dX = acts[name]
            G.gemm(dY, False, W, True, dX)  # bwd-data dX = dY . W^T
            woff, _ = offs[pre + tn + ".weight"]
            boff, _ = offs[pre + tn + ".bias"]
            probs.append((X, dY, g[woff: woff + fin * fout].view(fin, fout), g[boff: boff + fout], woff))
        wire = (tgt[0], tgt[1], tgt[2], tgt[3], tgt[4]) if tgt is not None else None
        if group_wgrad:
            # the layer's four bwd-weight GEMMs in one dispatch, after its bwd-data chain (each projection's dW
            # needs only its own X and dY)
            G.gemm_wgrad_group(probs, wire=wire)
        else:
            for X, dY, dW, db, woff in probs:
                if wire is not None:
                    G.gemm(X, True, dY, False, dW, G.EPI_WIRE, colsum=db, wire=wire + (woff,))
                else:
                    G.gemm(X, True, dY, False, dW, G.EPI_NONE, colsum=db)
        for ln in ("attention.output.LayerNorm", "output.LayerNorm"):  # [weight | bias], no GEMM
            lo, _ = offs[pre + ln + ".weight"]
            encode_range(g, tgt, lo, lo + 2 * bert.HIDDEN)

    on_producer_ok = last_on_producer and hasattr(eng, "C") and not getattr(eng, "inline", True)
    if group_wgrad is None:
        group_wgrad = os.environ.get("FAN_GROUP_WGRAD", "1") != "0" and G.wgrad_group_supported(
            [(acts[nm][0], acts[nm][1]) for nm, _, _, _ in _LINEARS])

    def comm(bi):
        b, g, w, lp, L, tgt, _ = bufs[bi]
        kw = {"prepacked": (tgt[0], L.n_pad)} if tgt is not None else {}
        if on_producer_ok and bi == len(bufs) - 1:
            # the backward's last bucket (embeddings): nothing left to overlap it with, so on the compute stream (the
            # trainer's schedule, dp.py last_on_producer)
            kw["on_producer"] = True
        return eng.allreduce_sgd(g, w, lp, n_valid=b.numel, lr=1e-4, grad_scale=1.0 / world, name=b.name, **kw)

    enq = {}

    def run(do_compute, do_comm):
        D.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hs = []
        for bi in range(len(bufs)):
            if do_compute:
                produce(bi)
            if do_comm:
                hs.append(comm(bi))
        for h in hs:
            h.wait()
        # host time to issue the round (close to the total: the round is launch-bound, not GPU-bound)
        enq.setdefault((do_compute, do_comm), []).append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        return D.max_over_ranks(time.perf_counter() - t0)

    kinds = {"compute": (True, False), "comm": (False, True), "overlap": (True, True)}
    run(True, False)  # the buckets' wire buffers hold a producer's encoding before any comm-only round
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
            "overlap_vs_compute": round(to / tc, 3) if tc > 0 else None,
            "producer_encoded_buckets": prepacked_buckets, "buckets": len(bufs), "grouped_wgrad": bool(group_wgrad),
            "bwd_gemm_tflops": round(flops / (tc / 1e3) / 1e12, 1) if tc > 0 else None,
            "comm_algo_bw_GBps": round(bert.num_params(layers) * 4 / (tm / 1e3) / 1e9, 1) if tm > 0 else None,
            "enqueue_ms": {k: round(statistics.median(enq.get(v, [0.0])) * 1e3, 3) for k, v in kinds.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096, help="batch x seq rows per GPU (e.g. 8 x 512)")
    ap.add_argument("--compress", default="bfp", choices=["bfp", "raw", "rccl"])
    ap.add_argument("--algo", default="mesh", choices=["mesh", "ring"])
    ap.add_argument("--rings", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--engine", default="native", choices=["python", "native"])
    ap.add_argument("--forced", action="store_true",
                    help="world 1 through the multi-rank path (1-rank RCCL group, sharded update: bench.py extra.config5)")
    ap.add_argument("--only", default="", choices=["", "compute", "comm", "overlap"],
                    help="profiling: run only rounds of this kind (one kernel trace per kind, for tools/overlap_report.py)")
    a = ap.parse_args()
    rank, world, _, dev = D.init_distributed(force=a.forced)
    transport = TorchDistTransport() if world > 1 else ThreadFabric(1).transport(0)
    if a.forced:
        from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce
        from fpga_ai_nic_amd.parallel.transport import NativeTransport

        eng = NativeAllReduce(NativeTransport(force_collectives=True), codec="bfp_rne", algo="mesh", force_comm=True,
                              shard_update=True)
    elif a.engine == "native" and a.compress != "rccl":
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

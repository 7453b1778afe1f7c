#!/usr/bin/env python3
"""Flagship benchmark: data-parallel MLP 1024-4096-4096-1024 training on MI355X.

BASELINE.json config 3: bf16 MLP, BFP-compressed all-reduce of every layer's gradient bucket with the SGD
weight update fused into the all-gather epilogue, comm overlapped with backward on a side HIP stream.
Metric: whole-job training throughput in samples/s (weak scaling: per-GPU batch fixed as N grows).

Contract: ``python bench.py --gpus N --steps K --warmup W`` (N>1 under torch.distributed.run, one rank per
GPU over RCCL). W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier +
torch.cuda.synchronize() on both sides; max time over ranks; rank 0 prints ONE JSON line.

Synthetic data (random bf16 inputs, random labels) and random-init weights of the named architecture.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fpga_ai_nic_amd.models.mlp import MLP  # noqa: E402
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import (NativeTransport, ThreadFabric, TorchDistTransport,  # noqa: E402
                                                make_p2p_comm)
from fpga_ai_nic_amd.utils import dist as D  # noqa: E402

SIZES = [1024, 4096, 4096, 1024]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # per-GPU minibatch (weak scaling). The reference fixes only the architecture for this config; 8192 rows per
    # GPU keeps the MFMA GEMMs out of the tile-quantisation regime (measured: 2048 -> 4.6M samples/s,
    # 8192 -> 6.9M samples/s on one MI355X) and gives the overlapped all-reduce a ~1.2 ms backward to hide in.
    ap.add_argument("--mb-per-gpu", type=int, default=8192)
    ap.add_argument("--compress", default="bfp", choices=["bfp", "raw", "raw_bf16", "rccl", "local"])
    ap.add_argument("--rounding", default="rne", choices=["rne", "trunc"])
    ap.add_argument("--algo", default="mesh", choices=["mesh", "ring"])
    ap.add_argument("--rings", type=int, default=1)
    ap.add_argument("--transport", default="torch", choices=["torch", "native", "p2p"],
                    help="torch/native: RCCL collectives; p2p: direct HIP-IPC peer writes + stream flags "
                         "(C++ engine only)")
    ap.add_argument("--engine", default="native", choices=["python", "native"],
                    help="request path: Python-issued engine or the C++ engine (csrc/comm/engine.cpp)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--graph", action="store_true",
                    help="capture one training step in a HIP graph and replay it (world 1, inline engine)")
    ap.add_argument("--side-stream", action="store_true",
                    help="world 1: run the engine's requests (BFP decode + fused SGD) on its high-priority side stream, "
                         "overlapped with the following GEMMs, instead of inline on the compute stream")
    ap.add_argument("--force-dist", action="store_true",
                    help="world 1 through the full multi-rank path (1-rank RCCL group, side-stream engine)")
    ap.add_argument("--epi", default="producer", choices=["comm", "producer"],
                    help="side-stream engine: run each request's decode+SGD epilogue on the comm stream (overlapped "
                         "with the remaining backward) or on the compute stream after the last backward GEMM")
    a = ap.parse_args()

    rank, world, local, device = D.init_distributed(force=a.force_dist)
    if world != a.gpus and rank == 0:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if device.type != "cuda":
        print("[bench] no GPU visible: running the CPU path (functional only)", file=sys.stderr)
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    comm = None
    if world > 1 or a.force_dist:
        transport = NativeTransport(force_collectives=a.force_dist) if a.transport == "native" else \
            TorchDistTransport(force_collectives=a.force_dist)
        if a.transport == "p2p" and device.type == "cuda" and a.engine == "native":
            comm = make_p2p_comm()
    else:
        transport = ThreadFabric(1).transport(0)
    kind = "local" if a.compress == "local" else a.compress
    engine = make_engine(transport, kind, rounding=a.rounding, algo=a.algo, rings=a.rings,
                         force_comm=a.force_dist, impl=a.engine if device.type == "cuda" else "python", comm=comm,
                         side_stream=a.side_stream)
    if hasattr(engine, "epilogue_on_producer"):
        engine.epilogue_on_producer = a.epi == "producer"
    pad_fn = (lambda n: engine.layout(n).n_pad) if engine is not None else None
    model = MLP(SIZES, dtype=dtype, device=device, pad_fn=pad_fn, seed=1)
    if world > 1:
        for l in model.layers:
            transport.broadcast_(l.master, 0)
        model.sync_lp()
    trainer = DataParallelTrainer(model, engine, lr=a.lr)
    mb = a.mb_per_gpu
    g = torch.Generator().manual_seed(1234 + rank)
    x = (torch.rand(mb, SIZES[0], generator=g) * 2 - 1).to(device=device, dtype=dtype)
    y = torch.randint(0, SIZES[-1], (mb,), generator=g, dtype=torch.int32).to(device)

    for _ in range(a.warmup):
        trainer.step(x, y)
    trainer.finish()
    step = lambda: trainer.step(x, y)  # noqa: E731
    graphed = False
    if a.graph and device.type == "cuda" and world == 1 and (engine is None or getattr(engine, "inline", False)):
        # the whole step (fwd, loss, bwd GEMMs, BFP encode, fused SGD) is a fixed kernel sequence on one
        # stream at world 1: capture it once, replay per step (removes the host launch path entirely)
        try:
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                trainer.step(x, y)
                trainer.finish_async()
            torch.cuda.synchronize()
            step = gr.replay
            graphed = True
        except RuntimeError as e:  # capture unsupported for this configuration: stay eager
            print(f"[bench] HIP graph capture failed ({e}); running eagerly", file=sys.stderr)
            torch.cuda.synchronize()
    D.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    loss_rows = model.loss_rows
    t_enqueue = time.perf_counter() - t0  # host time to issue K steps (GPU may still be running)
    trainer.finish()
    if device.type == "cuda":
        torch.cuda.synchronize()
    D.barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t0)
    loss = float(loss_rows.float().mean().item())

    ms = elapsed / a.steps * 1e3
    global_batch = mb * world
    value = global_batch * a.steps / elapsed
    flops = model.flops_per_sample() * global_batch * a.steps / elapsed
    grad_bytes = sum(l.n for l in model.layers) * 4
    if rank == 0:
        rec = {
            "metric": "MLP training samples/sec (1024-4096-4096-1024, BFP all-reduce + fused SGD)",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic (random inputs/labels, random-init weights)",
            "config": {
                "model": "mlp-1024-4096-4096-1024",
                "global_batch": global_batch,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "mb_per_gpu": mb,
                "compress": a.compress,
                "rounding": a.rounding,
                "algo": a.algo,
                "rings": engine.rings if engine is not None else 0,
                "transport": a.transport if world > 1 else "none",
                "engine": a.engine if device.type == "cuda" else "python",
                "hip_graph": graphed,
                "fused_sgd": True,
                "epilogue_stream": ("compute" if getattr(engine, "epilogue_on_producer", False) else "comm")
                if engine is not None and not getattr(engine, "inline", True) else "inline",
            },
            "extra": {
                "achieved_tflops": round(flops / 1e12, 2),
                "host_enqueue_ms_per_step": round(t_enqueue / a.steps * 1e3, 4),
                "grad_bytes_f32_per_step": grad_bytes,
                "effective_allreduce_algo_bw_GBps": round(grad_bytes / (ms / 1e3) / 1e9, 2),
                "final_loss": round(loss, 5),
                **({"engine_counters": engine.counters()} if hasattr(engine, "counters") else {}),
            },
        }
        print(json.dumps(rec), flush=True)
    D.cleanup()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Flagship benchmark: data-parallel MLP 1024-4096-4096-1024 training on MI355X.

BASELINE.json config 3: bf16 MLP, BFP-compressed all-reduce of every layer's gradient bucket with the SGD
weight update fused into the all-gather epilogue, comm overlapped with backward on a side HIP stream.
Metric: whole-job training throughput in samples/s (weak scaling: per-GPU batch fixed as N grows), plus the
all-reduce algo-BW of the requests that ran inside the timed steps (device timestamps of each request's
communication phase, ``extra.allreduce``).

Contract: ``python bench.py --gpus N --steps K --warmup W``. Under torch.distributed.run (RANK / WORLD_SIZE set)
every process is one rank on one GPU over RCCL. Without that environment and N > 1, this script starts
``torch.distributed.run --nproc-per-node N`` itself as a CHILD process before anything touches the GPU, and
exits with its code (the parent never initialises HIP). W untimed warmup steps, then EXACTLY K timed steps
bracketed by barrier + torch.cuda.synchronize() on both sides; max time over ranks; rank 0 prints ONE JSON line.

Synthetic data (random bf16 inputs, random labels) and random-init weights of the named architecture.
Reference workload shapes: sw/run.sh:16 (global MB 5376 over 3 ranks = 1792 per rank) — reported as
``extra.mb1792`` next to the headline per-GPU batch.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import time

SIZES = [1024, 4096, 4096, 1024]
REF_MB_PER_RANK = 1792  # sw/run.sh:16: global MB 5376 / 3 ranks
REF_STEPS = 100  # timed steps of the reference-batch measurement (extra.mb1792) at least


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # per-GPU minibatch (weak scaling). The reference fixes only the architecture for this config; 8192 rows per
    # GPU keeps the MFMA GEMMs out of the tile-quantisation regime (measured: 2048 -> 4.6M samples/s,
    # 8192 -> 7.2M samples/s on one MI355X) and gives the overlapped all-reduce a ~1.1 ms backward to hide in.
    # The reference's own per-rank batch (1792) is measured as well and reported in extra.mb1792.
    ap.add_argument("--mb-per-gpu", type=int, default=8192)
    ap.add_argument("--ref-mb", type=int, default=REF_MB_PER_RANK,
                    help="also time K steps at this per-GPU batch (extra.mb<ref>); 0 disables")
    ap.add_argument("--compress", default="bfp", choices=["bfp", "raw", "raw_bf16", "rccl", "local"])
    ap.add_argument("--rounding", default="rne", choices=["rne", "trunc"])
    ap.add_argument("--algo", default="mesh", choices=["mesh", "ring"])
    ap.add_argument("--rings", type=int, default=1)
    ap.add_argument("--transport", default="native", choices=["torch", "native", "p2p"],
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
    ap.add_argument("--no-trace", action="store_true",
                    help="skip the separate traced pass that measures the all-reduce phases (extra.allreduce)")
    ap.add_argument("--timeout", type=float, default=300.0,
                    help="watchdog budget per phase in seconds (init, warmup, timed steps, ...) and the bound of every "
                         "all-reduce wait: on expiry the engine's debug_status() goes to stderr, the communicator is "
                         "aborted and the rank exits with code 124 (0 disables)")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(a, argv) -> int | None:
    """--gpus N > 1 without a torch.distributed environment: run N ranks under torch.distributed.run as a child
    process (this process never touches the GPU) and return its exit code; None when no launch is needed."""
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL / CUDA-tensor sharing across processes)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    print(f"[bench] launching {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def _time_steps(step, steps, device, D):
    import torch

    D.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    return t0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    rc = self_launch(a, argv)
    if rc is not None:
        return rc

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import (NativeTransport, ThreadFabric, TorchDistTransport,
                                                    make_p2p_comm)
    from fpga_ai_nic_amd.utils import dist as D
    from fpga_ai_nic_amd.utils.watchdog import Watchdog

    # watchdog: every phase of the run is bounded; on expiry the engine state goes to stderr and the rank exits 124
    held = {"engine": None, "comm": None, "transport": None}
    env_rank = int(os.environ.get("RANK", "0"))

    def _dump():
        e = held["engine"]
        d = {"rank": env_rank, "world": int(os.environ.get("WORLD_SIZE", "1"))}
        if e is not None and hasattr(e, "debug_status"):
            d["engine"] = e.debug_status()
        if held["comm"] is not None and hasattr(held["comm"], "flags_snapshot"):
            d["p2p_flags"] = list(held["comm"].flags_snapshot(2.0))
        return d

    def _abort():
        for k in ("comm", "transport"):
            if held[k] is not None and hasattr(held[k], "abort"):
                held[k].abort()

    wd = Watchdog(a.timeout, dump=_dump, on_abort=_abort, tag=f"bench rank {env_rank}")
    wd.arm("init")
    hook = sys.excepthook

    def _excepthook(et, ev, tb):  # an uncaught error (e.g. an all-reduce timeout) also reports the engine state
        try:
            print(f"[bench rank {env_rank}] debug_status " + json.dumps(_dump(), default=str), file=sys.stderr,
                  flush=True)
        except Exception:  # noqa: BLE001
            pass
        hook(et, ev, tb)

    sys.excepthook = _excepthook
    rank, world, local, device = D.init_distributed(force=a.force_dist)
    if world != a.gpus and rank == 0:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if device.type != "cuda":
        print("[bench] no GPU visible: running the CPU path (functional only)", file=sys.stderr)
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    comm = None
    impl = a.engine if device.type == "cuda" else "python"
    if world > 1 or a.force_dist:
        transport = None
        if a.transport == "native" and impl == "native":
            try:  # the C++ engine's own RCCL communicator (unique id exchanged over torch.distributed)
                transport = NativeTransport(force_collectives=a.force_dist)
            except Exception as e:  # noqa: BLE001 - keep the run measurable on torch.distributed's communicator
                print(f"[bench] rank {rank}: native communicator failed ({e}); using torch.distributed", file=sys.stderr)
                a.transport = "torch"
            if world > 1:  # every rank on the same communicator
                ok = torch.tensor([0 if transport is None else 1], device=device)
                torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
                if int(ok.item()) == 0:
                    transport, a.transport = None, "torch"
        if transport is None:
            transport = TorchDistTransport(force_collectives=a.force_dist)
        if a.transport == "p2p" and device.type == "cuda" and impl == "native":
            comm = make_p2p_comm()
        if comm is None:  # report the transport the gradient plane actually uses
            a.transport = getattr(transport, "name", a.transport)
    else:
        transport = ThreadFabric(1).transport(0)
    held["transport"], held["comm"] = transport, comm
    engine = make_engine(transport, a.compress, rounding=a.rounding, algo=a.algo, rings=a.rings,
                         force_comm=a.force_dist, impl=impl, comm=comm, side_stream=a.side_stream,
                         timeout_s=a.timeout + 30.0 if a.timeout > 0 else 600.0)  # the watchdog fires first
    held["engine"] = engine
    if hasattr(engine, "epilogue_on_producer") and not getattr(engine, "inline", True):
        engine.epilogue_on_producer = a.epi == "producer"
    pad_fn = (lambda n: engine.layout(n).n_pad) if engine is not None else None
    model = MLP(SIZES, dtype=dtype, device=device, pad_fn=pad_fn, seed=1)
    if world > 1:
        for l in model.layers:
            transport.broadcast_(l.master, 0)
        model.sync_lp()
    trainer = DataParallelTrainer(model, engine, lr=a.lr)
    # device-timed communication phases of the requests (C++ engine, multi-rank path): measured in a separate
    # traced pass, so the headline steps run with tracing off (its timing events and timed flag waits cost time)
    can_trace = (not a.no_trace and hasattr(engine, "trace") and not getattr(engine, "inline", True))
    stall_rank = int(os.environ.get("FAN_BENCH_STALL_RANK", "-1"))

    def batch(mb, seed):
        g = torch.Generator().manual_seed(seed + rank)
        x = (torch.rand(mb, SIZES[0], generator=g) * 2 - 1).to(device=device, dtype=dtype)
        y = torch.randint(0, SIZES[-1], (mb,), generator=g, dtype=torch.int32).to(device)
        return x, y

    def run(mb, seed, graph_ok, trace=False, warmup=None, tag="timed", steps=None):
        """W warmup + K timed steps at per-GPU batch mb: (elapsed s max over ranks, host enqueue s, loss,
        trace summary or None, graphed). The garbage collector is off inside (a collection pause in the launch loop
        starves the GPU: one 20-step MB-1792 window once read 0.46 instead of 0.38 ms/step)."""
        steps = a.steps if steps is None else steps
        gc.collect()
        gc.disable()
        try:
            return _run(mb, seed, graph_ok, trace, warmup, tag, steps)
        finally:
            gc.enable()

    def _run(mb, seed, graph_ok, trace, warmup, tag, steps):
        x, y = batch(mb, seed)
        wd.arm(f"warmup {tag} mb={mb}")
        if stall_rank == rank:  # test hook: this rank stops taking part (a hung peer for the watchdog test)
            time.sleep(float(os.environ.get("FAN_BENCH_STALL_S", "600")))
        for _ in range(a.warmup if warmup is None else warmup):
            trainer.step(x, y)
        trainer.finish()
        wd.arm(f"{tag} mb={mb}")
        step = lambda: trainer.step(x, y)  # noqa: E731
        graphed = False
        if graph_ok and a.graph and device.type == "cuda" and world == 1 and \
                (engine is None or getattr(engine, "inline", False)):
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
        if trace:
            engine.trace(True)
        t0 = _time_steps(step, steps, device, D)
        loss_rows = model.loss_rows
        t_enqueue = time.perf_counter() - t0  # host time to issue K steps (GPU may still be running)
        trainer.finish()
        if device.type == "cuda":
            torch.cuda.synchronize()
        D.barrier()
        elapsed = D.max_over_ranks(time.perf_counter() - t0)
        tr = None
        if trace:
            tr = engine.trace_summary()
            engine.trace(False)
            tr["comm_ms"] = D.max_over_ranks(tr["comm_ms"])  # the slowest rank's communication time
            tr["ms_per_step"] = elapsed / steps * 1e3
        return elapsed, t_enqueue, float(loss_rows.float().mean().item()), tr, graphed

    mb = a.mb_per_gpu
    ref = None
    if a.ref_mb and a.ref_mb != mb:
        # The reference-batch measurement runs first. A short step: a longer window on the GPU (a host hiccup is then
        # a smaller share of it). Its ~50 ms of sustained load also brings the shader clock to the level a training
        # run holds, which a short headline window right after start-up would otherwise partly miss (same box:
        # 5 warmup + 20 steps read 1.080-1.100 ms/step, 40 + 20 read 1.039-1.051, 5 + 200 read 1.029;
        # profiles/r3_warmup_clock_ramp.txt). The headline still times exactly W warmup + K steps of its own batch.
        ref_steps = max(a.steps, REF_STEPS) if device.type == "cuda" else a.steps
        e2, _, _, _, _ = run(a.ref_mb, 4321, False, tag="ref", steps=ref_steps)
        ref = {"mb_per_gpu": a.ref_mb, "global_batch": a.ref_mb * world, "steps": ref_steps,
               "samples_per_s": round(a.ref_mb * world * ref_steps / e2, 2),
               "ms_per_step": round(e2 / ref_steps * 1e3, 4)}
    elapsed, t_enqueue, loss, _, graphed = run(mb, 1234, True)
    tr = run(mb, 1234, False, trace=True, warmup=1, tag="traced")[3] if can_trace else None
    # replicas after every step of the run: bit-identical weights on every rank (the reference reads its NIC
    # registers back to stdout after programming them, sw/mlp_mpi_example_f32.cpp:65-98; here the run proves
    # what it ran on and that the replicas agree)
    wd.arm("verify")
    dist_rec = _dist_report(a, engine, model, world, rank, device, D)
    wd.disarm()

    ms = elapsed / a.steps * 1e3
    global_batch = mb * world
    value = global_batch * a.steps / elapsed
    flops = model.flops_per_sample() * global_batch * a.steps / elapsed
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
                "transport": a.transport if (world > 1 or a.force_dist) else "none",
                "engine": impl,
                "hip_graph": graphed,
                "fused_sgd": True,
                # world 1: dW's BFP round trip + SGD inside the bwd-weight GEMM epilogue (no separate update pass)
                "fused_update_in_gemm": bool(getattr(trainer, "fused_update", False)),
                "epilogue_stream": ("compute" if getattr(engine, "epilogue_on_producer", False) else "comm")
                if engine is not None and not getattr(engine, "inline", True) else "inline",
            },
            "extra": {
                "achieved_tflops": round(flops / 1e12, 2),
                "host_enqueue_ms_per_step": round(t_enqueue / a.steps * 1e3, 4),
                "grad_bytes_f32_per_step": sum(l.n for l in model.layers) * 4,
                "allreduce": _allreduce_report(tr, world),
                f"mb{a.ref_mb}": ref,
                "final_loss": round(loss, 5),
                "dist": dist_rec,
                "gemm_tuning": _tuning_report(),
                **({"engine_counters": engine.counters()} if hasattr(engine, "counters") else {}),
            },
        }
        print(json.dumps(rec), flush=True)
    wd.arm("cleanup")
    D.cleanup()
    wd.close()
    if not dist_rec["replicas_identical"]:
        print(f"[bench] rank {rank}: replicas DIVERGED: {dist_rec['replica_digests']}", file=sys.stderr, flush=True)
        return 2
    return 0


def _tuning_report():
    """The GEMM plans the on-device tuner chose on this rank (shape key, static plan, chosen plan, their times)."""
    from fpga_ai_nic_amd.ops import gemm_tune

    t = gemm_tune.tuner()
    return {"enabled": t.enabled, "decisions": t.log}


def replica_digest(tensors):
    """Per tensor: (exact bit hash, fp64 sum). The hash is integer arithmetic on the f32 bit patterns (position-
    weighted, wrapping mod 2^64), so it is order-independent and equal across ranks iff the bits are."""
    import torch

    out = []
    for t in tensors:
        b = t.detach().reshape(-1).contiguous().view(torch.int32).to(torch.int64)
        w = torch.arange(b.numel(), device=b.device, dtype=torch.int64).mul_(2).add_(1)
        h = int((b * w).sum().item()) & 0xFFFFFFFFFFFFFFFF
        out.append([f"{h:016x}", float(t.detach().double().sum().item())])
    return out


def _dist_report(a, engine, model, world, rank, device, D):
    """extra.dist: what the run actually ran on — torch's and the engine communicator's rank counts (RCCL:
    ncclCommCount), the transport, the ring orders and link matrix the planner used, the devices (PCI bus ids) of
    the ranks — and whether the replicas' weights are bit-identical after the run (all-gathered digests)."""
    from fpga_ai_nic_amd.utils import topology

    C = getattr(engine, "C", None)
    mine = {
        "digest": replica_digest([l.master for l in model.layers]),
        "comm_ranks": int(C.comm_ranks) if C is not None else (world if engine is not None else 1),
        "bus_id": topology.device_bus_id(device.index) if device.type == "cuda" else None,
    }
    every = D.all_gather_object(mine)
    digests = [e["digest"] for e in every]
    ident = all(d == digests[0] for d in digests)
    return {
        "world": world,
        "torch_backend": D.backend(),
        "transport": a.transport if world > 1 or a.force_dist else "none",
        "engine_comm": (C.comm_kind if C is not None else ("python" if engine is not None else "none")),
        "comm_ranks": [e["comm_ranks"] for e in every],
        "algo": getattr(engine, "algo", None),
        "ring_orders": getattr(engine, "orders", None) if getattr(engine, "algo", None) == "ring" else None,
        "links": getattr(engine, "links", None),
        "bus_ids": [e["bus_id"] for e in every],
        "replicas_identical": ident,
        "replica_digests": digests if not ident else digests[0],
    }


def _allreduce_report(tr, world):
    """All-reduce algo-BW of the requests of the traced pass (the same K steps again, with per-request device
    timestamps): logical (f32 gradient) bytes / summed device time of their communication phases (request start on
    the comm stream -> end of the all-gather, slowest rank); bus-BW = algo-BW x 2(N-1)/N; wire-BW = bytes this rank
    actually sent (BFP-packed) / the same time. None when no collective ran (world 1 inline engine: no wire)."""
    if not tr or not tr.get("requests") or tr.get("comm_ms", 0) <= 0:
        return None
    s = tr["comm_ms"] / 1e3
    algo = tr["logical_bytes"] / s / 1e9
    return {
        "traced_ms_per_step": round(tr["ms_per_step"], 4),
        "requests": tr["requests"],
        "comm_ms_total": round(tr["comm_ms"], 4),
        "allreduce_algo_bw_GBps": round(algo, 2),
        "bus_bw_GBps": round(algo * 2 * (world - 1) / world, 2) if world > 1 else 0.0,
        "wire_bw_GBps": round(tr["wire_bytes"] / s / 1e9, 2),
        "phase_ms": {k: round(tr[k], 4) for k in ("pack_ms", "exchange_ms", "reduce_ms", "gather_ms", "epilogue_ms")},
        "dropped": tr.get("dropped", 0),
    }


if __name__ == "__main__":
    sys.exit(main())

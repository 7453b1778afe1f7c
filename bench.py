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
exits with its code (the parent never initialises HIP). On the GPU, untimed steps of the headline batch for
``--settle-ms`` (300 ms: the shader clock's ramp, ``extra.settle``); then W untimed warmup steps and EXACTLY K timed steps
bracketed by barrier + torch.cuda.synchronize() on both sides; max time over ranks; rank 0 prints ONE JSON line.

World > 1 (GPU): the run chooses its own schedule and checks it before timing anything (``--schedule auto``):
* every available arm — the C++ engine's mesh over its own RCCL communicator, the direct-P2P mesh and the direct-P2P
  ring over the link-disjoint rings, each with persistent or tile-grid GEMMs while a request is in flight, and the
  P2P arms with their pure copies on the copy engines — passes a bit-exact all-reduce gate (one production-path
  request vs the NumPy simulators, :mod:`fpga_ai_nic_amd.parallel.gate`) and is timed for a few steps;
  ``extra.schedule_ab`` lists every arm (ms/step, exactness, or the error that excluded it), ``extra.gates_failed``
  the arms whose all-reduce was not bit-exact (excluded; the run still records the fastest exact arm);
* the headline runs on the fastest exact arm; ``extra.dist.allreduce_exact`` is its gate. Exit codes: an A/B arm
  that fails the gate is excluded and listed in ``extra.gates_failed`` (the run still exits 0 with the fastest exact
  arm); only a failed gate of ``--schedule fixed``'s own engine exits 3 (after printing the line), diverged replicas
  exit 2, and no exact arm at all exits 3 without a line;
* after the headline (bounded by ``--extra-budget`` seconds): ``extra.config4`` (256 MB all-reduce + fused SGD:
  BFP mesh / ring, the uncompressed f32 all-reduce over the same transport and RCCL f32 + SGD kernel: algo- and
  bus-BW; BASELINE configs 2/4) and ``extra.uncompressed`` (the same MLP step with an uncompressed all-reduce:
  the analogue of the reference's smart-NIC vs MPI_Iallreduce comparison, sw/mlp_mpi_example_f32.cpp:615-643 vs
  :752-787).
World 1 also reports ``extra.forced_dist_ms_per_step`` (the multi-rank path over a 1-rank group) and
``extra.unfused_update_ms_per_step`` (decode + SGD as a separate pass instead of inside the bwd-weight GEMM), so a
1 -> N curve splits into compute, update pass and exposed communication.

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
CONFIG4_MB = 256  # BASELINE config 4: 256 MB synthetic gradient


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="GPU: before the headline's W warmup steps, untimed steps of the same batch until this much "
                         "wall time has passed (the shader clock's ramp; extra.settle); 0 = off")
    # per-GPU minibatch (weak scaling). The reference fixes only the architecture for this config; 8192 rows per
    # GPU keeps the MFMA GEMMs out of the tile-quantisation regime (measured: 2048 -> 4.6M samples/s,
    # 8192 -> 7.2M samples/s on one MI355X) and gives the overlapped all-reduce a ~1.1 ms backward to hide in.
    # The reference's own per-rank batch (1792) is measured as well and reported in extra.mb1792.
    ap.add_argument("--mb-per-gpu", type=int, default=8192)
    ap.add_argument("--ref-mb", type=int, default=REF_MB_PER_RANK,
                    help="also time K steps at this per-GPU batch (extra.mb<ref>); 0 disables")
    ap.add_argument("--compress", default="bfp", choices=["bfp", "raw", "raw_bf16", "rccl", "local"])
    ap.add_argument("--rounding", default="rne", choices=["rne", "trunc"])
    ap.add_argument("--schedule", default="auto", choices=["auto", "fixed"],
                    help="world > 1: auto = A/B every available transport x algorithm x GEMM form in warmup and run "
                         "the fastest exact one; fixed = exactly --transport / --algo / --rings")
    ap.add_argument("--algo", default="mesh", choices=["mesh", "ring"])
    ap.add_argument("--rings", type=int, default=1)
    ap.add_argument("--transport", default="native", choices=["torch", "native", "p2p"],
                    help="torch/native: RCCL collectives; p2p: direct HIP-IPC peer writes + stream flags "
                         "(C++ engine only)")
    ap.add_argument("--p2p-flags", default="cp", choices=["cp", "kernel"],
                    help="fixed schedule, p2p transport: flag writes/waits as command-processor packets or as kernels "
                         "(system-scope release store, bounded in-kernel spin)")
    ap.add_argument("--p2p-copy", default="kernel", choices=["kernel", "sdma"],
                    help="--schedule fixed over --transport p2p: pure copies on CUs (kernel) or the copy engines")
    ap.add_argument("--shard-update", type=int, default=-1, choices=[-1, 0, 1],
                    help="--schedule fixed: sharded weight update (1), the gathered-gradient update (0), env default (-1)")
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
    ap.add_argument("--gemm-inflight", default="persistent", choices=["persistent", "grid"],
                    help="schedule fixed: GEMM form while a request is in flight (see DataParallelTrainer)")
    ap.add_argument("--ab-steps", type=int, default=4, help="timed steps per arm of the schedule A/B (stage 1)")
    ap.add_argument("--ab2-steps", type=int, default=10,
                    help="schedule A/B stage 2: timed steps per round of each of the --ab2-top fastest stage-1 arms, "
                         "3 interleaved rounds after a warmup; the arm with the lowest median is chosen (0: stage 1 "
                         "decides)")
    ap.add_argument("--ab2-top", type=int, default=3, help="arms kept for stage 2 of the schedule A/B")
    ap.add_argument("--no-trace", action="store_true",
                    help="skip the separate traced pass that measures the all-reduce phases (extra.allreduce)")
    ap.add_argument("--extra-budget", type=float, default=240.0,
                    help="seconds the extras after the headline may take in total (config 4, uncompressed step, the "
                         "world-1 split); what does not fit is recorded as skipped; 0 disables them")
    ap.add_argument("--arm-timeout", type=float, default=90.0,
                    help="world > 1 schedule A/B: bound of each arm's exactness gate and of its steps' waits; an arm "
                         "whose transport hangs fails at this bound, the transport is aborted on every rank and its "
                         "remaining arms are excluded")
    ap.add_argument("--timeout", type=float, default=300.0,
                    help="watchdog budget per phase in seconds (init, warmup, timed steps, ...) and the bound of every "
                         "all-reduce wait: on expiry the engine's debug_status() goes to stderr, the communicator is "
                         "aborted and the rank exits with code 124 (0 disables)")
    return ap.parse_args(argv)


def _transport_error(t) -> str:
    """The communicator's sticky error ("p2p transport aborted", "aborted", an RCCL async error) or ""."""
    try:
        return t.async_error() or ""
    except Exception as e:  # noqa: BLE001
        return str(e) or "error"


def _release_mode() -> int:
    from fpga_ai_nic_amd import _ext

    return _ext.require().p2p_release_mode()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _device_count() -> int:
    """GPUs visible to this process, counted without initialising the HIP runtime (torch's count on this image)."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 0


def colocated_hw_queues(nranks: int, env) -> str | None:
    """Hardware queues per rank when several ranks share one GPU (the one-GPU rehearsals of a multi-GPU run).

    Every HIP stream of a process is served by one of that process's hardware queues (up to GPU_MAX_HW_QUEUES, 4 by
    default, beside the null stream's): ranks that build several engines (the schedule A/B) reach 5 queues each,
    and with 3 ranks on one GPU that is more user queues than the GPU maps at once. The command processor then
    time-slices the processes' queues, and a rank whose flag wait (a command-processor wait or a kernel-flag spin)
    is resident while the peer that must write the flag is switched out loses a time slice per hand-off: 50-840 ms
    kernels and a 1254 ms/step arm in the 3-rank trace (profiles/r6_hw_queue_oversubscription.txt). Capped at 2 per
    rank (3 with the null stream's) the co-located ranks stay mapped together (the same A/B: that arm 4.3-4.6 ms/step
    at 2 or 1 queues per rank). A smaller inherited GPU_MAX_HW_QUEUES is kept (the GPU boxes export 4, HIP's default).
    None: one GPU per rank (the driver's multi-GPU run: nothing to share), FAN_KEEP_HW_QUEUES=1, or no GPU."""
    if env.get("FAN_KEEP_HW_QUEUES") == "1":
        return None
    n = _device_count()
    if not 0 < n < nranks:
        return None
    try:
        cur = int(env.get("GPU_MAX_HW_QUEUES") or 4)
    except ValueError:
        cur = 4
    return "2" if cur > 2 else None


def self_launch(a, argv) -> int | None:
    """--gpus N > 1 without a torch.distributed environment: run N ranks under torch.distributed.run as a child
    process (this process never touches the GPU) and return its exit code; None when no launch is needed."""
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL / CUDA-tensor sharing across processes)
    hwq = colocated_hw_queues(a.gpus, env)
    if hwq is not None:
        env["GPU_MAX_HW_QUEUES"] = hwq
        print(f"[bench] {a.gpus} ranks share {_device_count()} GPU(s): GPU_MAX_HW_QUEUES={hwq} per rank",
              file=sys.stderr, flush=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    print(f"[bench] launching {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


class Setup:
    """One arm of the run: an engine (or None), the model it trains and its trainer."""

    def __init__(self, name, engine, model, trainer, info):
        self.name, self.engine, self.model, self.trainer, self.info = name, engine, model, trainer, info


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    rc = self_launch(a, argv)
    if rc is not None:
        return rc

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel import gate
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import (NativeTransport, ThreadFabric, TorchDistTransport,
                                                    try_native_transport, try_p2p_comm)
    from fpga_ai_nic_amd.utils import dist as D
    from fpga_ai_nic_amd.utils import topology
    from fpga_ai_nic_amd.utils.watchdog import Watchdog

    t_begin = time.perf_counter()
    # watchdog: every phase of the run is bounded; on expiry the engine state goes to stderr and the rank exits 124
    held = {"engine": None, "comm": None, "transport": None, "record": None}
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
        ph = wd.phase or ""
        if env_rank == 0 and held.get("record") is not None and (ph.startswith("extra") or ph == "verify"):
            try:  # one JSON line with the headline measured before the phase that hung
                print(json.dumps(held["record"](ph)), flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"[bench] partial record unavailable: {e!r}", file=sys.stderr, flush=True)
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
    cuda = device.type == "cuda"
    impl = a.engine if cuda else "python"
    eng_timeout = a.timeout + 30.0 if a.timeout > 0 else 600.0  # the watchdog fires first
    multi = world > 1 or a.force_dist

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    # ------------------------------------------------------------------ building blocks
    ctrl = TorchDistTransport(force_collectives=a.force_dist) if multi else ThreadFabric(1).transport(0)
    ctx = {"native": None, "native_err": None, "p2p": None, "p2p_err": None, "bus": None}

    def native_transport():
        if ctx["native"] is None and ctx["native_err"] is None:
            if not cuda:
                ctx["native_err"] = "no GPU"
            else:
                bus = ctx["bus"] = D.all_gather_object(topology.own_bus_id())
                if world > 1 and len(set(bus)) < len(bus):  # RCCL refuses two ranks on one device
                    ctx["native_err"] = f"ranks share a GPU (bus ids {bus}): RCCL refuses duplicate devices"
                else:
                    ctx["native"], ctx["native_err"] = try_native_transport(force_collectives=a.force_dist)
        return ctx["native"]

    def p2p_comm():
        if ctx["p2p"] is None and ctx["p2p_err"] is None:
            if not (cuda and world > 1):
                ctx["p2p_err"] = "needs world > 1 on GPU"
            else:
                ctx["p2p"], ctx["p2p_err"] = try_p2p_comm()
                if ctx["p2p"] is not None and os.environ.get("FAN_P2P_TIMING", "0") == "1":
                    ctx["p2p"].set_timing(True)
        return ctx["p2p"]

    def build(name, kind, algo="mesh", rings=1, transport="auto", gemm="persistent", sdma=False, fused=None,
              force=False, ring_sub=0, epi=None, engine=None, sizes=None, mdtype=None, bias=True,
              relu="hidden", shard=None, kflag=False):
        """Engine + model + trainer of one arm. kind: bfp | raw | rccl | local; transport: native | p2p | torch |
        auto (the world-1 / CPU default); engine: python | native (default: the run's)."""
        comm = None
        t = ctrl
        eimpl = engine or (impl if kind != "rccl" else "python")
        if transport == "native":
            t = native_transport()
            if t is None:
                raise RuntimeError(f"RCCL communicator unavailable: {ctx['native_err']}")
        elif transport == "p2p":
            comm = p2p_comm()
            if comm is None:
                raise RuntimeError(f"P2P transport unavailable: {ctx['p2p_err']}")
            comm.sdma = sdma
            comm.kernel_flags = kflag
        elif force and cuda and impl == "native":  # world-1 split: the multi-rank path over a 1-rank RCCL group
            t = NativeTransport(force_collectives=True)
        eng = make_engine(t, kind, rounding=a.rounding, algo=algo, rings=rings, force_comm=force or a.force_dist,
                          impl=eimpl, comm=comm, side_stream=a.side_stream and not multi, timeout_s=eng_timeout,
                          **({"ring_sub": ring_sub, "shard_update": shard} if eimpl == "native" else {}))
        if hasattr(eng, "epilogue_on_producer") and not getattr(eng, "inline", True):
            eng.epilogue_on_producer = (epi or a.epi) == "producer"
        pad_fn = (lambda n: eng.layout(n).n_pad) if eng is not None else None
        model = MLP(sizes or SIZES, dtype=mdtype or dtype, device=device, pad_fn=pad_fn, seed=1, bias=bias, relu=relu)
        if world > 1:
            for l in model.layers:
                ctrl.broadcast_(l.master, 0)
            model.sync_lp()
        tr = DataParallelTrainer(model, eng, lr=a.lr, gemm_inflight=gemm, fused_update=fused)
        info = {"compress": kind, "algo": algo, "rings": getattr(eng, "rings", 0) if eng is not None else 0,
                "transport": (getattr(t, "name", transport) if comm is None else "p2p") if multi or force else "none",
                "gemm_inflight": tr.gemm_inflight, "copy": ("sdma" if sdma else "kernel") if comm is not None else None,
                "flags": ("kernel" if kflag else "cp") if comm is not None else None,
                "ring_sub": int(getattr(eng, "ring_sub", 1)) if algo == "ring" else None,
                "epilogue_stream": ("compute" if getattr(eng, "epilogue_on_producer", False) else "comm")
                if eng is not None and not getattr(eng, "inline", True) else "inline",
                "shard_update": bool(getattr(tr, "shard", False))}
        return Setup(name, eng, model, tr, info)

    def release(setup):
        if setup is None:
            return
        try:
            setup.trainer.finish()
        except Exception as ex:  # noqa: BLE001 - an arm that failed in flight: its transport was aborted
            log(f"release of {setup.name}: {str(ex)[:200]}")
        setup.engine = setup.model = setup.trainer = None
        gc.collect()
        if cuda:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    def batch(mb, seed, model=None):
        g = torch.Generator().manual_seed(seed + rank)
        sizes = model.sizes if model is not None else SIZES
        x = (torch.rand(mb, sizes[0], generator=g) * 2 - 1).to(device=device,
                                                                dtype=model.dtype if model is not None else dtype)
        y = torch.randint(0, sizes[-1], (mb,), generator=g, dtype=torch.int32).to(device)
        return x, y

    stall_rank = int(os.environ.get("FAN_BENCH_STALL_RANK", "-1"))
    settle = {}  # the headline's untimed settle steps (extra.settle)

    def run(setup, mb, seed, warmup, steps, tag, graph_ok=False, trace=False, wait_s=None):
        """W warmup + K timed steps of ``setup`` at per-GPU batch mb: (elapsed s max over ranks, host enqueue s,
        loss, trace summary or None, graphed). The garbage collector is off inside (a collection pause in the
        launch loop starves the GPU: one 20-step MB-1792 window once read 0.46 instead of 0.38 ms/step)."""
        gc.collect()
        gc.disable()
        held["engine"] = setup.engine
        if setup.info.get("copy") is not None and ctx["p2p"] is not None:  # the arm's copy path (shared comm)
            ctx["p2p"].sdma = setup.info["copy"] == "sdma"
            ctx["p2p"].kernel_flags = setup.info.get("flags") == "kernel"
        try:
            return _run(setup, mb, seed, warmup, steps, tag, graph_ok, trace, wait_s)
        finally:
            gc.enable()

    def _finish(trainer, wait_s):
        """trainer.finish(); with a bound (A/B arms) the outcome is agreed over every rank first, so a rank whose
        request failed and a rank whose request completed (one rank's abort can release another's waits) raise at
        the same point instead of meeting at different collectives."""
        if wait_s is None:
            trainer.finish()
            return
        err = None
        try:
            trainer.finish(wait_s)
        except Exception as e:  # noqa: BLE001
            err = f"rank {rank}: {e}"
        err = next((x for x in D.all_gather_object(err) if x), None)
        if err:
            raise RuntimeError(err[:600])

    def _run(setup, mb, seed, warmup, steps, tag, graph_ok, trace, wait_s=None):
        trainer, model, engine = setup.trainer, setup.model, setup.engine
        x, y = batch(mb, seed, model)
        wd.arm(f"warmup {tag} mb={mb}")
        if tag in ("timed", "ref", "split") and cuda and a.settle_ms > 0:
            # The shader clock needs ~50 ms of sustained load to reach the level a training run holds: the driver's
            # 5 warmup + 20 steps read 1.038-1.047 ms/step where 50 + 20 read 0.989 and 5 + 100 0.996
            # (profiles/r4_warmup_settle.jsonl). Untimed steps of the same batch in chunks of 10 until settle_ms
            # passed (the chunk count agreed over ranks, so every rank runs the same steps); then W + K as ever.
            # Both timed cells (the headline and the reference batch, extra.mb<ref>) get it, so they are measured
            # alike (extra.settle per cell), and so do the world-1 split cells (unfused update, forced multi-rank
            # path): built after the headline, they start from an idle clock (forced_dist read 1.15-1.18 ms/step
            # without it, 1.06-1.07 standalone with it).
            t_s, n_s = time.perf_counter(), 0
            while n_s < 5000:
                for _ in range(10):
                    trainer.step(x, y)
                n_s += 10
                _finish(trainer, wait_s)
                torch.cuda.synchronize()
                if D.max_over_ranks(time.perf_counter() - t_s) * 1e3 >= a.settle_ms:
                    break
            settle[tag] = {"steps": n_s, "ms": round((time.perf_counter() - t_s) * 1e3, 1)}
        if stall_rank == rank and tag == "timed":  # test hook: this rank stops taking part (a hung peer)
            time.sleep(float(os.environ.get("FAN_BENCH_STALL_S", "600")))
        for _ in range(warmup):
            trainer.step(x, y)
        _finish(trainer, wait_s)  # wait_s: an A/B arm's bound (a hung transport raises instead of parking the rank)
        wd.arm(f"{tag} mb={mb}")
        step = lambda: trainer.step(x, y)  # noqa: E731
        graphed = False
        if graph_ok and a.graph and cuda and world == 1 and (engine is None or getattr(engine, "inline", False)):
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
        D.barrier()
        if cuda:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        loss_rows = model.loss_rows
        t_enqueue = time.perf_counter() - t0  # host time to issue K steps (GPU may still be running)
        if wait_s is None:
            _finish(trainer, wait_s)
            if cuda:
                torch.cuda.synchronize()
            D.barrier()
            elapsed = D.max_over_ranks(time.perf_counter() - t0)
        else:
            # an A/B arm: each rank's clock stops when its own work has drained; the ranks agree on the outcome
            # after that (the agreement is a control-plane all_gather_object, ~1 ms: inside the window it read
            # stage 2's 10-step rounds 10-13 % above the headline, profiles/r5_ab_stability.jsonl)
            err = None
            try:
                trainer.finish(wait_s)
            except Exception as ex:  # noqa: BLE001
                err = f"rank {rank}: {ex}"
            if cuda and err is None:
                torch.cuda.synchronize()
            t_local = time.perf_counter() - t0
            err = next((x for x in D.all_gather_object(err) if x), None)
            if err:
                raise RuntimeError(err[:600])
            elapsed = D.max_over_ranks(t_local)
        tr = None
        if trace:
            tr = engine.trace_summary()
            engine.trace(False)
            tr["comm_ms"] = D.max_over_ranks(tr["comm_ms"])  # the slowest rank's communication time
            tr["ms_per_step"] = elapsed / steps * 1e3
        return elapsed, t_enqueue, float(loss_rows.float().mean().item()), tr, graphed

    mb = a.mb_per_gpu
    gates_failed = []
    schedule_ab = None
    gate_rec = None
    # ------------------------------------------------------------------ the schedule (world > 1: A/B + gate)
    if world > 1 and a.schedule == "auto" and a.compress == "bfp":
        arms = []
        if cuda and impl == "native":
            R = world - 1  # as many link-disjoint rings as the planner finds (7 on a fully connected 8-GPU node)
            for gm in ("persistent", "grid"):
                arms.append(dict(name=f"rccl_mesh_{gm}", kind="bfp", algo="mesh", transport="native", gemm=gm))
                arms.append(dict(name=f"p2p_mesh_{gm}", kind="bfp", algo="mesh", transport="p2p", gemm=gm))
                arms.append(dict(name=f"p2p_ring_{gm}", kind="bfp", algo="ring", rings=R, transport="p2p", gemm=gm))
            # pure copies on the copy engines: ~2x slower than the copy kernels at 2 ranks (profiles/
            # r4_final_bench_2rank_1gpu.jsonl: 4.2 / 5.2 vs 2.6 ms/step), so only on request (FAN_AB_SDMA=1)
            if os.environ.get("FAN_AB_SDMA", "0") == "1":
                arms.append(dict(name="p2p_mesh_sdma", kind="bfp", algo="mesh", transport="p2p", sdma=True))
                arms.append(dict(name="p2p_ring_sdma", kind="bfp", algo="ring", rings=R, transport="p2p", sdma=True))
            # each ring hop streamed in 3 sub-slices (a ready flag each; engine.cpp run_ring_direct)
            arms.append(dict(name="p2p_ring_stream3", kind="bfp", algo="ring", rings=R, transport="p2p", ring_sub=3))
            # sharded update (ZeRO-1 style): each owner reduces + applies SGD to its shard, the ranks all-gather the new
            # bf16 weights into the layer's next weight buffer (no deferred epilogue, 1/N of the update pass per rank)
            arms.append(dict(name="rccl_mesh_shard", kind="bfp", algo="mesh", transport="native", shard=True))
            arms.append(dict(name="p2p_mesh_shard", kind="bfp", algo="mesh", transport="p2p", shard=True))
            # the flag writes / waits as kernels (system-scope release store, bounded in-kernel spin + acquire) instead
            # of command-processor packets: the CP-independent synchronisation path (p2p_comm.h, kernel flags)
            arms.append(dict(name="p2p_mesh_kflag", kind="bfp", algo="mesh", transport="p2p", kflag=True))
            arms.append(dict(name="p2p_mesh_shard_kflag", kind="bfp", algo="mesh", transport="p2p", shard=True,
                             kflag=True))
            # each request's decode + SGD epilogue on the comm stream as soon as its all-gather lands (overlapping the
            # rest of the backward) instead of on the compute stream after the last backward GEMM
            arms.append(dict(name="rccl_mesh_epicomm", kind="bfp", algo="mesh", transport="native", epi="comm"))
            arms.append(dict(name="p2p_mesh_epicomm", kind="bfp", algo="mesh", transport="p2p", epi="comm"))
            # last resort, never the fastest: the Python-issued engine over the control plane's own collectives
            # (torch.distributed), so a run whose native transports all fail their gate or hang still records a
            # gate-checked compressed step instead of no line at all
            arms.append(dict(name="torch_mesh_python", kind="bfp", algo="mesh", transport="torch", engine="python",
                             fallback=True))
        else:
            arms.append(dict(name=f"{impl}_{a.algo}", kind="bfp", algo=a.algo, rings=a.rings, transport="torch"))
        only = [x for x in os.environ.get("FAN_AB_ARMS", "").split(",") if x]
        if only:  # diagnostics: the A/B over the named arms only (in the listed order), the fallback kept
            arms = [next(x for x in arms if x["name"] == n) for n in only if any(x["name"] == n for x in arms)] + [
                x for x in arms if x.get("fallback")]
        schedule_ab = []
        arm_gates = {}
        kept = []  # (record, setup) of the fastest exact arms of stage 1, fastest first (at most --ab2-top)
        arm_wait = min(eng_timeout, a.arm_timeout)  # gate and A/B waits: below the watchdog's per-phase budget
        for spec in arms:
            if spec.get("fallback") and kept:  # identical on every rank (agreed results and times)
                schedule_ab.append({"arm": spec["name"], "skipped": "a faster exact arm passed"})
                continue
            wd.arm(f"schedule A/B {spec['name']}")
            rec = {"arm": spec["name"]}
            setup = None
            try:
                setup = build(spec["name"], spec["kind"], algo=spec.get("algo", "mesh"), rings=spec.get("rings", 1),
                              transport=spec["transport"], gemm=spec.get("gemm", "persistent"),
                              sdma=spec.get("sdma", False), kflag=spec.get("kflag", False),
                              ring_sub=spec.get("ring_sub", 1), epi=spec.get("epi"), engine=spec.get("engine"),
                              shard=spec.get("shard", False))
                rec.update(setup.info)
                t_arm = time.perf_counter()
                log(f"arm {spec['name']}: built, running the exactness gate")
                g = gate.allreduce_exactness(setup.engine, timeout_s=arm_wait)
                if g["exact"] and cuda and hasattr(setup.engine, "C"):
                    # the update half too (seeded master / momentum, one allreduce_sgd): the sharded arms' owner
                    # SGD + weight all-gather, the others' decode + SGD epilogue, bit for bit against the oracle
                    gu = gate.update_exactness(setup.engine, timeout_s=arm_wait)
                    g = dict(g, update_exact=gu["exact"], update_sharded=gu["sharded"],
                             exact=g["exact"] and gu["exact"],
                             mismatch_ranks=sorted(set(g["mismatch_ranks"]) | set(gu["mismatch_ranks"])))
                rec["exact"] = g["exact"]
                log(f"arm {spec['name']}: gate exact={g['exact']} ({time.perf_counter() - t_arm:.1f} s)")
                arm_gates[spec["name"]] = g
                if not g["exact"]:
                    gates_failed.append({"arm": spec["name"], **g})
                    rec["gate"] = g
                    raise RuntimeError(f"all-reduce exactness gate failed: {g}")
                e, _, _, _, _ = run(setup, mb, 99, 2, a.ab_steps, f"ab {spec['name']}", wait_s=arm_wait)
                rec["ms_per_step"] = round(e / a.ab_steps * 1e3, 4)
                log(f"arm {spec['name']}: {rec['ms_per_step']} ms/step ({time.perf_counter() - t_arm:.1f} s)")
            except Exception as ex:  # noqa: BLE001 - a failing arm is recorded and skipped, never fatal
                rec["error"] = str(ex)[:300]
                log(f"arm {spec['name']} excluded: {rec['error']}")
            schedule_ab.append(rec)
            # A transport whose request timed out was aborted by the engine (poisoned P2P flags / ncclCommAbort release
            # the parked streams). Every rank learns which transports ANY rank lost and drops them together, so the
            # later arms and extras stay symmetric: a hung link costs its arms, not the run (the watchdog would
            # otherwise end every rank at --timeout with no record).
            lost = [k for k in ("p2p", "native") if ctx[k] is not None and _transport_error(ctx[k])]
            lost_any = sorted({k for ks in D.all_gather_object(lost) for k in ks})
            for k in lost_any:
                if ctx[k] is not None and not _transport_error(ctx[k]):
                    try:
                        ctx[k].abort()
                    except Exception:  # noqa: BLE001
                        pass
                ctx[k] = None
                ctx[k + "_err"] = f"aborted after arm {spec['name']} failed: {rec.get('error', '?')[:160]}"
                rec.setdefault("transport_lost", []).append(k)
                log(f"transport {k} aborted and excluded after arm {spec['name']}")
            if lost_any and "ms_per_step" in rec:  # its numbers came from a transport that is gone
                rec["error"] = ctx[lost_any[0] + "_err"]
                del rec["ms_per_step"]
            for kr, ks in list(kept):  # a kept arm ran on a transport that is gone
                if kr.get("transport") in lost_any:
                    kr["error"] = ctx[kr["transport"] + "_err"]
                    kr.pop("ms_per_step", None)
                    release(ks)
                    kept.remove((kr, ks))
            if "ms_per_step" in rec:
                kept.append((rec, setup))
                kept.sort(key=lambda x: x[0]["ms_per_step"])
                while len(kept) > max(1, a.ab2_top):
                    release(kept.pop()[1])
            else:
                release(setup)
        if not kept:
            log("no arm of the schedule A/B passed: " + json.dumps(schedule_ab))
            return 3
        if len(kept) > 1 and a.ab2_steps > 0:
            # Stage 2: stage 1's 4 steps per arm (no settle) read ~15 % above the headline and its top arms swapped
            # places between runs. The kept arms get a warmup each, then 3 interleaved rounds of
            # --ab2-steps steps; the lowest median decides. An arm that fails here is dropped with its error.
            wd.arm("schedule A/B stage 2")
            st2 = {r["arm"]: [] for r, _ in kept}
            for rnd in range(4):  # round 0: warmup (untimed in the decision)
                for kr, ks in list(kept):
                    try:
                        e, _, _, _, _ = run(ks, mb, 99, 2 if rnd == 0 else 1, a.ab2_steps, f"ab2 {kr['arm']}",
                                            wait_s=arm_wait)
                        if rnd > 0:
                            st2[kr["arm"]].append(round(e / a.ab2_steps * 1e3, 4))
                    except Exception as ex:  # noqa: BLE001
                        kr["error"] = f"stage 2: {str(ex)[:280]}"
                        kr.pop("ms_per_step", None)
                        release(ks)
                        kept.remove((kr, ks))
            import statistics

            for kr, _ in kept:
                kr["stage2_ms_per_step"] = st2[kr["arm"]]
                kr["stage2_median"] = statistics.median(st2[kr["arm"]]) if st2[kr["arm"]] else None
            kept.sort(key=lambda x: x[0]["stage2_median"] if x[0]["stage2_median"] is not None else 1e30)
            if not kept:
                log("no arm survived stage 2 of the schedule A/B: " + json.dumps(schedule_ab))
                return 3
        chosen_rec, main_setup = kept[0]
        for _, ks in kept[1:]:
            release(ks)
        kept = kept[:1]
        chosen_rec["chosen"] = True
        gate_rec = dict(arm_gates[chosen_rec["arm"]], arm=chosen_rec["arm"])
        log(f"schedule A/B: running {chosen_rec['arm']} ({chosen_rec.get('stage2_median', chosen_rec['ms_per_step'])}"
            f" ms/step in the A/B)")
    else:
        transport = "auto"
        if world > 1 or a.force_dist:
            transport = {"native": "native" if impl == "native" else "torch", "p2p": "p2p", "torch": "torch"}[
                a.transport]
            if transport == "native" and native_transport() is None:
                log(f"native communicator unavailable ({ctx['native_err']}); using torch.distributed")
                transport = "torch"
        main_setup = build("main", a.compress, algo=a.algo, rings=a.rings, transport=transport,
                           gemm=a.gemm_inflight, force=a.force_dist and impl == "native" and transport == "auto",
                           sdma=a.p2p_copy == "sdma" and transport == "p2p",
                           kflag=a.p2p_flags == "kernel" and transport == "p2p",
                           shard=None if a.shard_update < 0 else bool(a.shard_update))
        if multi and main_setup.engine is not None:
            gate_rec = gate.allreduce_exactness(main_setup.engine)
            if not gate_rec["exact"]:
                gates_failed.append({"arm": "main", **gate_rec})
    engine, model, trainer = main_setup.engine, main_setup.model, main_setup.trainer
    if multi and engine is not None and gate_rec is not None and gate_rec.get("exact"):
        # the chosen schedule once more, on every bucket layout the model actually trains (each layer's size at this
        # world's arena slot: chunking and ring block geometry differ from the 1 Mi-element gate request)
        wd.arm("layout gate")
        try:
            lg = gate.allreduce_exactness_layouts(engine, [l.n for l in model.layers],
                                                  timeout_s=min(eng_timeout, a.arm_timeout))
        except Exception as ex:  # noqa: BLE001
            lg = {"exact": False, "error": str(ex)[:300], "layouts": []}
        gate_rec = dict(gate_rec, layouts=lg.get("layouts"), layouts_exact=lg["exact"],
                        n_checked=[gate_rec.get("n")] + [x["n"] for x in lg.get("layouts") or []])
        if not lg["exact"]:
            gates_failed.append({"arm": "main", "layouts": lg.get("layouts"), "max_abs_diff": lg.get("max_abs_diff"),
                                 "mismatch_ranks": lg.get("mismatch_ranks"), "error": lg.get("error")})
            gate_rec["exact"] = False
    held["engine"] = engine
    held["comm"] = ctx["p2p"] if main_setup.info.get("transport") == "p2p" else None
    held["transport"] = ctx["native"] or ctrl
    can_trace = (not a.no_trace and hasattr(engine, "trace") and not getattr(engine, "inline", True))

    # ------------------------------------------------------------------ reference batch, headline, traced pass
    elapsed, t_enqueue, loss, _, graphed = run(main_setup, mb, 1234, a.warmup, a.steps, "timed", graph_ok=True)
    ms = elapsed / a.steps * 1e3
    log(f"headline: {ms:.4f} ms/step over {a.steps} steps")
    ref = None
    if a.ref_mb and a.ref_mb != mb:
        # The reference-batch cell runs after the headline, with its own settle phase (both cells are measured alike);
        # a short step, so a longer window (a host hiccup is then a smaller share of it).
        ref_steps = max(a.steps, REF_STEPS) if cuda else a.steps
        e2, _, _, _, g2 = run(main_setup, a.ref_mb, 4321, a.warmup, ref_steps, "ref", graph_ok=True)
        ref = {"mb_per_gpu": a.ref_mb, "global_batch": a.ref_mb * world, "steps": ref_steps,
               "samples_per_s": round(a.ref_mb * world * ref_steps / e2, 2),
               "ms_per_step": round(e2 / ref_steps * 1e3, 4), "hip_graph": g2}
    tr = run(main_setup, mb, 1234, 1, a.steps, "traced", trace=True)[3] if can_trace else None

    def record(dist_rec, extras_s, aborted=None):
        """The JSON record (rank 0). ``aborted``: the watchdog's phase when it ends the run during the extras or the
        verification — the headline was measured by then, so the record is printed without what did not finish."""
        global_batch = mb * world
        value = global_batch * a.steps / elapsed
        flops = model.flops_per_sample() * global_batch * a.steps / elapsed
        info = main_setup.info
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
                "compress": info["compress"],
                "rounding": a.rounding,
                "algo": info["algo"],
                "rings": info["rings"],
                "transport": info["transport"],
                "engine": impl,
                "schedule": main_setup.name if schedule_ab is not None else "fixed",
                "gemm_inflight": info["gemm_inflight"],
                "p2p_copy": info["copy"],
                # release of the peer-storing kernels' stores before each ready flag: "cp" (command processor,
                # one-GPU default) or "block" (in-kernel, chosen by P2PComm.connect when a peer is on another GPU)
                "p2p_release": ({0: "none", 1: "block", 2: "thread", 3: "cp"}[_release_mode()]
                                if info["copy"] is not None else None),
                "p2p_cross_device": bool(ctx["p2p"].cross_device) if ctx["p2p"] is not None else None,
                "p2p_flags": info.get("flags"),
                "hip_graph": graphed,
                "fused_sgd": True,
                # world 1: dW's BFP round trip + SGD inside the bwd-weight GEMM epilogue (no separate update pass)
                "fused_update_in_gemm": bool(getattr(trainer, "fused_update", False)),
                "epilogue_stream": ("compute" if getattr(engine, "epilogue_on_producer", False) else "comm")
                if engine is not None and not getattr(engine, "inline", True) else "inline",
                "shard_update": info.get("shard_update", False),
            },
            "extra": {
                "achieved_tflops": round(flops / 1e12, 2),
                "host_enqueue_ms_per_step": round(t_enqueue / a.steps * 1e3, 4),
                "settle": settle or None,
                "grad_bytes_f32_per_step": sum(l.n for l in model.layers) * 4,
                "allreduce": _allreduce_report(tr, world),
                f"mb{a.ref_mb}": ref,
                "final_loss": round(loss, 5),
                "schedule_ab": schedule_ab,
                "gates_failed": [{"arm": g["arm"], "max_abs_diff": g.get("max_abs_diff"),
                                  "mismatch_ranks": g.get("mismatch_ranks")} for g in gates_failed],
                "dist": dist_rec,
                **dict(extras),
                "extras_s": round(extras_s, 2),
                "run_s": round(time.perf_counter() - t_begin, 2),
                "gemm_tuning": _tuning_report(),
                # (not after an abort: the engine may be held by the thread the watchdog is ending)
                **({"engine_counters": engine.counters()} if hasattr(engine, "counters") and not aborted else {}),
                # the direct P2P transport's flag waits over the whole run (device-timed with FAN_P2P_TIMING=1)
                **({"p2p_stats": dict(ctx["p2p"].stats())} if ctx["p2p"] is not None and not aborted else {}),
                **({"aborted_in": aborted} if aborted else {}),
            },
        }
        return rec

    # the watchdog prints the measured headline if an extra or the verification never returns
    held["record"] = lambda phase: record(None, time.perf_counter() - t_extra0, aborted=phase)
    # ------------------------------------------------------------------ extras (bounded)
    extras = {}

    def budget_left():
        return a.extra_budget - (time.perf_counter() - t_extra0)

    def extra(name, fn, need_s):
        """Run one extra if the budget has room (rank 0's clock decides for every rank)."""
        ok = D.all_gather_object(budget_left() >= need_s)[0]
        if not ok:
            extras[name] = {"skipped": f"extra budget ({a.extra_budget:.0f} s) spent"}
            return
        wd.arm(f"extra {name}")
        log(f"extra {name}")
        stall = os.environ.get("FAN_BENCH_STALL_EXTRA", "")  # test hook "<extra>:<rank>": that rank stops there
        if stall and stall.rsplit(":", 1)[0] == name and int(stall.rsplit(":", 1)[1]) == rank:
            time.sleep(600)
        try:
            extras[name] = fn()
        except Exception as ex:  # noqa: BLE001 - an extra never costs the headline its record
            extras[name] = {"error": str(ex)[:300]}
            log(f"extra {name} failed: {ex}")

    t_extra0 = time.perf_counter()
    if a.extra_budget > 0:
        if world == 1 and not a.force_dist and engine is not None:
            def split(fused, force, shard=None):
                s = build("split", a.compress, transport="auto", fused=fused, force=force, shard=shard)
                try:
                    e, _, _, _, _ = run(s, mb, 1234, 3, a.steps, "split")
                    return round(e / a.steps * 1e3, 4)
                finally:
                    release(s)

            def forced(shard=False):
                if not (torch.distributed.is_initialized()):
                    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                    os.environ["MASTER_PORT"] = str(_free_port())
                    D.init_distributed(force=True)
                return split(None, True, shard)

            extra("unfused_update_ms_per_step", lambda: split(False, False), 10)
            extra("forced_dist_ms_per_step", forced, 20)
            # the same multi-rank path with the sharded update (owner reduce + SGD fused, weight all-gather)
            extra("forced_dist_shard_ms_per_step", lambda: forced(True), 20)

            def config5_forced():
                if not torch.distributed.is_initialized():
                    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                    os.environ["MASTER_PORT"] = str(_free_port())
                    D.init_distributed(force=True)
                return _config5(a, world, device, main_setup.info, ctx, native_transport, p2p_comm, make_engine, ctrl,
                                eng_timeout, forced=NativeTransport(force_collectives=True))

            extra("config5", config5_forced, 30)

        def ref_workload():
            """The reference's own benchmark (sw/run.sh:16: mlp_mpi_example_f32 20 5376 0 A 32 32 32 2048 x 11 over 3
            ranks): 10 FC layers of 2048, f32, fuse_type 0 (no bias, no ReLU), 1792 rows per rank, BFP all-reduce +
            SGD of every layer's gradient over this run's transport; the reference's report quantities (fp time =
            s/iter, GFLOPS by its formula, sw/mlp_mpi_example_f32.cpp:794-808)."""
            if not cuda:
                return {"skipped": "CPU run"}
            info = main_setup.info
            tp = info.get("transport") if multi else "auto"
            tp = tp if tp in ("p2p", "native", "torch") else ("auto" if not multi else "torch")
            s = build("ref_workload", a.compress, algo=info.get("algo", "mesh"), rings=max(1, info.get("rings") or 1),
                      transport=tp, sizes=[2048] * 11, mdtype=torch.float32, bias=False, relu="none",
                      engine="python" if tp == "torch" else None)
            try:
                iters = 10
                e, _, loss_r, _, _ = run(s, REF_MB_PER_RANK, 777, 3, iters, "ref_workload")
                t_it = e / iters
                gmb = REF_MB_PER_RANK * world
                gflop = s.model.flops_per_sample() * gmb / 1e9
                return {"sizes": [2048] * 11, "dtype": "f32", "fuse_type": 0, "mb_per_rank": REF_MB_PER_RANK,
                        "global_mb": gmb, "iters": iters, "fp_time_s": round(t_it, 6), "GFLOP": round(gflop, 2),
                        "GFLOPS": round(gflop / t_it, 1), "samples_per_s": round(gmb / t_it, 1),
                        "final_loss": round(loss_r, 5), "transport": s.info["transport"], "algo": s.info["algo"],
                        "compress": s.info["compress"]}
            finally:
                release(s)

        extra("ref_workload", ref_workload, 15)
        if world > 1:
            extra("config4", lambda: _config4(a, world, rank, device, ctx, native_transport, p2p_comm, make_engine,
                                              ctrl, eng_timeout), 30)

            def uncompressed():
                out = {}
                if cuda:
                    native_transport()  # (collective) the ranks' bus ids, for the speedup's same-GPU guard
                arms_u = ((("p2p_raw_f32_mesh", "raw", "p2p"), ("rccl_f32", "rccl", "native")) if cuda and
                          impl == "native" else (("torch_f32", "rccl", "torch"),))  # CPU: gloo's all-reduce
                for name, kind, tp in arms_u:
                    s = None
                    comm = ctx.get("p2p") if tp == "p2p" else None
                    try:
                        s = build(name, kind, transport=tp)
                        if comm is not None:  # device-timed flag waits of this arm's timed steps
                            comm.reset_stats()
                            comm.set_timing(True)
                        e, _, _, _, _ = run(s, mb, 1234, 2, a.steps, f"uncompressed {name}")
                        out[name] = {"ms_per_step": round(e / a.steps * 1e3, 4), **s.info}
                        if comm is not None:
                            st = comm.stats()
                            out[name]["p2p_stall_ms_per_step"] = round(
                                (st["ready_stall_ms"] + st["credit_stall_ms"]) / max(1, a.steps + 2), 4)
                            out[name]["p2p_flag_waits"] = int(st["ready_waits"] + st["credit_waits"])
                    except Exception as ex:  # noqa: BLE001
                        out[name] = {"skipped": str(ex)[:300]}
                    finally:
                        if comm is not None:
                            comm.set_timing(False)
                        release(s)
                out["compressed_ms_per_step"] = round(ms, 4)
                out["speedup_vs_best_uncompressed"], out["speedup_note"] = _uncompressed_speedup(
                    out, ms, ctx.get("bus") or [None])
                return out

            extra("uncompressed", uncompressed, 15)
            extra("config5", lambda: _config5(a, world, device, main_setup.info, ctx, native_transport, p2p_comm,
                                              make_engine, ctrl, eng_timeout), 30)
    extras_s = time.perf_counter() - t_extra0

    # replicas after every step of the run: bit-identical weights on every rank (the reference reads its NIC
    # registers back to stdout after programming them, sw/mlp_mpi_example_f32.cpp:65-98; here the run proves
    # what it ran on and that the replicas agree)
    wd.arm("verify")
    dist_rec = _dist_report(main_setup, world, rank, device, D, gate_rec)
    wd.disarm()

    if rank == 0:
        print(json.dumps(record(dist_rec, extras_s)), flush=True)
    wd.arm("cleanup")
    D.cleanup()
    wd.close()
    if not dist_rec["replicas_identical"]:
        print(f"[bench] rank {rank}: replicas DIVERGED: {dist_rec['replica_digests']}", file=sys.stderr, flush=True)
        return 2
    if gates_failed:
        print(f"[bench] rank {rank}: all-reduce exactness gate FAILED: {json.dumps(gates_failed)}", file=sys.stderr,
              flush=True)
        # a failing A/B arm is excluded (and listed in extra.gates_failed); the run fails only when the schedule
        # that produced the headline did (a fixed schedule's own gate) — the scaling record of an exact arm stays
        if any(g["arm"] == "main" for g in gates_failed):
            return 3
    return 0


def _config5(a, world, device, info, ctx, native_transport, p2p_comm, make_engine, ctrl, timeout_s, forced=None):
    """BASELINE config 5: a BERT-base backward whose bwd-weight GEMMs encode each layer bucket's gradient for its BFP
    all-reduce + fused SGD, issued right after the layer (bench/bert_overlap.py measure(): compute only, comm only,
    both; 3 rounds, max over ranks), over the headline's transport and algorithm; at world 1 (``forced``: the 1-rank
    native transport) through the full multi-rank path with its side-stream engine."""
    if device.type != "cuda":
        return {"skipped": "CPU run"}
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
    import bert_overlap

    comm, t = None, ctrl
    if forced is not None:
        t = forced
    elif info.get("transport") == "p2p":
        comm = p2p_comm()
        comm.sdma = info.get("copy") == "sdma"
    else:
        t = native_transport()
        if t is None:  # the headline ran on the control plane's collectives (the last-resort arm): no native engine
            return {"skipped": f"no native transport: {ctx['native_err']}"}
    # the headline's update form (the sharded update at world 1: the owner reduce + SGD is the whole exchange)
    shard = True if forced is not None else bool(info.get("shard_update"))
    eng = make_engine(t, "bfp", rounding=a.rounding, algo=info.get("algo", "mesh"), rings=max(1, info.get("rings", 1)),
                      impl="native", comm=comm, timeout_s=timeout_s, force_comm=forced is not None,
                      shard_update=shard if info.get("algo", "mesh") == "mesh" else None)
    r = bert_overlap.measure(eng, device, world, tokens=4096, layers=12, rounds=3)
    r.update(transport="p2p" if comm is not None else getattr(t, "name", "torch"), algo=info.get("algo", "mesh"),
             forced_1rank=forced is not None, shard_update=bool(getattr(eng, "shard_update", False)))
    return r


def _config4(a, world, rank, device, ctx, native_transport, p2p_comm, make_engine, ctrl, timeout_s):
    """BASELINE config 4 (and the config-2 uncompressed baseline): a 256 MB f32 gradient, all-reduce + fused SGD
    per request, over the transports this run has. BFP variants start from the producer's encoding (prepacked, as
    in training); ``rccl_f32`` is RCCL's ncclAllReduce + a separate SGD kernel (the reference's commented
    MPI_Iallreduce + host SGD path, sw/mlp_mpi_example_f32.cpp:615-647). Per variant: median per-request time over
    the slowest rank, algo-BW = logical bytes / time, bus-BW = algo x 2(N-1)/N."""
    import statistics

    import torch

    from fpga_ai_nic_amd import _ext
    from fpga_ai_nic_amd.utils import dist as D

    if device.type != "cuda":
        return {"skipped": "CPU run"}
    n = CONFIG4_MB * (1 << 20) // 4
    variants = []
    p2p = p2p_comm()
    nat = native_transport()
    if p2p is not None:
        variants += [("bfp_mesh_p2p", "bfp", "mesh", 1, None, p2p), ("bfp_ring_p2p", "bfp", "ring", world - 1, None, p2p),
                     ("raw_f32_mesh_p2p", "raw", "mesh", 1, None, p2p)]
    if nat is not None:
        variants += [("bfp_mesh_rccl", "bfp", "mesh", 1, nat, None), ("rccl_f32", "rccl", "mesh", 1, nat, None)]
    out = {"size_MB_f32": CONFIG4_MB, "n_gpus": world}
    if p2p is None:
        out["p2p"] = {"skipped": ctx["p2p_err"]}
    if nat is None:
        out["rccl_f32"] = {"skipped": ctx["native_err"]}
    for name, kind, algo, rings, t, comm in variants:
        eng = None
        try:
            if comm is not None:
                comm.sdma = False
            eng = make_engine(t if t is not None else ctrl, kind, rounding=a.rounding, algo=algo, rings=rings,
                              impl="python" if kind == "rccl" else "native", comm=comm, timeout_s=timeout_s)
            L = eng.layout(n)
            g = torch.randn(L.n_pad, device=device) * 1e-3
            w = torch.randn(L.n_pad, device=device)
            lp = w.to(torch.bfloat16)
            kw = {}
            if kind == "bfp" and getattr(eng, "prepack", False):
                tgt = eng.prepack_target(g, n)
                if tgt is not None:
                    _ext.require().wire_pack_range(g, tgt[0], tgt[1], 0, n, tgt[3])
                    kw["prepacked"] = (tgt[0], L.n_pad)

            def once():
                return eng.allreduce_sgd(g, w, lp, n_valid=n, lr=1e-6, grad_scale=1.0 / world, **kw)

            for _ in range(2):
                once().synchronize(timeout_s)
            times = []
            for _ in range(3):
                D.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                hs = [once() for _ in range(3)]
                for h in hs:
                    h.synchronize(timeout_s)
                torch.cuda.synchronize()
                times.append(D.max_over_ranks(time.perf_counter() - t0) / 3)
            t = statistics.median(times)
            algo_bw = n * 4 / t / 1e9
            out[name] = {"us": round(t * 1e6, 1), "algo_bw_GBps": round(algo_bw, 2),
                         "bus_bw_GBps": round(algo_bw * 2 * (world - 1) / world, 2),
                         "wire_bytes_per_rank": int(eng.wire_bytes(L)), "rings": int(getattr(eng, "rings", 1)),
                         "input": "prepacked" if kw else "f32"}
            if hasattr(eng, "trace"):  # one traced request: phase split (mesh) / per-hop split (ring), this rank
                eng.trace(True)
                once().synchronize(timeout_s)
                tr = eng.trace_summary()
                eng.trace(False)
                out[name]["comm_us"] = round(tr["comm_ms"] * 1e3, 1)
                if tr.get("hop_rounds"):
                    k = tr["hop_rounds"]
                    out[name]["ring_hops"] = {
                        "rounds": k, "credit_us": round(tr["hop_credit_ms"] * 1e3 / k, 2),
                        "ready_us": round(tr["hop_ready_ms"] * 1e3 / k, 2),
                        "kernel_us": round(tr["hop_kernel_ms"] * 1e3 / k, 2),
                        "max_round_us": round(tr["hop_max_ms"] * 1e3, 2)}
                else:
                    out[name]["phase_us"] = {p[:-3]: round(tr[p] * 1e3, 1) for p in
                                             ("pack_ms", "exchange_ms", "reduce_ms", "gather_ms", "epilogue_ms")}
        except Exception as ex:  # noqa: BLE001
            out[name] = {"error": str(ex)[:300]}
        finally:
            del eng
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    return out


def _tuning_report():
    """The GEMM plans the on-device tuner chose on this rank (shape key, static plan, chosen plan, their times)."""
    from fpga_ai_nic_amd.ops import gemm_tune

    t = gemm_tune.tuner()
    return {"enabled": t.enabled, "decisions": t.log}


def replica_digest(tensors):
    """Per tensor: (exact bit hash, fp64 sum). The hash is integer arithmetic on the f32 / bf16 bit patterns (position-
    weighted, wrapping mod 2^64), so it is order-independent and equal across ranks iff the bits are."""
    import torch

    out = []
    for t in tensors:
        bits = torch.int32 if t.element_size() == 4 else torch.int16
        b = t.detach().reshape(-1).contiguous().view(bits).to(torch.int64)
        w = torch.arange(b.numel(), device=b.device, dtype=torch.int64).mul_(2).add_(1)
        h = int((b * w).sum().item()) & 0xFFFFFFFFFFFFFFFF
        out.append([f"{h:016x}", float(t.detach().double().sum().item())])
    return out


def _uncompressed_speedup(out, ms, bus_ids):
    """(speedup of the compressed step over the fastest uncompressed arm, note). Withheld (None) when it would not
    measure the codec: ranks time-sharing one GPU (their flag waits cross processes through the command processor's
    hardware queues, which 3+ processes oversubscribe: docs/ROUND6.md), or an arm whose own device-timed P2P flag
    waits are more than half of its step."""
    done = {k: v for k, v in out.items() if isinstance(v, dict) and "ms_per_step" in v}
    if not done:
        return None, "no uncompressed arm ran"
    shared = len(bus_ids) > 1 and None not in bus_ids and len(set(bus_ids)) < len(bus_ids)
    stalled = [k for k, v in done.items() if v.get("p2p_stall_ms_per_step", 0.0) > 0.5 * v["ms_per_step"]]
    raw = round(min(v["ms_per_step"] for v in done.values()) / ms, 4)
    if shared:
        return None, f"ranks share a GPU ({len(bus_ids)} processes on {len(set(bus_ids))} devices): " \
                     f"same-GPU rehearsal ratio {raw} not a codec speedup"
    if stalled:
        return None, f"arm(s) {stalled} dominated by their own P2P flag-wait stalls (ratio {raw} withheld)"
    return raw, "fastest uncompressed arm / compressed step"


def _dist_report(setup, world, rank, device, D, gate_rec):
    """extra.dist: what the run actually ran on — torch's and the engine communicator's rank counts (RCCL:
    ncclCommCount), the transport, the ring orders and link matrix the planner used, the devices (PCI bus ids) of
    the ranks — whether the production all-reduce path passed the bit-exact gate, and whether the replicas' weights
    are bit-identical after the run (all-gathered digests). Sharded-update arms: every rank's master is the
    concatenation of the owners' shards after ``gather_state()``, identical by construction, so the check there is on
    the bf16 weights each rank actually trains with (``lp``, written by the weight all-gather), hashed BEFORE the
    gather, plus each rank's own check that its ``lp`` equals bf16(gathered master)."""
    import torch

    from fpga_ai_nic_amd.utils import topology

    engine, model = setup.engine, setup.model
    C = getattr(engine, "C", None)
    shard = bool(getattr(setup.trainer, "shard", False))
    lp_digest, lp_match = None, None
    if shard:  # owner-sharded master / momentum: gather them before comparing
        setup.trainer.finish()
        lp_digest = replica_digest([l.lp for l in model.layers if l.lp is not None])
        setup.trainer.gather_state()
        lp_match = all(torch.equal(l.lp[:l.n], l.master[:l.n].to(torch.bfloat16))
                       for l in model.layers if l.lp is not None)
    mine = {
        "digest": replica_digest([l.master for l in model.layers]) + (lp_digest or []),
        "lp_matches_master": lp_match,
        "comm_ranks": int(C.comm_ranks) if C is not None else (world if engine is not None else 1),
        "bus_id": topology.device_bus_id(device.index) if device.type == "cuda" else None,
    }
    every = D.all_gather_object(mine)
    digests = [e["digest"] for e in every]
    ident = all(d == digests[0] for d in digests) and all(e["lp_matches_master"] is not False for e in every)
    return {
        "world": world,
        "torch_backend": D.backend(),
        "transport": setup.info["transport"],
        "engine_comm": (C.comm_kind if C is not None else ("python" if engine is not None else "none")),
        "comm_ranks": [e["comm_ranks"] for e in every],
        "algo": getattr(engine, "algo", None),
        "ring_orders": getattr(engine, "orders", None) if getattr(engine, "algo", None) == "ring" else None,
        "links": getattr(engine, "links", None),
        "bus_ids": [e["bus_id"] for e in every],
        "allreduce_exact": gate_rec["exact"] if gate_rec is not None else None,
        "allreduce_gate": gate_rec,
        "replicas_identical": ident,
        "master_gathered_from_owners": shard,
        "lp_matches_master": [e["lp_matches_master"] for e in every] if shard else None,
        "replica_digests": digests if not ident else digests[0],
    }


def _allreduce_report(tr, world):
    """All-reduce algo-BW of the requests of the traced pass (the same K steps again, with per-request device
    timestamps): logical (f32 gradient) bytes / summed device time of their communication phases (request start on
    the comm stream -> end of the all-gather, slowest rank); bus-BW = algo-BW x 2(N-1)/N; wire-BW = bytes this rank
    actually sent (BFP-packed) / the same time. Ring schedules add the per-hop split (credit wait, hop kernels,
    upstream ready wait, longest round). None when no collective ran (world 1 inline engine: no wire)."""
    if not tr or not tr.get("requests") or tr.get("comm_ms", 0) <= 0:
        return None
    s = tr["comm_ms"] / 1e3
    algo = tr["logical_bytes"] / s / 1e9
    rec = {
        "traced_ms_per_step": round(tr["ms_per_step"], 4),
        "requests": tr["requests"],
        "comm_ms_total": round(tr["comm_ms"], 4),
        "allreduce_algo_bw_GBps": round(algo, 2),
        "bus_bw_GBps": round(algo * 2 * (world - 1) / world, 2) if world > 1 else 0.0,
        "wire_bw_GBps": round(tr["wire_bytes"] / s / 1e9, 2),
        "phase_ms": {k: round(tr[k], 4) for k in ("pack_ms", "exchange_ms", "reduce_ms", "gather_ms", "epilogue_ms")},
        "dropped": tr.get("dropped", 0),
    }
    if tr.get("hop_rounds"):
        n = tr["hop_rounds"]
        rec["ring_hops"] = {"rounds": n, "credit_ms": round(tr["hop_credit_ms"], 4),
                            "kernel_ms": round(tr["hop_kernel_ms"], 4), "ready_ms": round(tr["hop_ready_ms"], 4),
                            "mean_round_us": round((tr["hop_credit_ms"] + tr["hop_kernel_ms"] + tr["hop_ready_ms"])
                                                   / n * 1e3, 2),
                            "max_round_us": round(tr["hop_max_ms"] * 1e3, 2)}
    return rec


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""All-reduce bandwidth sweep (BASELINE config 4: 256 MB synthetic gradient, BFP all-reduce + fused SGD).

For each message size and variant it times ``allreduce_sgd`` — compressed all-reduce + fused SGD, the reference
NIC's whole request (hw/all_reduce.sv + hw/weight_update.sv; sw/mlp_mpi_example_f32.cpp:114-180) — on the
production path: the C++ engine (csrc/comm/engine.cpp) over its own RCCL communicator (``--transport native``,
default), torch.distributed's RCCL (``torch``) or the direct HIP-IPC peer transport (``p2p``). At world 1 the
requests run through the full multi-rank path by default (a 1-rank RCCL group: every collective is on the timed
path; ``--local`` times the inline world-1 engine instead, which has no collectives).

Reported per (variant, size):
* ``us`` / ``algo_bw_GBps`` = logical f32 gradient bytes / wall time per request (all-reduce + SGD), and
  ``bus_bw_GBps`` = algo x 2(N-1)/N;
* ``comm_us`` / ``comm_algo_bw_GBps``: device time of the communication phase only (request start on the comm
  stream -> end of the all-gather, from the engine's request trace, slowest rank), and the phase split;
* ``wire_bytes_per_rank``: bytes one rank sends (BFP: 17 B per 16 values).
Both variants start from f32 gradients (the mesh packs its shards, the ring packs per hop), or with
``--prepacked`` both from the producer's BFP encoding (as in training, where the bwd-weight GEMM encodes), so mesh
vs ring is a like-for-like comparison; ``rccl`` is the uncompressed baseline (RCCL f32 all-reduce + a separate SGD kernel,
BASELINE config 2; the reference's commented MPI_Iallreduce path, sw:615-647).

1 GPU:  python bench/allreduce_bw.py
N GPUs: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench/allreduce_bw.py
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpga_ai_nic_amd.parallel.dp import make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import (NativeTransport, ThreadFabric, TorchDistTransport,  # noqa: E402
                                                make_p2p_comm)
from fpga_ai_nic_amd.utils import dist as D  # noqa: E402
from fpga_ai_nic_amd.utils.metrics import allreduce_bw  # noqa: E402

VARIANTS = {
    "bfp_mesh": dict(kind="bfp", algo="mesh", rings=1),
    "bfp_ring": dict(kind="bfp", algo="ring", rings=1),
    "bfp_ring7": dict(kind="bfp", algo="ring", rings=7),
    "raw_mesh": dict(kind="raw", algo="mesh", rings=1),
    "rccl": dict(kind="rccl", algo="mesh", rings=1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,64,256")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--engine", default="native", choices=["native", "python"])
    ap.add_argument("--transport", default="native", choices=["native", "torch", "p2p"])
    ap.add_argument("--local", action="store_true", help="world 1: inline engine (no collectives)")
    ap.add_argument("--grad-dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--prepacked", action="store_true",
                    help="the gradient arrives already BFP-encoded by its producer (the training path: the bwd-weight "
                         "GEMM's wire epilogue; encoded once here, outside the timed requests): the mesh skips its "
                         "pack pass, the ring sends the producer's slices at every SEND_LOCAL hop")
    a = ap.parse_args()
    force = not a.local
    rank, world, _, dev = D.init_distributed(force=force)
    multi = world > 1 or force
    gdt = torch.float32 if a.grad_dtype == "f32" else torch.bfloat16
    p2p = make_p2p_comm() if (a.transport == "p2p" and a.engine == "native" and multi) else None
    for vname in a.variants.split(","):
        v = VARIANTS[vname]
        impl = a.engine if v["kind"] != "rccl" else "python"
        if not multi:
            transport = ThreadFabric(1).transport(0)
        elif v["kind"] == "rccl" or impl == "python" or a.transport in ("torch", "p2p"):  # p2p: gloo/RCCL control
            transport = TorchDistTransport(force_collectives=force)
        else:
            transport = NativeTransport(force_collectives=force)
        eng = make_engine(transport, v["kind"], algo=v["algo"], rings=v["rings"], impl=impl, force_comm=force,
                          comm=p2p if impl == "native" else None)
        can_trace = hasattr(eng, "trace") and not getattr(eng, "inline", True)
        for mb in (int(x) for x in a.sizes_mb.split(",")):
            n = mb * (1 << 20) // 4
            L = eng.layout(n)
            g = torch.randn(L.n_pad, device=dev).to(gdt) * 1e-3
            w = torch.randn(L.n_pad, device=dev)
            lp = w.to(torch.bfloat16)

            kw = {}
            if a.prepacked and hasattr(eng, "prepack_target") and gdt == torch.float32:
                tgt = eng.prepack_target(g, n)
                if tgt is not None:  # the "producer": encode the whole gradient once into the engine's wire layout
                    n16 = n // 16 * 16
                    from fpga_ai_nic_amd import _ext

                    _ext.require().wire_pack_range(g, tgt[0], tgt[1], 0, n16, tgt[3])
                    kw["prepacked"] = (tgt[0], n16)

            def once():
                return eng.allreduce_sgd(g, w, lp, n_valid=n, lr=1e-6, grad_scale=1.0 / world, **kw)

            once().synchronize()
            times, comm = [], []
            for _ in range(a.rounds):
                D.barrier()
                torch.cuda.synchronize()
                if can_trace:
                    eng.trace(True)
                t0 = time.perf_counter()
                hs = [once() for _ in range(a.iters)]
                for h in hs:
                    h.synchronize()
                torch.cuda.synchronize()
                times.append(D.max_over_ranks(time.perf_counter() - t0) / a.iters)
                if can_trace:
                    tr = eng.trace_summary()
                    eng.trace(False)
                    tr["comm_ms"] = D.max_over_ranks(tr["comm_ms"])
                    comm.append(tr)
            t = statistics.median(times)
            algo_bw, bus_bw = allreduce_bw(n * 4, t, world)
            rec = {"bench": "allreduce_sgd_bw", "variant": vname, "engine": impl,
                   "transport": (a.transport if impl == "native" else "torch") if multi else "none",
                   "n_gpus": world, "size_MB_f32": mb, "rings": eng.rings, "rings_requested": v["rings"],
                   "us": round(t * 1e6, 1), "algo_bw_GBps": round(algo_bw, 1), "bus_bw_GBps": round(bus_bw, 1),
                   "wire_bytes_per_rank": eng.wire_bytes(L), "grad_dtype": a.grad_dtype,
                   "input": "prepacked" if kw else "f32",
                   # the torch.distributed backend: with FAN_CTRL_BACKEND=gloo the "rccl" variant is a gloo all-reduce
                   "torch_backend": dist.get_backend() if dist.is_initialized() else None,
                   "direct_rounds": eng.counters().get("direct_rounds", 0) if hasattr(eng, "counters") else 0}
            if comm:
                tr = sorted(comm, key=lambda x: x["comm_ms"])[len(comm) // 2]  # median round
                cus = tr["comm_ms"] * 1e3 / max(1, tr["requests"])
                calgo, cbus = allreduce_bw(n * 4, cus / 1e6, world)
                rec.update({"comm_us": round(cus, 1), "comm_algo_bw_GBps": round(calgo, 1),
                            "comm_bus_bw_GBps": round(cbus, 1),
                            "phase_us": {k[:-3]: round(tr[k] * 1e3 / max(1, tr["requests"]), 1)
                                         for k in ("pack_ms", "exchange_ms", "reduce_ms", "gather_ms", "epilogue_ms")}})
            if rank == 0:
                print(json.dumps(rec), flush=True)
    D.cleanup()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""All-reduce bandwidth sweep (BASELINE config 4: 256 MB synthetic gradient, BFP ring all-reduce).

For each message size and engine variant it times ``allreduce_sgd`` (compressed all-reduce + fused SGD, the
reference NIC's whole request) and reports algo-BW = logical fp32 gradient bytes / time and bus-BW =
algo * 2(N-1)/N, next to the uncompressed RCCL baseline (dist.all_reduce f32 + SGD kernel).

1 GPU:  python bench/allreduce_bw.py          (codec / epilogue kernel throughput only: no wire)
N GPUs: torchrun --nproc-per-node N --master-addr 127.0.0.1 bench/allreduce_bw.py
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
from fpga_ai_nic_amd.parallel.dp import make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import NativeTransport, ThreadFabric, TorchDistTransport  # noqa: E402
from fpga_ai_nic_amd.utils import dist as D  # noqa: E402
from fpga_ai_nic_amd.utils.metrics import allreduce_bw  # noqa: E402

VARIANTS = {
    "bfp_mesh": dict(kind="bfp", algo="mesh", rings=1),
    "bfp_ring": dict(kind="bfp", algo="ring", rings=1),
    "bfp_ring_multi": dict(kind="bfp", algo="ring", rings=7),
    "raw_mesh": dict(kind="raw", algo="mesh", rings=1),
    "rccl": dict(kind="rccl", algo="mesh", rings=1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,64,256")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--transport", default="torch", choices=["torch", "native"])
    ap.add_argument("--grad-dtype", default="f32", choices=["f32", "bf16"])
    a = ap.parse_args()
    rank, world, _, dev = D.init_distributed()
    if world > 1:
        transport = NativeTransport() if a.transport == "native" else TorchDistTransport()
    else:
        transport = ThreadFabric(1).transport(0)
    gdt = torch.float32 if a.grad_dtype == "f32" else torch.bfloat16
    for vname in a.variants.split(","):
        v = VARIANTS[vname]
        eng = make_engine(transport, v["kind"], algo=v["algo"], rings=v["rings"])
        for mb in (int(x) for x in a.sizes_mb.split(",")):
            n = mb * (1 << 20) // 4
            L = eng.layout(n)
            g = torch.randn(L.n_pad, device=dev).to(gdt) * 1e-3
            w = torch.randn(L.n_pad, device=dev)
            lp = w.to(torch.bfloat16)

            def once():
                return eng.allreduce_sgd(g, w, lp, n_valid=n, lr=1e-6, grad_scale=1.0 / world)

            once().synchronize()
            times = []
            for _ in range(a.rounds):
                D.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                hs = [once() for _ in range(a.iters)]
                for h in hs:
                    h.synchronize()
                torch.cuda.synchronize()
                times.append(D.max_over_ranks(time.perf_counter() - t0) / a.iters)
            t = statistics.median(times)
            algo_bw, bus_bw = allreduce_bw(n * 4, t, world)
            if rank == 0:
                print(json.dumps({"bench": "allreduce_sgd_bw", "variant": vname, "n_gpus": world,
                                  "size_MB_f32": mb, "rings": eng.rings, "us": round(t * 1e6, 1),
                                  "algo_bw_GBps": round(algo_bw, 1), "bus_bw_GBps": round(bus_bw, 1),
                                  "wire_bytes_per_rank": eng.wire_bytes(L), "grad_dtype": a.grad_dtype}),
                      flush=True)
    D.cleanup()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Multi-rank probe of the RCCL data path on whatever GPUs exist (ranks may share one GPU).

Run: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dist_probe.py [--transport torch|native]
Checks the engine (mesh / ring / multi-ring, BFP) against the spec simulator and the DP trainer's replica
consistency over the real torch.distributed "nccl" (RCCL) backend. Prints one PASS/FAIL line per check.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpga_ai_nic_amd.models.mlp import MLP  # noqa: E402
from fpga_ai_nic_amd.parallel import sim  # noqa: E402
from fpga_ai_nic_amd.parallel.allreduce import CompressedAllReduce  # noqa: E402
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import NativeTransport, TorchDistTransport  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transport", default="torch")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % ndev)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    t = NativeTransport() if a.transport == "native" else TorchDistTransport()
    ok_all = True
    n = 100_000
    rng = np.random.default_rng(11)
    grads = [rng.standard_normal(n).astype(np.float32) for _ in range(world)]
    for algo, rings in (("mesh", 1), ("ring", 1), ("ring", 3)):
        eng = CompressedAllReduce(t, codec="bfp_rne", algo=algo, rings=rings, max_slice_elems=8192)
        L = eng.layout(n)
        g = torch.zeros(L.n_pad, device=dev)
        g[:n] = torch.from_numpy(grads[rank]).to(dev)
        out = torch.zeros(L.n_pad, device=dev)
        t0 = time.time()
        eng.allreduce(g, out, n_valid=n).synchronize(timeout=60)
        gin = [np.pad(x, (0, L.n_pad - n)) for x in grads]
        exp = sim.mesh_allreduce(gin, L.shard) if algo == "mesh" else \
            sim.ring_allreduce(gin, eng.orders, L.slice_elems, L.blocks)[0]
        ok = bool(np.array_equal(out.cpu().numpy()[:n], exp[:n]))
        ok_all &= ok
        print(f"[rank {rank}] {'PASS' if ok else 'FAIL'} engine algo={algo} rings={eng.rings} "
              f"transport={t.name} ({time.time() - t0:.2f}s)", flush=True)
    # DP trainer replicas stay identical
    eng = make_engine(t, "bfp")
    sizes = [256, 512, 512, 256]
    model = MLP(sizes, dtype=torch.bfloat16, device=dev, pad_fn=lambda k: eng.layout(k).n_pad, seed=1)
    for l in model.layers:
        t.broadcast_(l.master, 0)
    model.sync_lp()
    tr = DataParallelTrainer(model, eng, lr=0.05)
    gx = torch.Generator().manual_seed(rank)
    x = torch.randn(256, sizes[0], generator=gx).to(dev, torch.bfloat16)
    y = torch.randint(0, sizes[-1], (256,), generator=gx, dtype=torch.int32).to(dev)
    for _ in range(3):
        tr.step(x, y)
    tr.finish()
    w = torch.cat([l.master for l in model.layers])
    ws = [torch.empty_like(w) for _ in range(world)]
    dist.all_gather(ws, w)
    ok = all(torch.equal(ws[0], z) for z in ws)
    ok_all &= ok
    print(f"[rank {rank}] {'PASS' if ok else 'FAIL'} dp replicas identical after 3 steps", flush=True)
    dist.barrier(device_ids=[dev.index])
    dist.destroy_process_group()
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()

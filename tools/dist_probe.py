#!/usr/bin/env python3
"""Multi-rank probe of the RCCL data path on whatever GPUs exist (ranks may share one GPU).

Run: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dist_probe.py [--transport torch|native|p2p]
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
from fpga_ai_nic_amd.parallel.transport import NativeTransport, P2PTransport, TorchDistTransport  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transport", default="torch")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % ndev)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    # p2p: the Python engine's byte transport AND the C++ engine's communicator are the direct HIP-IPC peer transport
    t = {"native": NativeTransport, "torch": TorchDistTransport, "p2p": P2PTransport}[a.transport]()
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
    # the C++ engine over its own RCCL communicator: mesh / ring / multi-ring, both BFP codecs, vs the simulators
    from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce
    from fpga_ai_nic_amd.ops import bfp_oracle as O

    nt = t if isinstance(t, NativeTransport) else NativeTransport()
    comm = t.comm if isinstance(t, P2PTransport) else None  # C++ engine over the P2P communicator
    w0 = rng.standard_normal(n).astype(np.float32)
    for codec in ("bfp_rne", "bfp_trunc"):
        for algo, rings in (("mesh", 1), ("ring", 1), ("ring", min(7, max(1, world - 1)))):
            eng = NativeAllReduce(nt, codec=codec, algo=algo, rings=rings, max_slice_elems=8192, comm=comm)
            L = eng.layout(n)
            g = torch.zeros(L.n_pad, device=dev)
            g[:n] = torch.from_numpy(grads[rank]).to(dev)
            out = torch.zeros(L.n_pad, device=dev)
            w = torch.zeros(L.n_pad, device=dev)
            w[:n] = torch.from_numpy(w0).to(dev)
            t0 = time.time()
            eng.allreduce(g, out, n_valid=n).synchronize(60)
            h = eng.allreduce_sgd(g, w, None, n_valid=n, lr=0.5, defer=True)
            h.commit_after_current()
            h.synchronize(60)
            torch.cuda.synchronize()
            gin = [np.pad(x, (0, L.n_pad - n)) for x in grads]
            exp = sim.mesh_allreduce(gin, L.shard, codec) if algo == "mesh" else \
                sim.ring_allreduce(gin, eng.orders, L.slice_elems, L.blocks, codec)[0]
            ok = bool(np.array_equal(out.cpu().numpy()[:n], exp[:n]))
            ref_w, _ = O.sgd(w0, exp[:n], 0.5)
            got_w = w.cpu().numpy()[:n]
            ulp = np.abs(got_w.view(np.int32).astype(np.int64) - ref_w.view(np.int32).astype(np.int64)).max()
            ws = [torch.empty_like(w) for _ in range(world)]
            dist.all_gather(ws, w)
            same = all(torch.equal(ws[0], z) for z in ws)
            ok = ok and ulp <= 1 and same
            ok_all &= ok
            print(f"[rank {rank}] {'PASS' if ok else 'FAIL'} native engine codec={codec} algo={algo} rings={eng.rings} "
                  f"sum-bitexact + sgd<=1ulp ({ulp}) + replicas-identical={same} ({time.time() - t0:.2f}s)", flush=True)
    # uncompressed f32 wire over the C++ ring == RCCL's own all-reduce within fp32 reassociation
    eng = NativeAllReduce(nt, codec="raw_f32", algo="ring", rings=1, max_slice_elems=8192, comm=comm)
    L = eng.layout(n)
    g = torch.zeros(L.n_pad, device=dev)
    g[:n] = torch.from_numpy(grads[rank]).to(dev)
    out = torch.zeros(L.n_pad, device=dev)
    eng.allreduce(g, out, n_valid=n).synchronize(60)
    ref = g.clone()
    dist.all_reduce(ref)
    torch.cuda.synchronize()
    err = (out - ref).abs().max().item()
    ok = err <= 1e-5 * world
    ok_all &= ok
    print(f"[rank {rank}] {'PASS' if ok else 'FAIL'} raw f32 ring vs RCCL all_reduce max|diff|={err:.2e}", flush=True)
    # DP trainer replicas stay identical (C++ engine; bwd-weight GEMM encodes straight into the wire)
    eng = make_engine(nt, "bfp", impl="native", comm=comm)
    sizes = [256, 512, 512, 256]
    model = MLP(sizes, dtype=torch.bfloat16, device=dev, pad_fn=lambda k: eng.layout(k).n_pad, seed=1)
    for l in model.layers:
        t.broadcast_(l.master, 0)
    model.sync_lp()
    tr = DataParallelTrainer(model, eng, lr=0.05, momentum=0.9)
    gx = torch.Generator().manual_seed(rank)
    x = torch.randn(256, sizes[0], generator=gx).to(dev, torch.bfloat16)
    y = torch.randint(0, sizes[-1], (256,), generator=gx, dtype=torch.int32).to(dev)
    for _ in range(3):
        tr.step(x, y)
    tr.finish()
    w = torch.cat([l.master for l in model.layers])
    ws = [torch.empty_like(w) for _ in range(world)]
    dist.all_gather(ws, w)
    ok = all(torch.equal(ws[0], z) for z in ws) and tr.prepack
    ok_all &= ok
    print(f"[rank {rank}] {'PASS' if ok else 'FAIL'} native dp replicas identical after 3 steps (prepack={tr.prepack})",
          flush=True)
    # DP trainer replicas stay identical (Python engine)
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
